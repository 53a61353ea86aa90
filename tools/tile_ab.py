#!/usr/bin/env python3
"""k_ed_tile workload for A/B timing (measurement tooling, not the product).

All-pairs k-NN over 4,096 traces of ~300 events drawn from a 3,000-symbol alphabet (a query pair's symbols overflow
the bit-parallel compact tables, so the plan takes k_ed_tile) at bands 8, 16 and 32, three runs each, printing a
checksum of the k-NN lists so two builds can be compared (the parity tests cover correctness). Run it under `rocprofv3 --kernel-trace --stats` and read k_ed_tile<W>'s average duration; with
NMZ_LIB_PATH pointing at another build the same workload times that build.

usage (GPU box, repo root): python tools/tile_ab.py
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from namazu_amd import _lib  # noqa: E402
from namazu_amd import historystorage as hs  # noqa: E402


def traces(n, length, alphabet, mut, seed):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, alphabet, length)
    out = []
    for i in range(n):
        t = base[:length - (i % 5)].copy()
        m = rng.random(len(t)) < mut
        t[m] = rng.integers(0, alphabet, int(m.sum()))
        out.append(t.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(1000))
    return hs.TraceSet(out)


def main():
    ctx = _lib.Context(0)
    ts = traces(4096, 300, 3000, 0.04, 2)
    for w in (8, 16, 32):
        ms = []
        for rep in range(3):
            t0 = time.perf_counter()
            ids, ds = hs.allpairs_knn(ts, 4, w, ctx=ctx)
            ms.append((time.perf_counter() - t0) * 1e3)
        print(f"band {w}: all-pairs k-NN {np.median(ms):.2f} ms (plan + kernel), checksum "
              f"{int(ds.astype(np.uint64).sum())}:{int(ids.astype(np.uint64).sum())}", flush=True)


if __name__ == "__main__":
    main()
