#!/usr/bin/env python3
"""Phase timing of the replayable plan kernel k_replayable_wt_build (measurement tooling, not the product).

Needs the timing-only library variant built with `make -C namazu_amd/csrc VARIANT=wttrace EXTRA=-DWT_BUILD_TRACE`
(every workgroup's thread 0 stamps wall_clock64() at the phase boundaries). Builds the configs[1] plan (4,096
ZooKeeper-style hints, maxInterval 100 ms) a few times and prints, per segment size, the median time of each
phase in microseconds (wall_clock64 runs at 100 MHz on gfx950), plus the kernel's first-start-to-last-end span.

usage (GPU box, repo root): NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_wttrace.so python tools/wt_build_trace.py
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from namazu_amd import _lib  # noqa: E402
from namazu_amd.explorepolicy import to_csr  # noqa: E402

PHASES = ["entries (fused: FNV + C sort) + row sum", "keys", "Cm sort", "rank arrays", "bucket indexes", "(empty: the per-d maxima, removed in round 5)", "levels",
          "block masks"]  # between the kernel's stamps 0..8
NP = 10
TICK_US = 0.01  # wall_clock64 at 100 MHz


def zk_hints(n, seed=0x5EED):
    # the bench's trace (bench.py zk_hints)
    from namazu_amd.synth import splitmix64 as sm
    return [str(int(x)) for x in sm(seed, n).view(np.int64)]


def main():
    L = _lib.load()
    L.nmz_debug_wt_build_trace.restype = ctypes.c_int
    L.nmz_debug_wt_build_trace.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    ctx = _lib.Context(0)
    ho, hb = to_csr(zk_hints(4096))
    lens = np.diff(ho.astype(np.int64))
    sizes = np.unique(lens, return_counts=True)[1].tolist()  # classes in ascending hint length (plan order)
    per = {}
    for rep in range(5):
        plan = ctypes.c_void_p()
        _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), 4096, 100_000_000, 1 << 20,
                                                ctypes.byref(plan)))
        buf = np.zeros(8192 * NP, np.uint64)
        assert L.nmz_debug_wt_build_trace(buf.ctypes.data, buf.size) == 0
        L.nmz_replayable_plan_destroy(plan)
        if rep == 0:
            continue  # first build: module load
        n_cls = len(sizes)
        t = buf.reshape(-1, NP)[:256 * n_cls].astype(np.int64)
        span = (t[:, 8].max() - t[:, 0].min()) * TICK_US
        per.setdefault("span", []).append(span)
        for c in range(n_cls):
            rows = t[np.arange(256) * n_cls + c]  # blockIdx.y = row L, blockIdx.x = segment
            ok = rows[:, 8] > 0
            if not ok.any():
                continue
            d = np.diff(rows[ok][:, :9], axis=1) * TICK_US
            per.setdefault(sizes[c], []).append(np.median(d, axis=0))
    print(f"kernel span (first start .. last end): {np.median(per.pop('span')):.1f} us")
    print("segment n | " + " | ".join(PHASES))
    for n, v in per.items():
        m = np.median(np.array(v), axis=0)
        print(f"{n:9d} | " + " | ".join(f"{x:6.2f}" for x in m))


if __name__ == "__main__":
    main()
