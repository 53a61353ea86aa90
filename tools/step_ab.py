#!/usr/bin/env python3
"""Steady-state cost of the parts of one configs[1] step (measurement tooling, GPU box): 200 steps pipelined over 3
streams as bench.py runs them, per variant:
  full      decimal seeds generated, hashed and bucketed on the device + K1 + top-64 (the headline's step)
  no_topk   the same without the top-64 (k = 0: K1 writes the stats only)
  seedset   K1 + top-64 over one prepared seed set (hashes bucketed once, outside the timing)
  seedset0  K1 alone over the prepared set (k = 0)
The differences price the bucketing kernels and the top-k kernels in the pipeline (their effect on K1 included).

usage: python tools/step_ab.py [steps=200] [reps=3]   (NMZ_STEP_NP: pipeline streams, NMZ_STEP_KINDS: variants)
"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from namazu_amd import _lib  # noqa: E402
from namazu_amd.explorepolicy import to_csr  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    L = _lib.load()
    dev = torch.device("cuda", 0)
    # NMZ_STEP_ORDER: "ctx_first" (context, then the streams), "streams_first" (streams created before the context's
    # own stream), "use_ctx" (the context's stream is pipeline stream 0), "three_ctx" (below): which HIP streams share
    # a hardware queue
    order = os.environ.get("NMZ_STEP_ORDER", "ctx_first")
    pre_streams = [torch.cuda.Stream(dev) for _ in range(int(os.environ.get("NMZ_STEP_NP", "3")))] \
        if order == "streams_first" else None
    ctx = _lib.Context(0)
    # "three_ctx": one context per pipeline slot, each slot on its context's own stream (plans on their contexts)
    ctxs = [ctx] + [_lib.Context(0) for _ in range(int(os.environ.get("NMZ_STEP_NP", "3")) - 1)] \
        if order == "three_ctx" else [ctx] * int(os.environ.get("NMZ_STEP_NP", "3"))
    E, S = 4096, 1 << 20
    NP = int(os.environ.get("NMZ_STEP_NP", "3"))
    ho, hb = to_csr(bench.zk_hints(E))
    plans = []
    for j in range(NP):
        p = ctypes.c_void_p()
        _lib.check(L.nmz_replayable_plan_create(ctxs[j].handle, _lib.ptr(ho), _lib.ptr(hb), E, bench.MAX_INTERVAL_NS,
                                                S, ctypes.byref(p)))
        plans.append(p)
    so, sb = bench.decimal_csr(0, S)
    d_so = torch.from_numpy(so.view(np.int32)).to(dev)
    d_sb = torch.from_numpy(sb).to(dev)
    ss = ctypes.c_void_p()
    _lib.check(L.nmz_replayable_seeds_create(ctx.handle, ctypes.c_void_p(d_so.data_ptr()),
                                             ctypes.c_void_p(d_sb.data_ptr()), S, 0, ctypes.byref(ss)))
    streams = pre_streams or [torch.cuda.Stream(dev) for _ in range(NP)]
    stats = [torch.empty(S * 32, dtype=torch.uint8, device=dev) for _ in range(NP)]
    lists = torch.empty(steps * 64 * 24, dtype=torch.uint8, device=dev)

    def call(kind, i):
        sp = i % NP
        st = ctypes.c_void_p(None if (order == "use_ctx" and sp == 0) or order == "three_ctx"
                             else streams[sp].cuda_stream)
        out = ctypes.c_void_p(lists.data_ptr() + i * 64 * 24)
        k = 0 if kind in ("no_topk", "seedset0") else 64
        if kind in ("full", "no_topk"):
            _lib.check(L.nmz_replayable_sweep_decimal_topk_dev(plans[sp], i * S, S, k,
                                                               ctypes.c_void_p(stats[sp].data_ptr()), out, st))
        else:
            _lib.check(L.nmz_replayable_sweep_seeds_topk_dev(plans[sp], ss, 0, k,
                                                             ctypes.c_void_p(stats[sp].data_ptr()), out, st))

    kinds = tuple(os.environ.get("NMZ_STEP_KINDS", "full,no_topk,seedset,seedset0").split(","))
    for kind in kinds:
        for i in range(6):
            call(kind, i)
    torch.cuda.synchronize()
    res = {k: [] for k in kinds}
    for _ in range(reps):
        for kind in kinds:
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i in range(steps):
                call(kind, i)
            torch.cuda.synchronize()
            res[kind].append((time.perf_counter() - t) / steps * 1e6)
    for kind in kinds:
        v = res[kind]
        print(f"{kind:9s} us per step: min {min(v):6.2f}  median {sorted(v)[len(v) // 2]:6.2f}  all "
              + " ".join(f"{x:.2f}" for x in v))
    L.nmz_replayable_seeds_destroy(ss)
    for p in plans:
        L.nmz_replayable_plan_destroy(p)
    for c in ctxs[1:] if order == "three_ctx" else []:
        c.close()
    ctx.close()


if __name__ == "__main__":
    main()
