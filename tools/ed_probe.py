#!/usr/bin/env python3
"""Time the all-pairs banded-ED k-NN kernels on synthetic configs[2]-style traces.

usage: python tools/ed_probe.py N L W [k] [reps]
"""
import ctypes
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    N, L, W = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    k = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    import torch
    from namazu_amd import _lib
    from namazu_amd.synth import clustered_traces, etcd_traces, synth_traces
    t0 = time.time()
    gen = sys.argv[6] if len(sys.argv) > 6 else ""
    ts = etcd_traces(N, L) if gen == "etcd" else (clustered_traces(N, L, family=1024) if gen == "clustered"
                                                  else synth_traces(N, L))
    print(f"synth {time.time() - t0:.1f}s", flush=True)
    Lb = _lib.load()
    ctx = _lib.Context(0)
    plan = ctypes.c_void_p()
    t0 = time.time()
    _lib.check(Lb.nmz_ed_plan_create(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), N, W, ctypes.byref(plan)))
    print(f"plan {time.time() - t0:.2f}s kind={Lb.nmz_ed_plan_is_fast(plan)} (2=bit-parallel, 1=tile, 0=generic)", flush=True)
    d_knn = torch.empty(N * k, dtype=torch.int64, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(Lb.nmz_timing_enable(ctx.handle, 1))
    tot, cnt = ctypes.c_double(), ctypes.c_uint64()
    for r in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _lib.check(Lb.nmz_ed_allpairs_knn_dev(plan, k, ctypes.c_void_p(d_knn.data_ptr()), stream))
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        pairs = N * (N - 1) / 2
        print(f"rep {r}: {el * 1e3:.2f} ms  {pairs / el:.3e} pairs/s  "
              f"{pairs * (L * (2 * W + 1) - W * (W + 1)) / el:.3e} band-cells/s", flush=True)
    kname = {3: b"ed_wide", 2: b"ed_bv", 1: b"ed_tile"}.get(Lb.nmz_ed_plan_is_fast(plan), b"none")
    _lib.check(Lb.nmz_timing_read(ctx.handle, kname, ctypes.byref(tot), ctypes.byref(cnt), 1))
    print(f"kernel avg {tot.value / max(cnt.value, 1):.3f} ms over {cnt.value}")
    keys = d_knn.cpu().numpy().view(np.uint64).reshape(N, k)
    d = (keys >> np.uint64(32)).astype(np.int64)
    print("knn first-col dist: min", d[:, 0].min(), "median", int(np.median(d[:, 0])), "max", d[:, 0].max())
    Lb.nmz_ed_plan_destroy(plan)
    ctx.close()


if __name__ == "__main__":
    main()
