#!/usr/bin/env python3
"""Host-side enqueue cost of one configs[1] step (measurement tooling, GPU box): the time the host spends in one
nmz_replayable_sweep_decimal_topk_dev call while the GPU is still busy with earlier calls (so no call waits for the
device), with and without the library's timing events and torch's stream context, beside an empty ABI call.

usage: python tools/host_enqueue.py [calls=60]
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
from namazu_amd.synth import splitmix64  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    L = _lib.load()
    ctx = _lib.Context(0)
    dev = torch.device("cuda", 0)
    E, S = 4096, 1 << 20
    hints = [str(int(x)) for x in splitmix64(0x5EED, E).view(np.int64)]
    ho, hb = to_csr(hints)
    plans = []
    for _ in range(3):
        p = ctypes.c_void_p()
        _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), E, 100_000_000, S,
                                                ctypes.byref(p)))
        plans.append(p)
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    stats = [torch.empty(S * 32, dtype=torch.uint8, device=dev) for _ in range(3)]
    lists = torch.empty(n * 64 * 24, dtype=torch.uint8, device=dev)

    def call(i, use_ctx):
        sp = i % 3
        if use_ctx:
            with torch.cuda.stream(streams[sp]):
                _lib.check(L.nmz_replayable_sweep_decimal_topk_dev(
                    plans[sp], i * S, S, 64, ctypes.c_void_p(stats[sp].data_ptr()),
                    ctypes.c_void_p(lists.data_ptr() + i * 64 * 24), ctypes.c_void_p(streams[sp].cuda_stream)))
        else:
            _lib.check(L.nmz_replayable_sweep_decimal_topk_dev(
                plans[sp], i * S, S, 64, ctypes.c_void_p(stats[sp].data_ptr()),
                ctypes.c_void_p(lists.data_ptr() + i * 64 * 24), ctypes.c_void_p(streams[sp].cuda_stream)))

    for i in range(6):
        call(i, False)
    torch.cuda.synchronize()
    res = {}
    for name, use_ctx, timing in (("plain", False, 0), ("stream_ctx", True, 0), ("timing_events", False, 1),
                                  ("stream_ctx+timing", True, 1), ("plain_again", False, 0)):
        _lib.check(L.nmz_timing_enable(ctx.handle, timing))
        torch.cuda.synchronize()
        per = []
        t_all = time.perf_counter()
        for i in range(n):
            t = time.perf_counter()
            call(i, use_ctx)
            per.append(time.perf_counter() - t)
        host = time.perf_counter() - t_all
        torch.cuda.synchronize()
        gpu = time.perf_counter() - t_all
        per = np.array(per[3:]) * 1e6
        res[name] = per
        print(f"{name:20s} host per call: median {np.median(per):6.1f} us  p10 {np.percentile(per, 10):6.1f}  "
              f"p90 {np.percentile(per, 90):6.1f}   all {n} calls enqueued in {host * 1e3:.2f} ms, done after "
              f"{gpu * 1e3:.2f} ms ({gpu * 1e3 / n:.1f} us per step)")
    _lib.check(L.nmz_timing_enable(ctx.handle, 0))
    t = time.perf_counter()
    for _ in range(1000):
        L.nmz_abi_version()
    print(f"empty ABI call: {(time.perf_counter() - t) * 1e3:.2f} us")
    t = time.perf_counter()
    for _ in range(1000):
        ctypes.c_void_p(stats[0].data_ptr())
    print(f"c_void_p(tensor.data_ptr()): {(time.perf_counter() - t) * 1e3:.2f} us")
    for p in plans:
        L.nmz_replayable_plan_destroy(p)
    ctx.close()


if __name__ == "__main__":
    main()
