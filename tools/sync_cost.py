#!/usr/bin/env python3
"""Host cost of an idle torch.cuda.synchronize() (hipDeviceSynchronize) as HIP streams accumulate in the process
(measurement tooling, GPU box): before any torch stream exists, after library contexts open, after torch's stream
pool is created (torch.cuda.Stream()), and of torch.cuda.stream() context switches.

usage: python tools/sync_cost.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from namazu_amd import _lib  # noqa: E402


def cost(fn, n=200):
    for _ in range(10):
        fn()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t) / n * 1e6


def main():
    torch.cuda.init()
    torch.empty(1, device="cuda")
    torch.cuda.synchronize()
    print(f"idle synchronize, fresh process: {cost(torch.cuda.synchronize):.1f} us")
    ctxs = [_lib.Context(0) for _ in range(3)]
    print(f"idle synchronize, + 3 library contexts: {cost(torch.cuda.synchronize):.1f} us")
    ext = torch.cuda.ExternalStream(ctxs[0].stream())
    torch.cuda.set_stream(ext)
    print(f"idle synchronize, current stream = a context's stream: {cost(torch.cuda.synchronize):.1f} us")
    s = torch.cuda.Stream()
    print(f"idle synchronize, + torch stream pool: {cost(torch.cuda.synchronize):.1f} us")

    def ctx_switch():
        with torch.cuda.stream(s):
            pass
    print(f"torch.cuda.stream() enter + exit: {cost(ctx_switch):.1f} us")
    ev = torch.cuda.Event()
    ev.record(s)
    print(f"event record: {cost(lambda: ev.record(s)):.1f} us; query: {cost(ev.query):.1f} us")
    print(f"stream.synchronize (idle): {cost(s.synchronize):.1f} us")
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
