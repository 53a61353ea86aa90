"""K2 timing probe: the bench's configs[3] share (2^20 seeds x 10^4 events) through the library at NMZ_LIB_PATH.

Prints the kernel's average duration (HIP events on the launch stream) and a checksum of the stats, so that
two library builds can be compared for speed and for identical results.
usage: NMZ_LIB_PATH=... python3 tools/k2_probe.py [seeds] [reps]
"""
import ctypes
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from namazu_amd import _lib  # noqa: E402
from bench import splitmix64  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    E = 10_000
    L = _lib.load()
    ctx = _lib.Context(0)
    ent = np.arange(E) % 16
    evhash = splitmix64(0x5EED1, E)
    evclass = np.where(ent < 4, _lib.NMZ_EV_PRIORITIZED, 0).astype(np.uint8) | np.uint8(_lib.NMZ_EV_FAULTABLE)
    params = _lib.resolve_random_params(30_000_000, 100_000_000, 0.1)
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_random_plan_create(ctx.handle, evhash.ctypes.data, evclass.ctypes.data, E,
                                        ctypes.byref(params), S, ctypes.byref(plan)))
    d_stats = torch.empty(S * 32, dtype=torch.uint8, device="cuda:0")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(L.nmz_random_sweep_dev(plan, 0, S, ctypes.c_void_p(d_stats.data_ptr()), stream))
    torch.cuda.synchronize()
    _lib.check(L.nmz_timing_enable(ctx.handle, 1))
    tot, cnt = ctypes.c_double(), ctypes.c_uint64()
    L.nmz_timing_read(ctx.handle, b"random_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1)
    for _ in range(reps):
        _lib.check(L.nmz_random_sweep_dev(plan, 0, S, ctypes.c_void_p(d_stats.data_ptr()), stream))
    torch.cuda.synchronize()
    _lib.check(L.nmz_timing_read(ctx.handle, b"random_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1))
    L.nmz_random_plan_destroy(plan)
    ms = tot.value / max(cnt.value, 1)
    digest = hashlib.sha1(d_stats.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"k_random_sweep {ms:.3f} ms  {S * E / ms * 1e3:.4g} decisions/s  stats sha1 {digest}", flush=True)


if __name__ == "__main__":
    main()
