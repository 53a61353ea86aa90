"""K1 (order-query sweep) kernel time against the number of seeds per launch (GPU box).

One workgroup per table row takes that row's seeds 64 per wave, 16 waves per round, so a row with more than
4,096 seeds needs a fifth round. This prints, per seed count, the largest row's seed count, the rounds it
needs and the kernel's execution span, to show how much of a launch is that partial last round.
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from namazu_amd import _lib  # noqa: E402
from namazu_amd.explorepolicy import to_csr  # noqa: E402
from namazu_amd.synth import splitmix64  # noqa: E402

FNV_OFF, FNV_PRIME = np.uint64(0xCBF29CE484222325), np.uint64(0x100000001B3)


def row_counts(lo, n):
    """Seeds per table row (low byte of FNV-1a 64 over the decimal seed string)."""
    s = np.arange(lo, lo + n)
    strs = s.astype(str)
    lens = np.char.str_len(strs)
    low = np.zeros(n, np.uint64)
    for ln in np.unique(lens):
        sel = lens == ln
        b = np.frombuffer("".join(strs[sel]).encode(), np.uint8).reshape(-1, ln)
        h = np.full(b.shape[0], FNV_OFF, np.uint64)
        with np.errstate(over="ignore"):
            for k in range(ln):
                h = (h ^ b[:, k].astype(np.uint64)) * FNV_PRIME
        low[sel] = h
    return np.bincount((low & np.uint64(0xFF)).astype(np.int64), minlength=256)


def main():
    L = _lib.load()
    ctx = _lib.Context(0)
    dev = torch.device("cuda", 0)
    E = 4096
    hints = [str(int(x)) for x in splitmix64(0x5EED, E).view(np.int64)]
    ho, hb = to_csr(hints)
    smax = int(1.125 * (1 << 20))
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), E, 100_000_000, smax,
                                            ctypes.byref(plan)))
    stream = torch.cuda.current_stream(dev)
    d_stats = torch.empty(smax * 32, dtype=torch.uint8, device=dev)
    d_topk = torch.empty(64 * 24, dtype=torch.uint8, device=dev)
    tot, cnt = ctypes.c_double(), ctypes.c_uint64()
    for frac in (0.875, 0.9375, 0.96875, 1.0, 1.015625, 1.03125, 1.0625, 1.125):
        S = int(frac * (1 << 20))
        so, sb = to_csr([str(i) for i in range(S)])
        d_so = torch.from_numpy(so.view(np.int32)).to(dev)
        d_sb = torch.from_numpy(sb).to(dev)
        rc = row_counts(0, S)

        def run():
            _lib.check(L.nmz_replayable_sweep_topk_dev(plan, ctypes.c_void_p(d_so.data_ptr()),
                                                       ctypes.c_void_p(d_sb.data_ptr()), S, 0, 64,
                                                       ctypes.c_void_p(d_stats.data_ptr()),
                                                       ctypes.c_void_p(d_topk.data_ptr()),
                                                       ctypes.c_void_p(stream.cuda_stream)))
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        _lib.check(L.nmz_timing_enable(ctx.handle, 1))
        L.nmz_timing_read_span(ctx.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1)
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        _lib.check(L.nmz_timing_read_span(ctx.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1))
        _lib.check(L.nmz_timing_enable(ctx.handle, 0))
        span = tot.value / max(cnt.value, 1)
        chunks = (rc + 63) // 64
        print(f"S={S:8d} mean/row={S / 256:7.1f} max/row={rc.max():5d} min/row={rc.min():5d} "
              f"rounds(max)={int(((chunks + 15) // 16).max())} rows>4096={int((rc > 4096).sum()):3d} "
              f"span={span:.4f} ms  ns/seed={1e6 * span / S:.4f}", flush=True)
    L.nmz_replayable_plan_destroy(plan)
    ctx.close()


if __name__ == "__main__":
    main()
