"""Per-wave timeline of one K1 launch, from a -DOQ_TRACE build (order-query kernel) or a -DWT_TRACE build
(wavelet-tree kernel, --wt) (GPU box).

  NMZ_LIB_PATH=.../libnmz_gpu_trace.so python tools/k1_trace.py [--wt]

Stamps (wall_clock64, 100 MHz) per (row, wave): kernel start, row image staged, end of each 64-seed chunk.
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


def main():
    L = _lib.load()
    ctx = _lib.Context(0)
    dev = torch.device("cuda", 0)
    E, S = 4096, 1 << 20
    hints = [str(int(x)) for x in splitmix64(0x5EED, E).view(np.int64)]
    ho, hb = to_csr(hints)
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), E, 100_000_000, S,
                                            ctypes.byref(plan)))
    stream = torch.cuda.current_stream(dev)
    so, sb = to_csr([str(i) for i in range(S)])
    d_so = torch.from_numpy(so.view(np.int32)).to(dev)
    d_sb = torch.from_numpy(sb).to(dev)
    d_stats = torch.empty(S * 32, dtype=torch.uint8, device=dev)
    d_topk = torch.empty(64 * 24, dtype=torch.uint8, device=dev)
    for _ in range(5):
        _lib.check(L.nmz_replayable_sweep_topk_dev(plan, ctypes.c_void_p(d_so.data_ptr()),
                                                   ctypes.c_void_p(d_sb.data_ptr()), S, 0, 64,
                                                   ctypes.c_void_p(d_stats.data_ptr()),
                                                   ctypes.c_void_p(d_topk.data_ptr()),
                                                   ctypes.c_void_p(stream.cuda_stream)))
    torch.cuda.synchronize()
    report(L)
    tot, cnt = ctypes.c_double(), ctypes.c_uint64()
    for it in range(3):
        if it == 2:  # the last launch with the library's timing on (events + in-kernel span), as bench.py runs it
            _lib.check(L.nmz_timing_enable(ctx.handle, 1))
            L.nmz_timing_read_span(ctx.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1)
            L.nmz_timing_read(ctx.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1)
        _lib.check(L.nmz_replayable_sweep_topk_dev(plan, ctypes.c_void_p(d_so.data_ptr()),
                                                   ctypes.c_void_p(d_sb.data_ptr()), S, 0, 64,
                                                   ctypes.c_void_p(d_stats.data_ptr()),
                                                   ctypes.c_void_p(d_topk.data_ptr()),
                                                   ctypes.c_void_p(stream.cuda_stream)))
        torch.cuda.synchronize()
        print("--- again" + (" (timing on)" if it == 2 else ""))
        report(L)
        if it == 2:
            _lib.check(L.nmz_timing_read_span(ctx.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1))
            print(f"library span: {1e3 * tot.value / max(cnt.value, 1):.1f} us over {cnt.value} launches")
            _lib.check(L.nmz_timing_read(ctx.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1))
            print(f"library events: {1e3 * tot.value / max(cnt.value, 1):.1f} us over {cnt.value} launches")
    L.nmz_replayable_plan_destroy(plan)
    ctx.close()


WT = "--wt" in sys.argv


def report(L):
    tr = np.zeros((256, 16, 10), np.uint64)
    fn = L.nmz_debug_wt_trace if WT else L.nmz_debug_oq_trace
    fn.argtypes = [ctypes.c_void_p]
    assert fn(tr.ctypes.data) == 0
    tr = tr.astype(np.int64)

    t0 = tr[:, :, 9].min()
    start = (tr[:, :, 9] - t0) / 100.0  # us
    staged = (tr[:, :, 0] - t0) / 100.0
    ce = 9 if WT else 8  # chunk-end slots 1..ce-1 (the WT trace has no cooperative-tail slot)
    ends = np.where(tr[:, :, 1:ce] > 0, (tr[:, :, 1:ce] - t0) / 100.0, np.nan)
    tail_end = np.full(tr.shape[:2], np.nan) if WT else np.where(tr[:, :, 8] > 0, (tr[:, :, 8] - t0) / 100.0, np.nan)
    last = np.fmax(np.nanmax(ends, axis=2), tail_end)
    nchunks = np.sum(tr[:, :, 1:ce] > 0, axis=2)
    if np.any(~np.isnan(tail_end)):
        rows_t = ~np.all(np.isnan(tail_end), axis=1)
        tail_dur = np.nanmax(tail_end, axis=1) - np.nanmax(np.nanmax(ends, axis=2), axis=1)
        print(f"cooperative tail: {int(rows_t.sum())} rows, duration (last chunk end -> tail end) median "
              f"{np.nanmedian(tail_dur[rows_t]):.1f} max {np.nanmax(tail_dur[rows_t]):.1f} us")
    print(f"kernel span (first start -> last wave end): {np.nanmax(last):.1f} us")
    print(f"workgroup start: min {start.min():.1f} median {np.median(start):.1f} max {start.max():.1f} us")
    print(f"staging done:    min {staged.min():.1f} median {np.median(staged):.1f} max {staged.max():.1f} us; "
          f"staging time median {np.median(staged - start):.1f} us")
    dur = np.diff(np.concatenate([staged[:, :, None], ends], axis=2), axis=2)
    for k in range(dur.shape[2]):
        d = dur[:, :, k]
        if np.all(np.isnan(d)):
            break
        n = np.sum(~np.isnan(d))
        print(f"chunk {k}: waves {n:5d}  duration median {np.nanmedian(d):6.1f}  p10 {np.nanpercentile(d, 10):6.1f}  "
              f"p90 {np.nanpercentile(d, 90):6.1f} us")
    print(f"wave end: median {np.nanmedian(last):.1f}  p90 {np.nanpercentile(last, 90):.1f}  max {np.nanmax(last):.1f} us")
    print("chunks per wave histogram:", np.bincount(nchunks.ravel()).tolist())
    # per XCD (workgroups are dealt to the 8 XCDs round-robin) and per row
    rowdur = np.nanmedian(dur[:, :, :4], axis=1)  # [row][chunk] median over waves
    for x in range(8):
        rows = np.arange(x, 256, 8)
        print(f"  xcd {x}: chunk medians " + " ".join(f"{np.nanmedian(rowdur[rows, k]):5.1f}" for k in range(4))
              + f"  row end max {np.nanmax(last[rows]):.1f}")
    slow = np.argsort(-rowdur[:, 0])[:8]
    print("  slowest rows in chunk 0:", [(int(r), round(float(rowdur[r, 0]), 1)) for r in slow])
    # rows finishing last
    rl = np.nanmax(last, axis=1)
    order = np.argsort(-rl)[:5]
    for r in order:
        print(f"  row {r}: ends {rl[r]:.1f} us, start {start[r].min():.1f}, staged {staged[r].max():.1f}, "
              f"chunks {nchunks[r].tolist()}")


if __name__ == "__main__":
    main()
