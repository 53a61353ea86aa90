#!/usr/bin/env python3
"""Work balance of the all-pairs search's multi-GPU dealing, measured on one GPU.

Runs each of n_shards shards of the configs[2] search (nmz_ed_allpairs_knn_shard_dev: every n_shards-th
work chunk) one after the other on one device and records, per shard, the kernel time (HIP events) and
k_ed_bv's executed-block counter. The job finishes when the slowest rank does, so max / mean of these is
the dealing's loss at n_shards GPUs. ED_BAL_ORDER=reverse runs the shards last to first (separates a trend over
the run, e.g. the clock, from one over the shard index); ED_BAL_REPS=r times each shard r times back to back and
keeps the last. The record's "uninstrumented" block times every search again with the library's timing off (two
events around ED_BAL_OUTER back-to-back searches): the bound without the per-phase event markers. usage: ed_shard_balance.py [generator] [n_shards] > out.json
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    gen = sys.argv[1] if len(sys.argv) > 1 else "clustered_traces"
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    import torch
    from namazu_amd import _lib, synth
    L = _lib.load()
    ctx = _lib.Context(0)
    N, Lx, w, k = 100_000, 2048, 32, 8
    ts = getattr(synth, gen)(N, Lx, **({"family": 1024} if gen == "clustered_traces" else {}))
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_ed_plan_create(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), N, w, ctypes.byref(plan)))
    d = torch.empty(N * k, dtype=torch.int64, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for s in range(S):  # untimed: each shard's first call builds its tile list and the search's scratch
        _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, s, S, ctypes.c_void_p(d.data_ptr()), stream))
    torch.cuda.synchronize()
    _lib.check(L.nmz_timing_enable(ctx.handle, 1))
    # the unsharded search on the same plan: the reference for max shard time (ideal: unsharded / S)
    _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, 0, 1, ctypes.c_void_p(d.data_ptr()), stream))
    torch.cuda.synchronize()
    tot, c = ctypes.c_double(), ctypes.c_uint64()
    L.nmz_timing_read(ctx.handle, b"ed_bv", ctypes.byref(tot), ctypes.byref(c), 1)
    _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, 0, 1, ctypes.c_void_p(d.data_ptr()), stream))
    torch.cuda.synchronize()
    _lib.check(L.nmz_timing_read(ctx.handle, b"ed_bv", ctypes.byref(tot), ctypes.byref(c), 1))
    full_ms = tot.value
    rows = []
    cnt = np.zeros(_lib.NMZ_ED_NCOUNTERS, np.uint64)
    order = list(range(S))[::-1] if os.environ.get("ED_BAL_ORDER") == "reverse" else list(range(S))
    reps = max(1, int(os.environ.get("ED_BAL_REPS", "1")))
    for s in order:
        for _ in range(reps - 1):
            _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, s, S, ctypes.c_void_p(d.data_ptr()), stream))
        torch.cuda.synchronize()
        tot, c = ctypes.c_double(), ctypes.c_uint64()
        ph = {n: (ctypes.c_double(), ctypes.c_uint64()) for n in (b"ed_qg_filter", b"ed_bv_dp")}
        L.nmz_timing_read(ctx.handle, b"ed_bv", ctypes.byref(tot), ctypes.byref(c), 1)
        for n, (a, b) in ph.items():
            L.nmz_timing_read(ctx.handle, n, ctypes.byref(a), ctypes.byref(b), 1)
        _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, s, S, ctypes.c_void_p(d.data_ptr()), stream))
        torch.cuda.synchronize()
        _lib.check(L.nmz_timing_read(ctx.handle, b"ed_bv", ctypes.byref(tot), ctypes.byref(c), 1))
        for n, (a, b) in ph.items():
            L.nmz_timing_read(ctx.handle, n, ctypes.byref(a), ctypes.byref(b), 1)
        _lib.check(L.nmz_ed_plan_counters(plan, _lib.ptr(cnt), stream))
        rows.append({"shard": s, "kernel_ms": tot.value, "filter_ms": ph[b"ed_qg_filter"][0].value,
                     "dp_ms": ph[b"ed_bv_dp"][0].value, "dp_pairs": int(cnt[0]), "blocks": int(cnt[2]),
                     "in_band": int(cnt[1])})
    rows.sort(key=lambda r: r["shard"])
    # The same searches with the library's timing off, each timed from outside: two events around ED_BAL_OUTER
    # back-to-back searches on the search's own stream. The instrumented pass above records an event pair per
    # timed phase inside every search (each record a queue marker of ~6 us): a fixed cost that 8 shards pay 8
    # times and the unsharded search once, which an 8-GPU job without timing does not pay at all.
    _lib.check(L.nmz_timing_enable(ctx.handle, 0))
    n_outer = max(1, int(os.environ.get("ED_BAL_OUTER", "4")))

    # (`stream` is torch's default stream, handle 0: the library then runs on its context's own stream, which the
    # events must bracket)
    cst = torch.cuda.ExternalStream(ctx.stream()) if stream.value is None else torch.cuda.current_stream()

    def outer(s, n_sh):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(cst)
        for _ in range(n_outer):
            _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, s, n_sh, ctypes.c_void_p(d.data_ptr()), stream))
        e1.record(cst)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n_outer

    u0 = outer(0, 1)
    for r in rows:
        r["outer_ms"] = outer(r["shard"], S)
    u1 = outer(0, 1)  # again after the shards: a drift check
    L.nmz_ed_plan_destroy(plan)
    om = np.array([r["outer_ms"] for r in rows])
    u = (u0 + u1) / 2
    uninstrumented = {"unsharded_ms": u, "unsharded_ms_before_after": [u0, u1], "max_shard_ms": float(om.max()),
                      "sum_shard_ms": float(om.sum()), "sum_over_unsharded": float(om.sum() / u),
                      "time_max_over_mean": float(om.max() / om.mean()), "speedup_bound": float(u / om.max()),
                      "searches_per_timing": n_outer}
    ms = np.array([r["kernel_ms"] for r in rows])
    bl = np.array([r["blocks"] for r in rows], np.float64)
    print(json.dumps({"generator": gen, "traces": N, "events": Lx, "band": w, "shards": S, "per_shard": rows,
                      "time_max_over_mean": float(ms.max() / ms.mean()),
                      "blocks_max_over_mean": float(bl.max() / bl.mean()),
                      "sum_shard_ms": float(ms.sum()), "unsharded_ms": full_ms,
                      "max_shard_ms": float(ms.max()), "speedup_bound": float(full_ms / ms.max()),
                      "item": int(os.environ.get("NMZ_ED_ITEM", "4096")),
                      "deal": os.environ.get("NMZ_ED_DEAL", "snake"),
                      "order": "reverse" if order[0] else "forward", "reps": reps,
                      "uninstrumented": uninstrumented}, indent=1))


if __name__ == "__main__":
    main()
