#!/usr/bin/env python3
"""Is the sharded search's overhead in the shards or in how they are timed? (measurement infrastructure)

configs[2] on one GPU, three ways, each after a warm-up of every shard: the unsharded search; the n_shards shards
launched back to back with one synchronisation at the end (the device never idles between them); and each shard
on its own, synchronised before and after (how tools/ed_shard_balance.py times them). Wall time by HIP events on
the stream. usage: ed_shard_backtoback.py [generator] [n_shards] > out.json
"""
import ctypes
import json
import os
import sys

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
    cs = torch.cuda.current_stream()
    stream = ctypes.c_void_p(cs.cuda_stream)

    def run(s, n):
        _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, s, n, ctypes.c_void_p(d.data_ptr()), stream))

    for s in range(S):
        run(s, S)
    run(0, 1)
    torch.cuda.synchronize()

    def timed(fn, reps=3):
        out = []
        for _ in range(reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cs)
            fn()
            e1.record(cs)
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1))
        return min(out)

    full = timed(lambda: run(0, 1))
    b2b = timed(lambda: [run(s, S) for s in range(S)])
    alone = [timed(lambda s=s: run(s, S)) for s in range(S)]
    L.nmz_ed_plan_destroy(plan)
    print(json.dumps({"generator": gen, "shards": S, "unsharded_ms": full, "shards_back_to_back_ms": b2b,
                      "shards_alone_ms": alone, "sum_alone_ms": sum(alone), "max_alone_ms": max(alone),
                      "back_to_back_over_unsharded": b2b / full, "sum_alone_over_unsharded": sum(alone) / full},
                     indent=1))


if __name__ == "__main__":
    main()
