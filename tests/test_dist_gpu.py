"""The N > 1 path on real hardware: two ranks (processes) on the one GPU of the box, gloo for the collectives
(RCCL refuses two ranks on one device), each rank running the product's own shard functions on the device --
dist.RandomShardSweep (configs[3]: seed-range share + device top-k) and nmz_ed_allpairs_knn_shard_dev (configs[2]:
its dealt chunks) -- then all_gather and the product's merges (dist.merge_topk, nmz_knn_merge_dev). The merged
results must equal one unsharded run and the oracle."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs():
    from namazu_amd import _lib
    from namazu_amd.synth import clustered_traces
    rng = np.random.default_rng(21)
    E = 3000
    eh = rng.integers(0, 2**64, size=E, dtype=np.uint64)
    ec = (np.where(np.arange(E) % 16 < 4, _lib.NMZ_EV_PRIORITIZED, 0) | _lib.NMZ_EV_FAULTABLE).astype(np.uint8)
    ts = clustered_traces(1500, 300, seed=3, family=100)
    return eh, ec, ts


def _worker(rank, world, port, q, opts_by_rank=(0, 0)):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch
    import torch.distributed as dist
    from namazu_amd import _lib
    from namazu_amd import dist as nd
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eh, ec, ts = _inputs()
        ctx = _lib.Context(0)
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        params = _lib.resolve_random_params(30_000_000, 100_000_000, 0.2)
        sh = nd.RandomShardSweep(ctx, torch, "cuda", eh, ec, params, 777, 50_001, world, rank, k=32)
        sh.step(stream)
        torch.cuda.synchronize()
        merged = nd.gather_topk(dist, sh.topk(), 32)
        sh.close()
        L = _lib.load()
        N, k = len(ts), 6
        plan = ctypes.c_void_p()
        _lib.check(L.nmz_ed_plan_create_opts(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), None, N, 32,
                                             opts_by_rank[rank], ctypes.byref(plan)))
        try:
            nd.check_ed_plans(dist, L, plan)
        except ValueError as e:
            L.nmz_ed_plan_destroy(plan)
            q.put((rank, "mismatch", str(e)))
            ctx.close()
            return
        part = torch.empty(N * k, dtype=torch.int64, device="cuda")
        _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, rank, world, ctypes.c_void_p(part.data_ptr()), stream))
        torch.cuda.synchronize()
        parts = [torch.empty(N * k, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(parts, part.cpu())
        d_parts = torch.cat(parts).cuda()
        out = torch.empty(N * k, dtype=torch.int64, device="cuda")
        _lib.check(L.nmz_knn_merge_dev(ctx.handle, ctypes.c_void_p(d_parts.data_ptr()), world, N, k,
                                       ctypes.c_void_p(out.data_ptr()), stream))
        _lib.check(L.nmz_ed_knn_fill_dev(plan, k, ctypes.c_void_p(out.data_ptr()), stream))
        torch.cuda.synchronize()
        L.nmz_ed_plan_destroy(plan)
        q.put((rank, merged.tobytes(), out.cpu().numpy().tobytes()))
        ctx.close()
    finally:
        dist.destroy_process_group()


def test_two_ranks_on_device_shard_and_merge(ctx):
    from namazu_amd import _lib
    from namazu_amd import dist as nd
    from namazu_amd import historystorage as hs
    from oracle import oracle as O
    world = 2
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    port = _free_port()
    procs = [mctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    eh, ec, ts = _inputs()
    import torch
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    full = nd.RandomShardSweep(ctx, torch, "cuda", eh, ec, _lib.resolve_random_params(30_000_000, 100_000_000, 0.2),
                               777, 50_001, 1, 0, k=32)
    full.step(stream)
    torch.cuda.synchronize()
    exp_top = full.topk()
    full.close()
    st, _, _ = O.random_sweep(777, 200, eh, ec, O.random_params(30_000_000, 100_000_000, 0.2))
    ids, ds = hs.allpairs_knn(ts, 6, 32, ctx=ctx)
    for rank, tk, kn in res:
        assert np.frombuffer(tk, _lib.TOPK_DTYPE).tolist() == exp_top.tolist()
        keys = np.frombuffer(kn, np.uint64).reshape(len(ts), 6)
        assert np.array_equal((keys >> np.uint64(32)).astype(np.uint32), ds)
        assert np.array_equal((keys & np.uint64(0xFFFFFFFF)).astype(np.uint32), ids)
    for qi in [0, 250, 1499]:  # the merged lists against the oracle's brute force
        pairs = np.array([[qi, c] for c in range(len(ts)) if c != qi], np.uint32)
        d = O.ed_pairs(ts.off, ts.sym, pairs, 32)
        order = np.lexsort((pairs[:, 1], d))[:6]
        assert ds[qi].tolist() == d[order].tolist() and ids[qi].tolist() == pairs[order, 1].tolist()
    # the winners' stats vs the oracle
    best = exp_top[0]
    ost, _, _ = O.random_sweep(int(best["seed"]), 1, eh, ec, O.random_params(30_000_000, 100_000_000, 0.2))
    assert int(ost["n_fault"][0]) == int(best["n_fault"])
    assert st is not None


def test_two_ranks_mismatched_ed_plans_fail(ctx):
    """Rank 1 builds its plan with the single-kernel search (NMZ_ED_OPT_SINGLE_KERNEL): the plans' fingerprints
    differ, so dist.check_ed_plans raises on both ranks before any shard runs, instead of merging k-NN lists from
    searches that might deal pairs differently."""
    from namazu_amd import _lib
    world = 2
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    port = _free_port()
    procs = [mctx.Process(target=_worker, args=(r, world, port, q, (0, _lib.NMZ_ED_OPT_SINGLE_KERNEL)))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(r[0] for r in res) == [0, 1]
    for rank, what, msg in res:
        assert what == "mismatch" and "ranks [1]" in msg, (rank, what)
