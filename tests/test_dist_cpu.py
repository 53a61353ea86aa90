"""CPU (gloo, world_size 2): the N>1 host logic -- seed-range sharding (dist.shard_range), all_gather of per-rank
top-k and k-NN partial lists (dist.gather_topk, dist.all_gather_bytes), deterministic merges (dist.merge_topk,
dist.merge_knn_keys) -- checked against the single-process oracle result. The shares are dealt by the product's
own rules (dist.shard_range for seeds; dist.ed_pair_shard, checked against the library's nmz_ed_block_shard, for
trace pairs); there is no device here, so each rank's share of the work is computed by the oracle. The same path
with every rank on the device (the product's shard functions and the device merge) runs in tests/test_dist_gpu.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from namazu_amd import dist as nd
from oracle import oracle as O


ED_N = 300  # five query blocks of 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        E, S, K = 40, 300, 16
        rng = np.random.default_rng(3)
        eh = rng.integers(0, 2**64, size=E, dtype=np.uint64)
        ec = rng.integers(0, 4, size=E, dtype=np.uint8)
        p = O.random_params(30_000_000, 100_000_000, 0.3)
        lo, hi = nd.shard_range(S, world, rank)
        # per-rank stats from the oracle stand in for the rank's GPU sweep here
        st, _, _ = O.random_sweep(1000 + lo, hi - lo, eh, ec, p)
        local = O.topk_from_stats(st, 1000 + lo, K)
        merged = nd.gather_topk(dist, local, K)
        # k-NN partial lists: each rank computes a disjoint subset of pairs
        N, k, w = ED_N, 5, 4
        trs = [rng.integers(0, 3, rng.integers(3, 10)).astype(np.uint64) for _ in range(N)]
        off = np.zeros(N + 1, np.uint64)
        off[1:] = np.cumsum([len(t) for t in trs])
        sym = np.concatenate(trs)
        # the two-phase search's dealing: pair (i, j), i < j, belongs to the shard of query block i // 64
        pairs = np.array([[i, j] for i in range(N) for j in range(i + 1, N) if nd.ed_pair_shard(i, j, world) == rank],
                         np.uint32).reshape(-1, 2)
        mine = pairs
        d = O.ed_pairs(off, sym, mine, w)
        keys = np.full((N, k), np.iinfo(np.uint64).max, np.uint64)
        # as a bit-parallel shard lists them: in-band results only; the merge is completed by fill_knn_keys
        for (i, j), dd in zip(mine, d):
            if dd > w:
                continue
            for a, b in ((i, j), (j, i)):
                row = np.append(keys[a], np.uint64((int(dd) << 32) | int(b)))
                keys[a] = np.sort(row)[:k]
        import torch
        t = torch.from_numpy(keys.view(np.uint8).reshape(-1).copy())
        parts = nd.all_gather_bytes(dist, t)
        merged_knn = nd.fill_knn_keys(nd.merge_knn_keys([pp.numpy().view(np.uint64).reshape(N, k) for pp in parts], k),
                                      N, w + 1)
        q.put((rank, merged.tobytes(), merged_knn.tobytes(), len(mine)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_topk_and_knn(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # reference: single-process oracle over all seeds / all pairs
    E, S, K = 40, 300, 16
    rng = np.random.default_rng(3)
    eh = rng.integers(0, 2**64, size=E, dtype=np.uint64)
    ec = rng.integers(0, 4, size=E, dtype=np.uint8)
    st, _, _ = O.random_sweep(1000, S, eh, ec, O.random_params(30_000_000, 100_000_000, 0.3))
    exp = O.topk_from_stats(st, 1000, K)
    N, k, w = ED_N, 5, 4
    trs = [rng.integers(0, 3, rng.integers(3, 10)).astype(np.uint64) for _ in range(N)]
    off = np.zeros(N + 1, np.uint64)
    off[1:] = np.cumsum([len(t) for t in trs])
    oi, od = O.ed_allpairs_knn(off, np.concatenate(trs), w, k)
    assert sum(r[3] for r in res) == N * (N - 1) // 2 and min(r[3] for r in res) > 0  # a partition, both busy
    for rank, tk, kn, _ in res:
        assert np.frombuffer(tk, O.TOPK_DTYPE).tolist() == exp.tolist()
        keys = np.frombuffer(kn, np.uint64).reshape(N, k)
        ids = (keys & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        ds = (keys >> np.uint64(32)).astype(np.uint32)
        empty = keys == np.iinfo(np.uint64).max
        ids[empty] = 0xFFFFFFFF
        ds[empty] = 0xFFFFFFFF
        assert np.array_equal(ids, oi) and np.array_equal(ds, od)


def test_shard_range_partitions():
    for total in [0, 1, 7, 1 << 20, 10_000_001]:
        for world in [1, 2, 3, 8]:
            rs = [nd.shard_range(total, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def test_merge_topk_is_order_independent():
    a = np.zeros(5, O.TOPK_DTYPE)
    a["seed"] = [5, 1, 9, 2, 7]
    a["n_fault"] = [1, 2, 2, 0, 1]
    a["sum_delay_ns"] = [10, 3, 3, 50, 10]
    m1 = nd.merge_topk([a[:2], a[2:]], 4)
    m2 = nd.merge_topk([a[3:], a[:3]], 4)
    assert m1.tolist() == m2.tolist()
    assert m1["seed"].tolist() == [1, 9, 5, 7]


@pytest.mark.parametrize("deal", [None, "snake", "hash"])
def test_ed_pair_dealing_matches_library(ab_knobs, monkeypatch, deal):
    """dist.ed_block_shard restates the library's dealing rule (csrc/ed.hip ed_block_shard; host-only entry point).
    The rule is fixed: the round-3 A/B knobs (NMZ_ED_DEAL, NMZ_ED_DEAL_UNIT) set in a process's environment change
    nothing, so ranks with different environments still deal the same blocks (a rank that dealt differently would
    drop or double pairs of the merged k-NN)."""
    from namazu_amd import _lib
    if deal:
        monkeypatch.setenv("NMZ_ED_DEAL", deal)
        monkeypatch.setenv("NMZ_ED_DEAL_UNIT", "4")
    L = _lib.load()

    def rotated_snake(qb, S):
        r = qb % (2 * S)
        return ((r if r < S else 2 * S - 1 - r) + qb // (2 * S)) % S

    for world in [1, 2, 3, 8]:
        for qb in list(range(300)) + [2**20 + 7, 2**31 - 1]:
            want = rotated_snake(qb, world) if world > 1 else 0
            assert L.nmz_ed_block_shard(qb, world) == nd.ed_block_shard(qb, world) == want
    # every block has an owner in range, and 8 shards all get blocks
    assert sorted({nd.ed_block_shard(qb, 8) for qb in range(1563)}) == list(range(8))
    # a block and its mirror share a shard; every 2S blocks give each shard exactly two
    for S in [2, 3, 8]:
        for g in range(5):
            own = [nd.ed_block_shard(2 * S * g + r, S) for r in range(2 * S)]
            assert sorted(own) == sorted(list(range(S)) * 2)
            assert all(own[r] == own[2 * S - 1 - r] for r in range(S))
    # rotated: over S periods a shard takes every pair position once
    S = 8
    for sh in range(S):
        pos = {min(qb % 16, 15 - qb % 16) for qb in range(16 * S) if nd.ed_block_shard(qb, S) == sh}
        assert pos == set(range(S))
