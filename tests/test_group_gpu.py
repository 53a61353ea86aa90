"""GPU: device groups (multi-GPU inside the C ABI, csrc/group.hip) vs the unsharded calls and the oracle.

On the one-GPU box a group has one device; `n_shards` > 1 makes virtual shards, so the seed-range split, the
per-rank merge of several shards' lists, the RCCL all_gather (one rank) and the final merge all run. The
results must equal one unsharded call bit for bit (cli/run.go:123-136 and cli/tools/visualize.go:138-172 are the
single-process callers this serves)."""
import ctypes

import numpy as np
import pytest

from namazu_amd import _lib
from namazu_amd import group as G
from namazu_amd import historystorage as hs
from namazu_amd.explorepolicy import to_csr
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def groups():
    cache = {}

    def get(n_shards):
        if n_shards not in cache:
            cache[n_shards] = G.Group((0,), n_shards=n_shards)
        return cache[n_shards]
    yield get
    for g in cache.values():
        g.close()


def _hints(n, seed):
    rng = np.random.default_rng(seed)
    return [str(int(x)) for x in rng.integers(-2**63, 2**63 - 1, size=n, dtype=np.int64)]


@pytest.mark.parametrize("n_shards", [1, 3, 8, 13])
def test_group_replayable_one_call_equals_oracle(groups, n_shards):
    g = groups(n_shards)
    assert g.n_ranks == 1 and g.n_local == 1 and g.n_shards == n_shards
    seeds = ["foobar", ""] + [str(i) for i in range(997)]
    so, sb = to_csr(seeds)
    ho, hb = to_csr(_hints(300, n_shards))
    m = 100_000_000
    st, tk = g.replayable_sweep(so, sb, ho, hb, m, k=16)
    ost, _ = O.replayable_sweep(so, sb, ho, hb, m)
    assert np.array_equal(st, ost)
    assert np.array_equal(tk, O.topk_from_stats(ost, 0, 16))


@pytest.mark.parametrize("n_seeds,n_shards,k", [(5, 8, 10), (0, 4, 3), (1, 1, 1), (64, 8, 64)])
def test_group_replayable_empty_and_small_shards(groups, n_seeds, n_shards, k):
    """Fewer seeds than shards (empty shards contribute sentinel lists) and k above the seed count."""
    g = groups(n_shards)
    seeds = [f"s{i}" for i in range(n_seeds)]
    so, sb = to_csr(seeds)
    ho, hb = to_csr(_hints(70, 7))
    st, tk = g.replayable_sweep(so, sb, ho, hb, 1_000_000_000, k=k)
    ost, _ = O.replayable_sweep(so, sb, ho, hb, 1_000_000_000)
    assert np.array_equal(st, ost)
    assert np.array_equal(tk, O.topk_from_stats(ost, 0, k))


@pytest.mark.parametrize("seed_lo", [0, 95, 999_999_990, 10**18 - 7, 2**64 - 40])
def test_group_replayable_decimal_seeds(groups, seed_lo):
    """nmz_replayable_group_sweep_decimal: seeds are the decimal strings of seed_lo + i (generated on the device,
    wrapping past 2^64), across the 10^9 and 10^18 digit-group boundaries; top-k .seed = the integer value."""
    g = groups(8)
    n = 100
    vals = [(seed_lo + i) % (1 << 64) for i in range(n)]
    so, sb = to_csr([str(v) for v in vals])
    ho, hb = to_csr(_hints(257, 3))
    m = 33_333_333
    p = G.ReplayableGroupPlan(g, ho, hb, m, max_seeds_per_shard=64)
    st, tk = p.sweep_decimal(seed_lo, n, k=12)
    st2, tk2 = p.sweep(so, sb, k=12)
    p.close()
    ost, _ = O.replayable_sweep(so, sb, ho, hb, m)
    assert np.array_equal(st, ost) and np.array_equal(st2, ost)
    ref = O.topk_from_stats(ost, 0, 12)
    assert np.array_equal(tk2, ref)
    # decimal form: .seed is seed_lo + index (mod 2^64)
    ref_dec = ref.copy()
    ref_dec["seed"] = [(seed_lo + int(s)) % (1 << 64) for s in ref["seed"]]
    assert np.array_equal(tk, ref_dec)


def test_replayable_decimal_single_device_matches_csr(ctx):
    """nmz_replayable_sweep_decimal_topk_dev on one context equals nmz_replayable_sweep_topk_dev over the CSR of
    the same strings (the bench's seed layout), 4,096 seeds x 1,024 hints through the order-query kernel."""
    import torch
    L = _lib.load()
    lo, n, E, m, k = 123_456_789, 4096, 1024, 100_000_000, 32
    so, sb = to_csr([str(lo + i) for i in range(n)])
    ho, hb = to_csr(_hints(E, 11))
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), E, m, n, ctypes.byref(plan)))
    d_soff = torch.from_numpy(so.view(np.int32)).cuda()
    d_sb = torch.from_numpy(sb).cuda()
    out = []
    for dec in (False, True):
        d_st = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        d_tk = torch.empty(k * 24, dtype=torch.uint8, device="cuda")
        if dec:
            _lib.check(L.nmz_replayable_sweep_decimal_topk_dev(plan, lo, n, k, ctypes.c_void_p(d_st.data_ptr()),
                                                               ctypes.c_void_p(d_tk.data_ptr()), None))
        else:
            _lib.check(L.nmz_replayable_sweep_topk_dev(plan, ctypes.c_void_p(d_soff.data_ptr()),
                                                       ctypes.c_void_p(d_sb.data_ptr()), n, lo, k,
                                                       ctypes.c_void_p(d_st.data_ptr()),
                                                       ctypes.c_void_p(d_tk.data_ptr()), None))
        torch.cuda.synchronize()
        out.append((d_st.cpu().numpy().tobytes(), d_tk.cpu().numpy().tobytes()))
    L.nmz_replayable_plan_destroy(plan)
    assert out[0] == out[1]
    ost, _ = O.replayable_sweep(so, sb, ho, hb, m, nthreads=16)
    assert np.frombuffer(out[1][0], _lib.SCHED_STATS_DTYPE).tobytes() == ost.tobytes()


@pytest.mark.parametrize("n_shards,seed0", [(1, 7), (5, 2**64 - 300), (8, 1234)])
def test_group_random_equals_oracle(groups, n_shards, seed0):
    g = groups(n_shards)
    E, n, k = 512, 777, 24
    rng = np.random.default_rng(n_shards)
    evhash = rng.integers(0, 2**64, size=E, dtype=np.uint64)
    evclass = rng.integers(0, 4, size=E).astype(np.uint8)
    params = _lib.resolve_random_params(30_000_000, 100_000_000, 0.1)
    st, tk = g.random_sweep(seed0, n, evhash, evclass, params, k=k)
    pr = O.random_params(30_000_000, 100_000_000, 0.1)
    ost, _, _ = O.random_sweep(seed0, n, evhash, evclass, pr, nthreads=16)
    assert np.array_equal(st, ost)
    assert np.array_equal(tk, O.topk_from_stats(ost, seed0, k))
    # the resident group plan, swept twice (the second sweep reuses every buffer)
    p = G.RandomGroupPlan(g, evhash, evclass, params, max_seeds_per_shard=(n + n_shards - 1) // n_shards)
    for _ in range(2):
        st2, tk2 = p.sweep(seed0, n, k=k)
        assert np.array_equal(st2, ost) and np.array_equal(tk2, tk)
    p.close()


def _family(n, length, alphabet, edits, seed):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, alphabet, size=length)
    out = []
    for i in range(n):
        t = base.copy()
        for _ in range(int(rng.integers(0, edits + 1))):
            t[int(rng.integers(0, length))] = int(rng.integers(0, alphabet))
        if i % 37 == 5:
            t = t[: length - int(rng.integers(1, 20))]
        out.append(t.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(5))
    return hs.TraceSet(out)


@pytest.mark.parametrize("band,n_shards", [(32, 1), (32, 8), (32, 11), (16, 3), (5, 8), (100, 3)])
def test_group_ed_allpairs_knn_equals_oracle(groups, band, n_shards):
    """All-pairs k-NN over a group: the store as 1/n_ranks shares + RCCL all_gather + device plan builds, shards by
    the plan's query-block deal, per-rank merge of the shards' partial lists (chained 8 at a time beyond 8
    shards), RCCL all_gather, merge and band + 1 fill; vs the oracle (band 100: the wide kernel)."""
    g = groups(n_shards)
    ts = _family(300, 200, 12, 40, band * 100 + n_shards)
    k = 8
    ids, ds = g.ed_allpairs_knn(ts, band, k)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, band, k, nthreads=16)
    assert np.array_equal(ids, oi) and np.array_equal(ds, od)
    p = G.EdGroupPlan(g, ts, band)
    i2, d2 = p.knn(k)
    t = p.timing()
    p.close()
    assert np.array_equal(i2, oi) and np.array_equal(d2, od)
    assert all(len(v) == g.n_local and all(x >= 0 for x in v) for v in t.values())
    assert t["build_ms"][0] > 0


def test_group_close_refuses_live_plans_and_keeps_caller_device():
    """nmz_close_group refuses while a group plan is alive (closing under a live plan freed what the plan
    still used), and group calls leave the calling thread's current device as it was."""
    import torch
    g = G.Group((0,), n_shards=2)
    ts = _family(40, 50, 6, 5, 1)
    p = G.EdGroupPlan(g, ts, 8)
    with pytest.raises(_lib.NmzError):
        g.close()
    p.knn(4)
    assert torch.cuda.current_device() == 0
    p.close()
    g.close()
    g.close()  # idempotent


def test_group_rank_form_single_rank(groups):
    """nmz_open_group_rank (one process per device) with one rank: the id from nmz_group_unique_id, every shard
    on this rank; equals the oracle."""
    uid = G.Group.unique_id()
    assert len(uid) == G.GROUP_ID_BYTES
    g = G.Group((0,), n_shards=4, unique_id=uid, n_ranks=1, rank=0)
    try:
        assert g.n_ranks == 1 and g.n_shards == 4
        seeds = [str(i) for i in range(300)]
        so, sb = to_csr(seeds)
        ho, hb = to_csr(_hints(128, 5))
        st, tk = g.replayable_sweep(so, sb, ho, hb, 10_000_000, k=8)
        ost, _ = O.replayable_sweep(so, sb, ho, hb, 10_000_000)
        assert np.array_equal(st, ost) and np.array_equal(tk, O.topk_from_stats(ost, 0, 8))
    finally:
        g.close()


def test_group_rejects_bad_arguments():
    L = _lib.load()
    h = ctypes.c_void_p()
    assert L.nmz_open_group(0, 0, ctypes.byref(h)) == _lib.NMZ_EINVAL  # no device
    assert L.nmz_open_group(1 << 31, 0, ctypes.byref(h)) == _lib.NMZ_EINVAL  # no such device


def _collectives(g):
    n = ctypes.c_uint64()
    _lib.check(g.L.nmz_group_collectives(g.handle, ctypes.byref(n)))
    return n.value


@pytest.mark.parametrize("where", ["sweep", "topk", "exchange", "ed_search"])
@pytest.mark.parametrize("rank_form", [False, True])
def test_group_failure_keeps_collectives_in_step(ab_knobs, monkeypatch, where, rank_form):
    """A rank that fails locally still enters the status all_gather in front of every payload collective
    (csrc/group.hip group_agree_status), so no peer waits in a collective it skipped. NMZ_GROUP_FAIL injects the
    failure at one step: the call returns the injected error, it entered exactly the status collective (the one
    its peers enter too; a healthy call enters the status collective and the payload all_gather), and the group's
    next call succeeds with the oracle's result. For "exchange" the status exchange's own staging fails: the rank
    still enters, and its send buffer's failure sentinel tells the peers."""
    if rank_form:
        g = G.Group((0,), n_shards=3, unique_id=G.Group.unique_id(), n_ranks=1, rank=0)
    else:
        g = G.Group((0,), n_shards=3)
    try:
        E, n, k = 256, 300, 8
        rng = np.random.default_rng(11)
        evhash = rng.integers(0, 2**64, size=E, dtype=np.uint64)
        evclass = rng.integers(0, 4, size=E).astype(np.uint8)
        params = _lib.resolve_random_params(30_000_000, 100_000_000, 0.1)
        ost, _, _ = O.random_sweep(5, n, evhash, evclass, O.random_params(30_000_000, 100_000_000, 0.1), nthreads=16)
        ts = _family(120, 100, 12, 30, 3)
        oi, od = O.ed_allpairs_knn(ts.off, ts.sym, 16, k, nthreads=16)
        p = G.RandomGroupPlan(g, evhash, evclass, params, max_seeds_per_shard=n)
        e = G.EdGroupPlan(g, ts, 16)
        try:
            def call():
                if where == "ed_search":
                    return e.knn(k)
                return p.sweep(5, n, k=k)

            c0 = _collectives(g)
            call()
            healthy = _collectives(g) - c0
            assert healthy == 2  # status agreement + payload all_gather
            monkeypatch.setenv("NMZ_GROUP_FAIL", where)
            c0 = _collectives(g)
            with pytest.raises(_lib.NmzError, match="injected failure at " + where):
                call()
            assert _collectives(g) - c0 == 1  # the status all_gather only, as on every healthy peer
            monkeypatch.setenv("NMZ_GROUP_FAIL_RANK", "1")  # another rank's knob: not this one
            call()
            monkeypatch.delenv("NMZ_GROUP_FAIL")
            c0 = _collectives(g)
            if where == "ed_search":
                ids, ds = call()
                assert np.array_equal(ids, oi) and np.array_equal(ds, od)
            else:
                st, tk = call()
                assert np.array_equal(st, ost) and np.array_equal(tk, O.topk_from_stats(ost, 5, k))
            assert _collectives(g) - c0 == 2
        finally:
            p.close()
            e.close()
    finally:
        g.close()
