"""GPU parity: K1 replayable sweep and K2 random sweep vs the CPU oracle,
through the C ABI (libnmz_gpu.so). Bit-exact comparison everywhere."""
import ctypes

import numpy as np
import pytest

from namazu_amd import _lib
from namazu_amd.explorepolicy import Random, Replayable, to_csr
from oracle import oracle as O

pytestmark = pytest.mark.gpu

RNG = np.random.default_rng(0xBEEF)


def zk_hints(n, rng=RNG):
    v = rng.integers(-2**63, 2**63 - 1, size=n, dtype=np.int64)
    return [str(int(x)) for x in v]


def rep_oracle(seeds, hints, m, n_dump=0):
    so, sb = O.to_csr(seeds)
    ho, hb = O.to_csr(hints)
    return O.replayable_sweep(so, sb, ho, hb, m, n_dump=n_dump)


# ---------------------------------------------------------------- K1
@pytest.fixture(params=["wt", "wt_sep", "wt_bb7", "wt_bb5", "oq"])
def k1(ab_knobs, request, monkeypatch):
    """K1's two statistics kernels: wavelet trees (the default) and order queries (NMZ_REPLAY_WT=0 at plan
    creation); plans that neither fits take the per-decision sweep either way. "wt" builds the wavelet-tree plan
    with the fused plan kernel (it computes and C-sorts the correction table itself), "wt_sep" with the separate
    table, sort and plan kernels (NMZ_WT_FUSED=0, the path for classes of 4,096 events or more). The wavelet plans
    take the widest rank blocks (at most 64 ranks) whose row image fits LDS; "wt_bb7" / "wt_bb5" set the cap to 128 /
    32 ranks (NMZ_WT_BB: 32 is the width of larger rows)."""
    monkeypatch.delenv("NMZ_WT_FUSED", raising=False)
    monkeypatch.delenv("NMZ_WT_BB", raising=False)
    if request.param in ("wt_bb7", "wt_bb5"):
        monkeypatch.setenv("NMZ_WT_BB", request.param[-1])
    if request.param == "oq":
        monkeypatch.setenv("NMZ_REPLAY_WT", "0")
    else:
        monkeypatch.delenv("NMZ_REPLAY_WT", raising=False)
        if request.param == "wt_sep":
            monkeypatch.setenv("NMZ_WT_FUSED", "0")
    return request.param


def test_replayable_plan_kernel_choice(ab_knobs, ctx, monkeypatch):
    """configs[1]-shaped traces take the wavelet-tree kernel (classes of 4,096 events or more as sub-segments);
    NMZ_REPLAY_WT=0 or a row image beyond LDS the order-query kernel; maxInterval >= 2^32 the per-decision sweep."""
    L = _lib.load()

    def kind(hints, m):
        ho, hb = to_csr(hints)
        plan = ctypes.c_void_p()
        _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), len(hints), m, 1024,
                                                ctypes.byref(plan)))
        try:
            return L.nmz_replayable_plan_kernel(plan)
        finally:
            L.nmz_replayable_plan_destroy(plan)

    monkeypatch.delenv("NMZ_REPLAY_WT", raising=False)
    hints = zk_hints(4096)
    assert kind(hints, 100_000_000) == 2
    assert kind(hints, 2**32 - 1) == 2
    assert kind(hints, 2**32) == 0
    assert kind(["x" * 5] * 4097, 100_000_000) == 2  # one class of 4,097: two wavelet-tree sub-segments
    assert kind(zk_hints(12_000), 100_000_000) == 1  # row image beyond LDS: order-query passes
    monkeypatch.setenv("NMZ_REPLAY_WT", "0")
    assert kind(hints, 100_000_000) == 1


def test_replayable_golden_foobar(ctx, golden):
    for case in golden("replayable_foobar.json")["cases"]:
        p = Replayable()
        p.MaxInterval = case["max_interval_ns"]
        seeds = [case["seed"]] if "seed" in case else case["seed_list"]
        r = p.Sweep(seeds, case["hints"], n_dump=len(seeds), ctx=ctx)
        exp = [case["delays_ns"]] if "seed" in case else case["delays_ns"]
        assert r.delays.tolist() == exp


@pytest.mark.parametrize("m", [100_000_000, 1_000_000_000, 10_000_000, 1, 2, 999, 2**30 - 1, 2**30, 2**30 + 5,
                               2_000_000_000, 2**31 - 1, 2**31, 3_000_000_000, 2**32 - 1, 2**32,
                               2**62 + 11, 2**63 - 1, -5_000_000, -1, 0])
def test_replayable_moduli(ctx, k1, m):
    seeds = [str(i) for i in range(700)] + ["", "foobar", "x" * 50]
    hints = zk_hints(97) + ["", "a", "hint-entity-0-0", "z" * 33]
    p = Replayable()
    p.MaxInterval = m
    r = p.Sweep(seeds, hints, n_dump=20, k=10, ctx=ctx)
    st, dl = rep_oracle(seeds, hints, m, n_dump=20)
    assert np.array_equal(r.stats, st)
    assert np.array_equal(r.delays, dl)
    assert np.array_equal(r.topk, O.topk_from_stats(st, 0, 10))


def test_replayable_many_length_classes_and_ties(ctx, k1):
    """Hints of every length 0..40 (41 classes) and a tiny modulus (many ties):
    argmax must be the first original event index."""
    hints = ["h" * (i % 41) + str(i % 3) * (i % 2) for i in range(300)]
    seeds = [str(i) for i in range(600)]
    for m in [3, 7, 1000]:
        p = Replayable()
        p.MaxInterval = m
        r = p.Sweep(seeds, hints, ctx=ctx)
        st, _ = rep_oracle(seeds, hints, m)
        assert np.array_equal(r.stats, st)


@pytest.mark.parametrize("m", [1, 2, 3, 7, 1000, 100_000_000, 2**30 - 1, 2**31 + 3, 2**32 - 1])
def test_replayable_order_query_block_edges(ctx, k1, m):
    """K1's order-query statistics (k_replayable_sweep_oq): length classes whose sizes sit on both sides of the
    8-, 64- and 512-event block edges and of the per-event threshold (24), shuffled so the original event order
    mixes the classes; tiny moduli make most maxima ties, which must resolve to the first original event."""
    rng = np.random.default_rng(m)
    sizes = [25, 64, 511, 512, 513, 1025, 8, 24, 1, 65, 1600]
    hints = []
    for c, n in enumerate(sizes):
        hints += ["".join(rng.choice(list("0123456789-"), size=3 + c)) for _ in range(n)]
    hints = [hints[i] for i in rng.permutation(len(hints))]
    seeds = [str(i) for i in range(700)] + ["", "foobar"]
    p = Replayable()
    p.MaxInterval = m
    r = p.Sweep(seeds, hints, n_dump=2, ctx=ctx)
    st, dl = rep_oracle(seeds, hints, m, n_dump=2)
    assert np.array_equal(r.stats, st) and np.array_equal(r.delays, dl)


def test_replayable_repeated_hints_plan_sort_fallback(ctx, k1):
    """Many identical hints give identical C values in every table row, so one top-12-bit bucket of the plan's
    segment sort overflows and the segment takes the bitonic sort; ties in C must keep the event order."""
    rng = np.random.default_rng(7)
    hints = ["1234567890123456789"] * 150 + zk_hints(60, rng) + ["-123456789012345678"] * 40
    hints = [hints[i] for i in rng.permutation(len(hints))]
    seeds = [str(i) for i in range(500)]
    for m in [100_000_000, 7]:
        p = Replayable()
        p.MaxInterval = m
        r = p.Sweep(seeds, hints, n_dump=2, k=8, ctx=ctx)
        st, dl = rep_oracle(seeds, hints, m, n_dump=2)
        assert np.array_equal(r.stats, st) and np.array_equal(r.delays, dl)
        assert np.array_equal(r.topk, O.topk_from_stats(st, 0, 8))


@pytest.mark.parametrize("E", [1, 3, 63, 64, 65, 127, 2047, 2048, 2049, 4097, 9000])
def test_replayable_event_counts_around_stage_and_chunk_edges(ctx, k1, E):
    """K1 stages 64 events at a time (the next chunk's load is clamped to the last event) and works in
    2,048-event items: trace lengths on either side of both edges, vs the oracle."""
    rng = np.random.default_rng(E)
    hints = zk_hints(E, rng)
    seeds = [str(i) for i in range(260)]
    p = Replayable()
    p.MaxInterval = 100_000_000
    r = p.Sweep(seeds, hints, n_dump=3, ctx=ctx)
    st, dl = rep_oracle(seeds, hints, 100_000_000, n_dump=3)
    assert np.array_equal(r.stats, st) and np.array_equal(r.delays, dl)


@pytest.mark.parametrize("m", [100_000_000, 7, 2**31 + 3])
def test_replayable_one_long_class_sub_segments(ctx, monkeypatch, m):
    """4,500 hints of one length (one class of 4,500 >= 4,096 events: two wavelet-tree sub-segments of the C-sorted
    class, each with its own carry split and statistics) plus a few short hints, tiny modulus for ties, vs the
    oracle; the plan must take the wavelet-tree kernel."""
    monkeypatch.delenv("NMZ_REPLAY_WT", raising=False)
    rng = np.random.default_rng(m % 1000)
    hints = [str(x) for x in rng.integers(10**9, 10**10, size=4500)] + ["ab", "abc", "q"] * 3
    hints = [hints[i] for i in rng.permutation(len(hints))]
    seeds = [str(i) for i in range(400)] + ["foobar"]
    L = _lib.load()
    ho, hb = to_csr(hints)
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), len(hints), m, 512,
                                            ctypes.byref(plan)))
    assert L.nmz_replayable_plan_kernel(plan) == 2
    L.nmz_replayable_plan_destroy(plan)
    p = Replayable()
    p.MaxInterval = m
    r = p.Sweep(seeds, hints, n_dump=2, k=8, ctx=ctx)
    st, dl = rep_oracle(seeds, hints, m, n_dump=2)
    assert np.array_equal(r.stats, st) and np.array_equal(r.delays, dl)
    assert np.array_equal(r.topk, O.topk_from_stats(st, 0, 8))


@pytest.mark.parametrize("E,m", [(10_000, 100_000_000), (10_000, 2_000_000_000), (6_500, 2**32 - 1)])
def test_replayable_long_trace_multi_pass(ctx, k1, E, m):
    """Traces whose order-query row image exceeds LDS (E > ~6k): length classes split into C-sorted sub-segments
    packed into passes, one kernel run per pass, statistics combined per seed (sum adds, max keys max), incl.
    maxInterval 2 s and 2^32 - 1 ns (m >= 2^31: 32-bit residue sums that overflow), vs the oracle."""
    rng = np.random.default_rng(E + m % 1000)
    hints = zk_hints(E, rng) + ["h" * (i % 7) for i in range(40)]
    seeds = [str(i) for i in range(300)] + ["foobar"]
    p = Replayable()
    p.MaxInterval = m
    r = p.Sweep(seeds, hints, n_dump=2, k=8, ctx=ctx)
    st, dl = rep_oracle(seeds, hints, m, n_dump=2)
    assert np.array_equal(r.stats, st) and np.array_equal(r.delays, dl)
    assert np.array_equal(r.topk, O.topk_from_stats(st, 0, 8))


@pytest.mark.parametrize("budget,m", [(16384, 100_000_000), (30_000, 7), (60_000, 2**31 + 9)])
def test_replayable_forced_passes(ab_knobs, ctx, monkeypatch, budget, m):
    """NMZ_REPLAY_OQ_BUDGET shrinks the row-image budget so a 3,000-event trace runs as many passes over small
    sub-segments (and the rows' partial chunks accumulate across passes); results equal the oracle's."""
    monkeypatch.setenv("NMZ_REPLAY_OQ_BUDGET", str(budget))
    monkeypatch.setenv("NMZ_REPLAY_WT", "0")  # the order-query kernel's passes
    rng = np.random.default_rng(budget)
    hints = zk_hints(3000, rng) + ["x" * (i % 5) for i in range(30)]
    seeds = [str(i) for i in range(1500)]
    p = Replayable()
    p.MaxInterval = m
    r = p.Sweep(seeds, hints, k=5, ctx=ctx)
    st, _ = rep_oracle(seeds, hints, m)
    assert np.array_equal(r.stats, st)
    assert np.array_equal(r.topk, O.topk_from_stats(st, 0, 5))


def _seeds_in_one_row(row, n):
    """n decimal seeds whose FNV-1a 64 has low byte `row`: they all share one table row, i.e. one K1 workgroup."""
    off, prime = np.uint64(0xCBF29CE484222325), np.uint64(0x100000001B3)
    strs = np.arange(0, 400 * n + 1000).astype(str)
    lens = np.char.str_len(strs)
    h = np.zeros(len(strs), np.uint64)
    for ln in np.unique(lens):
        sel = lens == ln
        b = np.frombuffer("".join(strs[sel]).encode(), np.uint8).reshape(-1, ln)
        x = np.full(b.shape[0], off, np.uint64)
        with np.errstate(over="ignore"):
            for k in range(ln):
                x = (x ^ b[:, k].astype(np.uint64)) * prime
        h[sel] = x
    out = strs[(h & np.uint64(0xFF)) == np.uint64(row)][:n]
    assert len(out) == n
    return [str(x) for x in out]


@pytest.mark.parametrize("n", [1, 37, 64, 960, 1024, 1064, 1088, 2100])
def test_replayable_one_row_chunks_and_partial_chunk(ctx, k1, n):
    """K1 takes a row's seeds in 64-seed chunks from an LDS counter and shares the row's partial chunk (n mod 64
    seeds) between its waves by class segment: all seeds in one row, counts on both sides of whole chunks and of
    one chunk per wave (1,024), with 20 length classes (some per-event, some order-query) so a wave takes
    several segments of the partial chunk; plus a few seeds of other rows. Stats vs the oracle."""
    rng = np.random.default_rng(n)
    sizes = [3, 70, 9, 130, 1, 600, 17, 64, 65, 200, 5, 513, 33, 90, 2, 300, 12, 48, 150, 7]
    hints = []
    for c, k in enumerate(sizes):
        hints += ["".join(rng.choice(list("0123456789"), size=c + 1)) for _ in range(k)]
    hints = [hints[i] for i in rng.permutation(len(hints))]
    seeds = _seeds_in_one_row(0x2A, n) + ["x", "yy", "zzz"]
    for m in [100_000_000, 7]:
        p = Replayable()
        p.MaxInterval = m
        r = p.Sweep(seeds, hints, n_dump=2, k=16, ctx=ctx)
        st, dl = rep_oracle(seeds, hints, m, n_dump=2)
        assert np.array_equal(r.stats, st) and np.array_equal(r.delays, dl)
        assert np.array_equal(r.topk, O.topk_from_stats(st, 0, 16))


def test_replayable_empty_inputs(ctx):
    p = Replayable()
    p.MaxInterval = 10_000_000
    r = p.Sweep([], ["a"], ctx=ctx)
    assert len(r.stats) == 0
    r = p.Sweep(["s1", "s2"], [], k=2, ctx=ctx)
    st, _ = rep_oracle(["s1", "s2"], [], 10_000_000)
    assert np.array_equal(r.stats, st)
    assert r.stats["argmax_event"].tolist() == [_lib.NMZ_NONE] * 2


def test_replayable_bucket_boundaries(ctx):
    """Seed counts around the 256-seed work unit and bucket sizes."""
    hints = zk_hints(33)
    for n in [1, 63, 64, 255, 256, 257, 4095, 20000]:
        seeds = [f"s{i}" for i in range(n)]
        p = Replayable()
        p.MaxInterval = 100_000_000
        r = p.Sweep(seeds, hints, ctx=ctx)
        st, _ = rep_oracle(seeds, hints, 100_000_000)
        assert np.array_equal(r.stats, st), n


def test_replayable_seed_prefix_staging(ctx):
    """k_seed_prefix stages a block's 2,048 seed offsets and bytes in LDS when the bytes fit 32 KB (whole dwords
    between partial head and tail dwords at any alignment) and hashes from global memory otherwise: short seeds
    (staged), long seeds (not staged), blocks of each kind side by side, empty and multi-byte UTF-8 seeds."""
    rng = np.random.default_rng(17)
    alphabet = list("0123456789abcdefXYZ-_") + ["\u00e9", "\u4e2d", "\U0001f600"]

    def rand_seeds(n, lmax):
        return ["".join(rng.choice(alphabet, size=int(rng.integers(0, lmax + 1)))) for _ in range(n)]

    hints = zk_hints(70)
    for seeds in (rand_seeds(6000, 12), rand_seeds(3000, 60), rand_seeds(2048, 6) + rand_seeds(2048, 40) +
                  rand_seeds(777, 3)):
        p = Replayable()
        p.MaxInterval = 100_000_000
        r = p.Sweep(seeds, hints, ctx=ctx)
        st, _ = rep_oracle(seeds, hints, 100_000_000)
        assert np.array_equal(r.stats, st)


def test_replayable_device_plan_api(ctx):
    """nmz_replayable_plan_create + nmz_replayable_sweep_dev on resident buffers."""
    import torch
    L = _lib.load()
    hints = zk_hints(128)
    seeds = [str(i) for i in range(3000)]
    ho, hb = to_csr(hints)
    so, sb = to_csr(seeds)
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), len(hints), 100_000_000,
                                            len(seeds), ctypes.byref(plan)))
    d_so = torch.from_numpy(so.view(np.int32)).cuda()
    d_sb = torch.from_numpy(sb).cuda()
    d_st = torch.empty(len(seeds) * 32, dtype=torch.uint8, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(L.nmz_replayable_sweep_dev(plan, ctypes.c_void_p(d_so.data_ptr()), ctypes.c_void_p(d_sb.data_ptr()),
                                          len(seeds), ctypes.c_void_p(d_st.data_ptr()), stream))
    d_tk = torch.empty(16 * 24, dtype=torch.uint8, device="cuda")
    _lib.check(L.nmz_topk_select_dev(ctx.handle, ctypes.c_void_p(d_st.data_ptr()), len(seeds), 0, 16,
                                     ctypes.c_void_p(d_tk.data_ptr()), stream))
    torch.cuda.synchronize()
    got = np.frombuffer(d_st.cpu().numpy().tobytes(), dtype=_lib.SCHED_STATS_DTYPE)
    st, _ = rep_oracle(seeds, hints, 100_000_000)
    assert np.array_equal(got, st)
    tk = np.frombuffer(d_tk.cpu().numpy().tobytes(), dtype=_lib.TOPK_DTYPE)
    assert np.array_equal(tk, O.topk_from_stats(st, 0, 16))
    # more seeds than planned -> error, not a fault
    rc = L.nmz_replayable_sweep_dev(plan, ctypes.c_void_p(d_so.data_ptr()), ctypes.c_void_p(d_sb.data_ptr()),
                                    len(seeds) + 1, ctypes.c_void_p(d_st.data_ptr()), stream)
    assert rc == _lib.NMZ_EINVAL
    L.nmz_replayable_plan_destroy(plan)


@pytest.mark.parametrize("E,m,k", [(4096, 100_000_000, 64), (512, 2**31 + 3, 17), (1000, 1000, 64)])
def test_replayable_topk_large_sweep(ctx, E, m, k):
    """The wavelet-tree sweep's own top-k at 2^18 decimal seeds (thousands of workgroups: tau from sampled group
    maxima, candidates ranked by counting) == the top-k of the same sweep's stats."""
    import torch
    L = _lib.load()
    S = 1 << 18
    ho, hb = to_csr(zk_hints(E, np.random.default_rng(E)))
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), E, m, S, ctypes.byref(plan)))
    d_st = torch.zeros(S * 32, dtype=torch.uint8, device="cuda")
    d_tk = torch.zeros(k * 24, dtype=torch.uint8, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(L.nmz_replayable_sweep_decimal_topk_dev(plan, 10**12, S, k, ctypes.c_void_p(d_st.data_ptr()),
                                                       ctypes.c_void_p(d_tk.data_ptr()), stream))
    torch.cuda.synchronize()
    L.nmz_replayable_plan_destroy(plan)
    st = np.frombuffer(d_st.cpu().numpy().tobytes(), dtype=_lib.SCHED_STATS_DTYPE)
    tk = np.frombuffer(d_tk.cpu().numpy().tobytes(), dtype=_lib.TOPK_DTYPE)
    assert tk.tolist() == O.topk_from_stats(st, 10**12, k).tolist()


@pytest.mark.parametrize("lo,S", [(0, 1 << 17), (3, 5000), (95, 1 << 17), (9_999_950, 1 << 17),
                                  (10**12 + 37, 1 << 17), (2**64 - (1 << 17) - 250, 1 << 17),
                                  (2**64 - 1000, 1 << 13), (123_400, 1_638_350)])
def test_decimal_sweep_at_scale(ctx, lo, S):
    """Decimal seed ranges (device-generated strings) of 5,000 to 1.6 M seeds: the bucketing's per-block count rows
    (up to 800), their column scans and the scatter, vs the oracle over the decimal strings (wrapping past 2^64;
    the largest case on its first 32,768 seeds), twice through one plan (nothing left from the first sweep); the
    sweep's top-64 == the top-64 of its stats."""
    import torch
    L = _lib.load()
    E, m, k = 512, 100_000_000, 64
    hints = zk_hints(E, np.random.default_rng(lo % 1000 + S))
    ho, hb = to_csr(hints)
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), E, m, S, ctypes.byref(plan)))
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    d_st = torch.zeros(S * 32, dtype=torch.uint8, device="cuda")
    d_tk = torch.zeros(k * 24, dtype=torch.uint8, device="cuda")
    for _ in range(2):
        _lib.check(L.nmz_replayable_sweep_decimal_topk_dev(plan, lo, S, k, ctypes.c_void_p(d_st.data_ptr()),
                                                           ctypes.c_void_p(d_tk.data_ptr()), stream))
    torch.cuda.synchronize()
    L.nmz_replayable_plan_destroy(plan)
    st = np.frombuffer(d_st.cpu().numpy().tobytes(), dtype=_lib.SCHED_STATS_DTYPE)
    n_or = S if S <= (1 << 17) else 1 << 15
    ost, _ = rep_oracle([str((lo + i) % 2**64) for i in range(n_or)], hints, m)
    assert st[:n_or].tobytes() == ost.tobytes()
    tk = np.frombuffer(d_tk.cpu().numpy().tobytes(), dtype=_lib.TOPK_DTYPE)
    assert tk.tolist() == O.topk_from_stats(st, lo, k).tolist()


@pytest.mark.parametrize("kind", ["csr", "decimal"])
def test_replayable_seed_set(ab_knobs, ctx, monkeypatch, kind):
    """nmz_replayable_sweep_seeds_topk_dev over one prepared seed set (prefix hashes bucketed once) == the plain
    sweep of the same seeds, on every statistics path: wavelet trees (fused and separate plan builds), order
    queries, and the per-decision sweeps (maxInterval >= 2^32: the prepared hashes bucketed per sweep), stats and
    top-k, with several plans sweeping the one set; more seeds than a plan was created for take the set's buckets."""
    import torch
    L = _lib.load()
    S, k = 3000, 16
    seeds = [str(i * 7) for i in range(S)] if kind == "csr" else None
    d_so = d_sb = None
    if kind == "csr":
        so, sb = to_csr(seeds)
        d_so = torch.from_numpy(so.view(np.int32)).cuda()
        d_sb = torch.from_numpy(sb).cuda()
    dec_lo = 10**9
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ss = ctypes.c_void_p()
    _lib.check(L.nmz_replayable_seeds_create(ctx.handle, ctypes.c_void_p(d_so.data_ptr() if d_so is not None else 0),
                                             ctypes.c_void_p(d_sb.data_ptr() if d_sb is not None else 0), S, dec_lo,
                                             ctypes.byref(ss)))
    try:
        cases = [("wt", 100_000_000, S), ("wt_sep", 100_000_000, S), ("oq", 7, S), ("fast", 2**32 + 5, S),
                 ("wt", 2**31 + 3, 1000)]
        for path, m, max_seeds in cases:
            monkeypatch.delenv("NMZ_REPLAY_WT", raising=False)
            monkeypatch.delenv("NMZ_WT_FUSED", raising=False)
            if path == "oq":
                monkeypatch.setenv("NMZ_REPLAY_WT", "0")
            if path == "wt_sep":
                monkeypatch.setenv("NMZ_WT_FUSED", "0")
            hints = zk_hints(257)
            ho, hb = to_csr(hints)
            plan = ctypes.c_void_p()
            _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), len(hints), m, max_seeds,
                                                    ctypes.byref(plan)))
            outs = []
            for use_set in ((True, False) if max_seeds >= S else (True,)):
                d_st = torch.zeros(S * 32, dtype=torch.uint8, device="cuda")
                d_tk = torch.zeros(k * 24, dtype=torch.uint8, device="cuda")
                if use_set:
                    _lib.check(L.nmz_replayable_sweep_seeds_topk_dev(plan, ss, 5, k, ctypes.c_void_p(d_st.data_ptr()),
                                                                     ctypes.c_void_p(d_tk.data_ptr()), stream))
                elif kind == "csr":
                    _lib.check(L.nmz_replayable_sweep_topk_dev(plan, ctypes.c_void_p(d_so.data_ptr()),
                                                               ctypes.c_void_p(d_sb.data_ptr()), S, 5, k,
                                                               ctypes.c_void_p(d_st.data_ptr()),
                                                               ctypes.c_void_p(d_tk.data_ptr()), stream))
                else:
                    _lib.check(L.nmz_replayable_sweep_decimal_topk_dev(plan, dec_lo, S, k,
                                                                       ctypes.c_void_p(d_st.data_ptr()),
                                                                       ctypes.c_void_p(d_tk.data_ptr()), stream))
                torch.cuda.synchronize()
                outs.append((d_st.cpu().numpy().copy(), d_tk.cpu().numpy().copy()))
            L.nmz_replayable_plan_destroy(plan)
            if len(outs) == 2:
                assert np.array_equal(outs[0][0], outs[1][0]), (path, m)
                if kind == "csr":  # the decimal sweep numbers its top-k seeds from dec_lo, the set's from seed0
                    assert np.array_equal(outs[0][1], outs[1][1]), (path, m)
            st = np.frombuffer(outs[0][0].tobytes(), dtype=_lib.SCHED_STATS_DTYPE)
            tk = np.frombuffer(outs[0][1].tobytes(), dtype=_lib.TOPK_DTYPE)
            assert tk.tolist() == O.topk_from_stats(st, 5, k).tolist()
            if kind == "csr" and path in ("wt", "oq", "fast"):
                ref, _ = rep_oracle(seeds, hints, m)
                assert np.array_equal(st, ref)
    finally:
        L.nmz_replayable_seeds_destroy(ss)


@pytest.mark.parametrize("m", [100_000_000, 2**31 + 3, 2**32 + 7])
def test_replayable_sweep_traces(ctx, m):
    """nmz_replayable_sweep_traces (a batch of traces over one decimal seed range, pipelined inside) == one
    nmz_replayable_sweep_decimal_topk_dev per trace on its own plan, for traces of several shapes (one-launch
    wavelet-tree plans, a 4,097-event class on the separate plan kernels, tiny traces); the top-k of a small
    trace also vs the oracle."""
    import torch
    L = _lib.load()
    rng = np.random.default_rng(m % 1000)
    traces = [zk_hints(600, rng), zk_hints(97, rng) + ["", "a"], ["x" * 5] * 4097, zk_hints(3, rng),
              zk_hints(2000, rng), zk_hints(64, rng), zk_hints(1, rng)]
    T, S, k, lo = len(traces), 2500, 16, 77
    csrs = [to_csr(h) for h in traces]
    offs = (ctypes.c_void_p * T)(*[ctypes.c_void_p(ho.ctypes.data) for ho, _ in csrs])
    byts = (ctypes.c_void_p * T)(*[ctypes.c_void_p(hb.ctypes.data) for _, hb in csrs])
    nev = np.array([len(h) for h in traces], np.uint32)
    out = np.zeros(T * k, _lib.TOPK_DTYPE)
    for rep in range(2):  # the second call reuses the pipeline's streams, helper context and pooled buffers
        _lib.check(L.nmz_replayable_sweep_traces(ctx.handle, T, offs, byts, _lib.ptr(nev), m, lo, S, k,
                                                 _lib.ptr(out)))
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for t, (ho, hb) in enumerate(csrs):
            plan = ctypes.c_void_p()
            _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), len(traces[t]), m, S,
                                                    ctypes.byref(plan)))
            d_st = torch.zeros(S * 32, dtype=torch.uint8, device="cuda")
            d_tk = torch.zeros(k * 24, dtype=torch.uint8, device="cuda")
            _lib.check(L.nmz_replayable_sweep_decimal_topk_dev(plan, lo, S, k, ctypes.c_void_p(d_st.data_ptr()),
                                                               ctypes.c_void_p(d_tk.data_ptr()), stream))
            torch.cuda.synchronize()
            L.nmz_replayable_plan_destroy(plan)
            ref = np.frombuffer(d_tk.cpu().numpy().tobytes(), dtype=_lib.TOPK_DTYPE)
            assert out[t * k:(t + 1) * k].tolist() == ref.tolist(), (rep, t)
    seeds = [str(lo + i) for i in range(S)]
    st, _ = rep_oracle(seeds, traces[3], m)
    assert out[3 * k:4 * k].tolist() == O.topk_from_stats(st, lo, k).tolist()


def test_replayable_plan_create_async(ctx):
    """nmz_replayable_plan_create_async: builds enqueued on two contexts' streams, sweeps enqueued at once on
    another stream (which must wait for each build on the device), plans of several shapes (the one-launch
    wavelet-tree build, a class of 4,096 events: the separate kernels, maxInterval >= 2^32: per-decision), the
    staging reused by the next build before the previous one ran, and a plan destroyed with its build in flight."""
    import torch
    L = _lib.load()
    ctx2 = _lib.Context(0)
    try:
        S = 2500
        seeds = [str(i * 31) for i in range(S)]
        so, sb = to_csr(seeds)
        d_so = torch.from_numpy(so.view(np.int32)).cuda()
        d_sb = torch.from_numpy(sb).cuda()
        cases = [(zk_hints(600), 100_000_000), (zk_hints(97) + ["", "a"], 7), (["x" * 5] * 4097, 100_000_000),
                 (zk_hints(300), 2**32 + 5), (zk_hints(2000), 2**31 + 3), (zk_hints(64), 1_000_000)]
        st = torch.cuda.Stream()
        plans, outs = [], []
        for i, (hints, m) in enumerate(cases):
            ho, hb = to_csr(hints)
            p = ctypes.c_void_p()
            _lib.check(L.nmz_replayable_plan_create_async((ctx, ctx2)[i % 2].handle, _lib.ptr(ho), _lib.ptr(hb),
                                                          len(hints), m, S, ctypes.byref(p)))
            del ho, hb  # the host arrays may go at once
            d_st = torch.zeros(S * 32, dtype=torch.uint8, device="cuda")
            d_tk = torch.zeros(16 * 24, dtype=torch.uint8, device="cuda")
            with torch.cuda.stream(st):
                _lib.check(L.nmz_replayable_sweep_topk_dev(p, ctypes.c_void_p(d_so.data_ptr()),
                                                           ctypes.c_void_p(d_sb.data_ptr()), S, 0, 16,
                                                           ctypes.c_void_p(d_st.data_ptr()),
                                                           ctypes.c_void_p(d_tk.data_ptr()),
                                                           ctypes.c_void_p(st.cuda_stream)))
            plans.append(p)
            outs.append((d_st, d_tk))
        for p in plans:
            L.nmz_replayable_plan_destroy(p)  # waits for its build and its sweep
        for (hints, m), (d_st, d_tk) in zip(cases, outs):
            got = np.frombuffer(d_st.cpu().numpy().tobytes(), dtype=_lib.SCHED_STATS_DTYPE)
            ref, _ = rep_oracle(seeds, hints, m)
            assert np.array_equal(got, ref), m
            tk = np.frombuffer(d_tk.cpu().numpy().tobytes(), dtype=_lib.TOPK_DTYPE)
            assert tk.tolist() == O.topk_from_stats(ref, 0, 16).tolist()
        # destroyed while its build may still run
        ho, hb = to_csr(zk_hints(3000))
        p = ctypes.c_void_p()
        _lib.check(L.nmz_replayable_plan_create_async(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), 3000, 100_000_000, S,
                                                      ctypes.byref(p)))
        L.nmz_replayable_plan_destroy(p)
    finally:
        ctx2.close()


@pytest.mark.parametrize("m,S,E,k,seed0", [
    (100_000_000, 5000, 300, 64, 0),          # MOD_FAST: top-k fused into the merge, 3 lists
    (100_000_000, 1500, 64, 100, 7),          # k not a power of two (LDS list-merge path)
    (100_000_000, 200, 40, 16, 2**64 - 50),   # one list; seeds wrap past 2^64
    (3_000_000_000, 2500, 50, 32, 5),         # MOD_GENERAL: separate selection
    (0, 700, 20, 8, 0),                       # maxInterval 0: constant stats, all ties
    (1_000_000, 0, 20, 8, 0),                 # no seeds: sentinels
    # wavelet-tree sweeps with their own top-k candidates (k <= 64, > 2,048 seeds):
    (100_000_000, 9000, 120, 64, 2**64 - 4000),  # candidates above the k-th workgroup maximum; seeds wrap
    (7, 6000, 100, 33, 3),                    # sums 0..600: heavy ties, candidates overflow -> gated selection
    (1, 5000, 40, 16, 11),                    # maxInterval 1: every sum 0, every seed a candidate -> gated
    (1, 3000, 40, 64, 2**64 - 1500),          # 3,000 tied candidates: two sorted chunks, then their best 64 each
    (1, 4096, 30, 5, 9),                      # exactly WT_CAND candidates: the last chunk full
    (2**31 + 3, 4000, 60, 1, 0),              # k = 1, m >= 2^31
])
def test_replayable_sweep_topk_dev_matches_separate_selection(ctx, m, S, E, k, seed0):
    """nmz_replayable_sweep_topk_dev (its own top-k path per kernel: on the wavelet-tree path the candidates above
    the k-th workgroup maximum, ranked by counting, or the gated general selection when they overflow) == the
    oracle's top-k of the oracle's stats."""
    import torch
    L = _lib.load()
    hints = zk_hints(E)
    seeds = [str(i * 7919) for i in range(S)]
    ho, hb = to_csr(hints)
    so, sb = to_csr(seeds)
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), E, m, max(S, 1),
                                            ctypes.byref(plan)))
    d_so = torch.from_numpy(so.view(np.int32)).cuda()
    d_sb = torch.from_numpy(sb).cuda()
    d_st = torch.zeros(max(S, 1) * 32, dtype=torch.uint8, device="cuda")
    d_tk = torch.zeros(k * 24, dtype=torch.uint8, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(L.nmz_replayable_sweep_topk_dev(plan, ctypes.c_void_p(d_so.data_ptr()),
                                               ctypes.c_void_p(d_sb.data_ptr()), S, seed0, k,
                                               ctypes.c_void_p(d_st.data_ptr()), ctypes.c_void_p(d_tk.data_ptr()),
                                               stream))
    torch.cuda.synchronize()
    L.nmz_replayable_plan_destroy(plan)
    got = np.frombuffer(d_st.cpu().numpy().tobytes(), dtype=_lib.SCHED_STATS_DTYPE)[:S]
    tk = np.frombuffer(d_tk.cpu().numpy().tobytes(), dtype=_lib.TOPK_DTYPE)
    st, _ = rep_oracle(seeds, hints, m) if S else (np.zeros(0, O.SCHED_STATS_DTYPE), None)
    assert np.array_equal(got, st)
    assert tk.tolist() == O.topk_from_stats(st, seed0, k).tolist()


# ---------------------------------------------------------------- K2
PARAMS = [(30_000_000, 100_000_000, 0.1), (5_000_000, 5_000_000, 0.5), (0, 1 << 20, 1.0),
          (80_000_000, 3_000_000_000, 0.999), (0, 0, 0.0), (-5_000_000, 5_000_000, 0.3), (7, 9, 0.25),
          (1, 1 + (1 << 40), 0.05), (0, (1 << 31) - 1, 0.2), (0, (1 << 31) + 1, 0.2), (3, 3 + (1 << 31), 0.7),
          # the edge of k_random_sweep's 32-bit f64-key form (every delay < 0x7ff00000) and one past it
          (0, 0x7ff00000, 0.2), (0, 0x7ff00001, 0.2), (0x7fe00000, 0x7ff00000, 0.4)]


@pytest.mark.parametrize("mn,mx,p", PARAMS)
def test_random_params_grid(ctx, mn, mx, p):
    E = 301
    eh = RNG.integers(0, 2**64, size=E, dtype=np.uint64)
    ec = RNG.integers(0, 4, size=E, dtype=np.uint8)
    rp = Random()
    rp.MinInterval, rp.MaxInterval, rp.FaultActionProbability = mn, mx, p
    seed0 = int(RNG.integers(0, 2**63))
    r = rp.Sweep(seed0, 600, eh, ec, n_dump=12, k=20, ctx=ctx)
    st, dl, fl = O.random_sweep(seed0, 600, eh, ec, O.random_params(mn, mx, p), n_dump=12)
    assert np.array_equal(r.stats, st)
    assert np.array_equal(r.delays, dl) and np.array_equal(r.faults, fl)
    assert np.array_equal(r.topk, O.topk_from_stats(st, seed0, 20))


def test_random_golden_decisions(ctx, golden):
    rp = Random()
    for rec in golden("random_decisions.json")["decisions"]:
        rp.MinInterval, rp.MaxInterval, rp.FaultActionProbability = rec["min_ns"], rec["max_ns"], rec["p"]
        r = rp.Sweep(rec["seed"], 1, np.array([rec["evhash"]], np.uint64), np.array([rec["evclass"]], np.uint8),
                     n_dump=1, ctx=ctx)
        assert int(r.delays[0, 0]) == rec["delay_ns"]
        assert bool(r.faults[0, 0]) == rec["fault"]


def test_random_rejection_path(ctx):
    """Force Go rejection re-draws: Int63n with n just above 2^62 rejects ~half the draws,
    so many decisions take the general closed-form path (outputs t >= 2)."""
    E = 64
    eh = RNG.integers(0, 2**64, size=E, dtype=np.uint64)
    ec = np.full(E, 2, np.uint8)  # faultable, not prioritized
    rp = Random()
    rp.MinInterval, rp.MaxInterval, rp.FaultActionProbability = 0, (1 << 62) + 1, 0.5
    r = rp.Sweep(11, 500, eh, ec, n_dump=500, ctx=ctx)
    st, dl, fl = O.random_sweep(11, 500, eh, ec, O.random_params(0, (1 << 62) + 1, 0.5), n_dump=500)
    assert np.array_equal(r.stats, st) and np.array_equal(r.delays, dl) and np.array_equal(r.faults, fl)
    # check rejection actually happened in the inputs
    nouts = [O.random_decide(11 + s, int(eh[e]), 2, O.random_params(0, (1 << 62) + 1, 0.5))[2]
             for s in range(20) for e in range(E)]
    assert max(nouts) >= 3


@pytest.mark.parametrize("kind,mn,mx", [("ranged", 30_000_000, 100_000_000),   # K32 sweep form
                                         ("ranged", 0, 3_000_000_000),          # 64-bit max form
                                         ("fixed", 5_000_000, 5_000_000),       # K32, no delay draw
                                         ("fixed", 3_000_000_000, 3_000_000_000)])
@pytest.mark.parametrize("p", [0.1, 0.3, 0.5, 0.7, 0.9])
def test_random_sweep_rejected_fault_draw(ctx, golden, kind, mn, mx, p):
    """decide_sweep's two rarely-taken re-draw branches (csrc/random.hip): a ranged delay accepted and the
    Intn(999) fault draw rejected (`slow |= v1 > INT31N_MAX`), and the fixed-duration class with a rejected fault
    draw (`slow = v > INT31N_MAX`). The vectors (tests/golden/random_rejections.json, searched with the oracle)
    force them; sweep path only (no dump, which goes through decide()), stats vs the oracle for every seed
    around the vectors' seed, both entity classes, several thresholds."""
    g = golden("random_rejections.json")
    hits = np.array(g[kind], np.uint64)
    fill = RNG.integers(0, 2**64, size=23, dtype=np.uint64)
    eh = np.concatenate([fill[:7], hits, fill[7:15], hits, fill[15:]])
    ec = np.full(len(eh), 2, np.uint8)
    ec[7 + len(hits) + 8:7 + 2 * len(hits) + 8] = 3  # second copy prioritized
    rp = Random()
    rp.MinInterval, rp.MaxInterval, rp.FaultActionProbability = mn, mx, p
    seed0 = g["seed"] - 100
    r = rp.Sweep(seed0, 201, eh, ec, k=8, ctx=ctx)
    st, _, _ = O.random_sweep(seed0, 201, eh, ec, O.random_params(mn, mx, p))
    assert np.array_equal(r.stats, st)
    assert np.array_equal(r.topk, O.topk_from_stats(st, seed0, 8))
    # the vectors do take the re-draw: the seed's decisions on them draw one more Go output than usual
    pr = O.random_params(mn, mx, p)
    assert all(O.random_decide(g["seed"], int(h), 2, pr)[2] == (3 if kind == "ranged" else 2) for h in hits)


def test_random_edge_cases(ctx):
    rp = Random()
    rp.MinInterval, rp.MaxInterval, rp.FaultActionProbability = 30_000_000, 100_000_000, 0.1
    r = rp.Sweep(0, 5, np.zeros(0, np.uint64), np.zeros(0, np.uint8), k=3, ctx=ctx)
    assert r.stats["argmax_event"].tolist() == [_lib.NMZ_NONE] * 5
    assert r.topk["seed"].tolist() == [0, 1, 2]
    with pytest.raises(_lib.NmzInvalidArgument):
        rp.Sweep(0, 5, np.zeros(2, np.uint64), np.array([4, 0], np.uint8), ctx=ctx)  # ProcSet-like class bit
    rp.MinInterval, rp.MaxInterval = 10, 5
    with pytest.raises(_lib.NmzInvalidArgument):
        rp.Sweep(0, 5, np.zeros(2, np.uint64), np.zeros(2, np.uint8), ctx=ctx)
    # seed range wrapping past 2^64
    rp.MinInterval, rp.MaxInterval = 1, 1000
    eh = RNG.integers(0, 2**64, size=50, dtype=np.uint64)
    ec = RNG.integers(0, 4, size=50, dtype=np.uint8)
    r = rp.Sweep(2**64 - 3, 7, eh, ec, ctx=ctx)
    st, _, _ = O.random_sweep(2**64 - 3, 7, eh, ec, O.random_params(1, 1000, 0.1))
    assert np.array_equal(r.stats, st)


@pytest.mark.parametrize("E,mn,mx,p", [(3000, 30_000_000, 100_000_000, 0.001), (2048, 5_000_000, 5_000_000, 0.002),
                                        (1025, 0, 1 << 20, 0.0), (4100, 7, 9, 0.0015)])
def test_random_event_chunks(ctx, E, mn, mx, p):
    """Traces longer than one work item (512 events): per-chunk partial stats merged in event order.
    Rare faults put first_fault in later chunks; fixed or 2-valued delays make argmax ties across chunks."""
    eh = RNG.integers(0, 2**64, size=E, dtype=np.uint64)
    ec = RNG.integers(0, 4, size=E, dtype=np.uint8)
    rp = Random()
    rp.MinInterval, rp.MaxInterval, rp.FaultActionProbability = mn, mx, p
    seed0 = int(RNG.integers(0, 2**63))
    r = rp.Sweep(seed0, 1500, eh, ec, k=16, ctx=ctx)
    st, _, _ = O.random_sweep(seed0, 1500, eh, ec, O.random_params(mn, mx, p))
    assert np.array_equal(r.stats, st)
    assert np.array_equal(r.topk, O.topk_from_stats(st, seed0, 16))
    if p:
        assert (st["first_fault"][st["n_fault"] > 0] >= 1024).any()


# ---------------------------------------------------------------- top-k
def _topk_dev(ctx, st, seed0, k):
    import torch
    L = _lib.load()
    d_st = torch.from_numpy(np.frombuffer(st.tobytes(), np.uint8).copy()).cuda()
    d_tk = torch.empty(max(k, 1) * 24, dtype=torch.uint8, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(L.nmz_topk_select_dev(ctx.handle, ctypes.c_void_p(d_st.data_ptr()), len(st), seed0, k,
                                     ctypes.c_void_p(d_tk.data_ptr()), stream))
    torch.cuda.synchronize()
    return np.frombuffer(d_tk.cpu().numpy().tobytes(), dtype=_lib.TOPK_DTYPE)[:k]


@pytest.mark.parametrize("n,k,mode", [
    (1, 1, "rand"), (5, 16, "rand"), (2047, 64, "rand"), (2048, 256, "rand"), (2049, 1, "rand"),
    (300_001, 64, "rand"), (300_001, 256, "rand"), (100_000, 64, "ties"), (70_000, 64, "const"),
    (70_000, 128, "sorted"), (70_000, 64, "faults"), (90_001, 100, "neg"), (50_000, 37, "bigfault"),
    (3, 100, "neg"), (200_000, 256, "sorted")])
def test_topk_select_dev(ctx, n, k, mode):
    """Threshold-filter top-k + list-merge tree vs the oracle: random keys,
    heavy ties (every entry a survivor), ascending keys (worst case for
    per-thread winners), n_fault-dominated order, negative int64 sums, fault
    counts past the coarse key's 16-bit saturation, k not a power of two,
    sizes around the 2048-entry chunk."""
    rng = np.random.default_rng(n * 7 + k)
    st = np.zeros(n, O.SCHED_STATS_DTYPE)
    if mode == "rand":
        st["sum_delay_ns"] = rng.integers(0, 2**62, n, dtype=np.uint64)
    elif mode == "ties":
        st["sum_delay_ns"] = rng.integers(0, 4, n, dtype=np.uint64)
    elif mode == "const":
        st["sum_delay_ns"] = 77
    elif mode == "sorted":
        st["sum_delay_ns"] = np.arange(n, dtype=np.uint64)
    elif mode == "neg":
        st["sum_delay_ns"] = rng.integers(-2**63, 2**63, n, dtype=np.int64).view(np.uint64)
    elif mode == "bigfault":
        st["n_fault"] = rng.integers(65530, 65540, n, dtype=np.uint32)
        st["n_fault"][::97] = 2**32 - 1
        st["sum_delay_ns"] = rng.integers(0, 2**40, n, dtype=np.uint64)
    else:
        st["n_fault"] = rng.integers(0, 3, n, dtype=np.uint32)
        st["sum_delay_ns"] = rng.integers(0, 1000, n, dtype=np.uint64)
    st["first_fault"] = rng.integers(0, 2**32, n, dtype=np.uint32)
    got = _topk_dev(ctx, st, 12345, k)
    exp = O.topk_from_stats(st, 12345, k)
    assert got.tolist() == exp[:k].tolist()
