"""GPU parity: banded edit distance (K3 fast tile kernel and the generic
kernel), all-pairs k-NN, storage search and uniqueness, vs the CPU oracle."""
import ctypes

import numpy as np
import pytest

from namazu_amd import _lib
from namazu_amd import historystorage as hs
from oracle import oracle as O

pytestmark = pytest.mark.gpu

RNG = np.random.default_rng(0xED)


def make_traces(n, lmin, lmax, mut, alphabet=12, rng=RNG):
    base = rng.integers(0, alphabet, size=max(lmax, 1))
    out = []
    for _ in range(n):
        l = int(rng.integers(lmin, lmax + 1))
        t = base[:l].copy()
        m = rng.random(l) < mut
        t[m] = rng.integers(0, alphabet, size=int(m.sum()))
        out.append(t.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(3))
    return hs.TraceSet(out)


def knn(ctx, ts, w, k):
    return hs.allpairs_knn(ts, k, w, ctx=ctx)


@pytest.mark.parametrize("n,lmin,lmax,w,mut,k", [
    (70, 0, 40, 8, 0.3, 6), (150, 180, 260, 32, 0.05, 8), (130, 100, 300, 16, 0.02, 5),
    (97, 1, 70, 32, 0.5, 4), (65, 30, 30, 32, 0.0, 3), (200, 50, 90, 32, 0.1, 64),
    (3, 5, 9, 32, 0.2, 8), (2, 0, 0, 8, 0.0, 1), (128, 500, 520, 8, 0.01, 2)])
def test_knn_fast_kernel(ctx, n, lmin, lmax, w, mut, k):
    ts = make_traces(n, lmin, lmax, mut)
    ids, ds = knn(ctx, ts, w, k)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, k)
    assert np.array_equal(ids, oi) and np.array_equal(ds, od)


@pytest.mark.parametrize("pool", [256, 2048, 4096])
def test_knn_bv_pool_sizes(ab_knobs, ctx, monkeypatch, pool):
    """k_ed_bv workgroups own pools of 256..4096 candidates (the plan picks 4096 for N >= 24576);
    forced here on a smaller N with short ragged traces, vs the oracle."""
    monkeypatch.setenv("NMZ_ED_POOL", str(pool))
    ts = make_traces(1500, 100, 200, 0.04, alphabet=20, rng=np.random.default_rng(pool))
    ids, ds = knn(ctx, ts, 32, 8)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, 32, 8, nthreads=16)
    assert np.array_equal(ids, oi) and np.array_equal(ds, od)


@pytest.mark.parametrize("w", [0, 1, 5, 31, 33, 100, 9000])
def test_knn_any_band_short_traces(ctx, w):
    """Short and empty traces at bands the kernels' template W does not equal (bit-parallel W >= w for w <= 64,
    wide for 64 < w <= 8192, generic beyond)."""
    ts = make_traces(60, 0, 60, 0.2)
    ids, ds = knn(ctx, ts, w, 5)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, 5)
    assert np.array_equal(ids, oi) and np.array_equal(ds, od)


def _plan_kind(ctx, ts, w):
    L = _lib.load()
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_ed_plan_create(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), len(ts), w, ctypes.byref(plan)))
    kind = L.nmz_ed_plan_is_fast(plan)
    L.nmz_ed_plan_destroy(plan)
    return kind


@pytest.mark.parametrize("w,n,lmin,lmax,mut,kind", [
    (1, 200, 100, 110, 0.004, 2), (5, 200, 100, 120, 0.02, 2), (20, 200, 150, 250, 0.05, 2),
    (33, 150, 200, 300, 0.08, 2), (50, 150, 300, 420, 0.1, 2), (64, 120, 300, 400, 0.12, 2),
    (100, 12, 600, 650, 0.08, 3), (700, 10, 1900, 2100, 0.2, 3), (1500, 8, 3800, 4200, 0.2, 3)])
def test_knn_band_routing(ctx, w, n, lmin, lmax, mut, kind):
    """Every band reaches a fast kernel: w <= 64 the bit-parallel kernels of the smallest W in {8, 16, 32, 64}
    >= w, 64 < w <= 8192 the wide kernel of the smallest W = 1024 * 2^k >= w, each with w applied at run time
    (length band, q-gram bound, cut-off, clamp at w + 1). Mutation rates put distances on both sides of w."""
    ts = make_traces(n, lmin, lmax, mut, alphabet=16, rng=np.random.default_rng(w * 31 + n))
    assert _plan_kind(ctx, ts, w) == kind
    k = min(6, n - 1)
    ids, ds = knn(ctx, ts, w, k)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, k, nthreads=16)
    assert np.array_equal(ids, oi) and np.array_equal(ds, od)
    assert (od <= w).any() and (od == w + 1).any()  # both sides of the band were exercised


def test_knn_large_alphabet_falls_back(ctx):
    """> 65533 distinct symbols -> exact generic path."""
    rng = np.random.default_rng(5)
    trs = [rng.integers(0, 2**64, size=700, dtype=np.uint64) for _ in range(100)]
    trs[7] = trs[3].copy()
    ts = hs.TraceSet(trs)
    ids, ds = knn(ctx, ts, 32, 2)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, 32, 2)
    assert np.array_equal(ids, oi) and np.array_equal(ds, od)
    assert ds[7][0] == 0 and ids[7][0] == 3


def test_ed_pairs(ctx):
    ts = make_traces(50, 0, 120, 0.1)
    pairs = RNG.integers(0, 50, size=(2000, 2)).astype(np.uint32)
    for w in [0, 3, 8, 32, 200]:
        assert np.array_equal(hs.ed_pairs(ts, pairs, w, ctx=ctx), O.ed_pairs(ts.off, ts.sym, pairs, w))


def test_ed_kat(ctx, golden):
    pairs = golden("ed_kat.json")["pairs"]
    ts = hs.TraceSet([np.frombuffer(p[k].encode(), np.uint8).astype(np.uint64) for p in pairs for k in "ab"])
    idx = np.array([[2 * i, 2 * i + 1] for i in range(len(pairs))], np.uint32)
    d = hs.ed_pairs(ts, idx, 32, ctx=ctx)
    assert d.tolist() == [p["d"] for p in pairs]


def test_zk_traces_golden(ctx, golden):
    z = golden("zk_traces.json")
    ts = hs.TraceSet([np.array([int(h, 16) for h in t["evhash"]], np.uint64) for t in z["traces"]])
    n = len(ts)
    pairs = np.array([[i, j] for i in range(n) for j in range(n)], np.uint32)
    for w, mat in z["banded"].items():
        d = hs.ed_pairs(ts, pairs, int(w), ctx=ctx).reshape(n, n)
        assert d.tolist() == mat
    d = hs.ed_pairs(ts, pairs, 64, ctx=ctx).reshape(n, n)
    assert d.tolist() == z["levenshtein"]
    for w in (8, 32):
        ids, ds = knn(ctx, ts, w, 3)
        oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, 3)
        assert np.array_equal(ids, oi) and np.array_equal(ds, od)


def test_distance_zero_iff_equal(ctx):
    ts = make_traces(80, 10, 40, 0.3, alphabet=3)
    pairs = np.array([[i, j] for i in range(80) for j in range(80)], np.uint32)
    d = hs.ed_pairs(ts, pairs, 8, ctx=ctx).reshape(80, 80)
    for i in range(80):
        for j in range(80):
            assert (d[i, j] == 0) == np.array_equal(ts.trace(i), ts.trace(j))


def test_unique_curve_and_search(ctx, tmp_path):
    from namazu_amd.signal import Event
    from tests.test_host import _make_storage
    evs = [Event.packet(f"entity-{i % 3}", "a", "b", {"n": i}) for i in range(8)]
    runs = [evs[:4], evs[1:6], evs[:4], evs[2:8], evs[1:6], evs[:3]]
    _make_storage(str(tmp_path), runs)
    st = hs.LoadStorage(str(tmp_path))
    ts = st.load_all()
    assert hs.unique_trace_curve(ts, ctx=ctx) == [1, 2, 2, 3, 3, 4]
    t0, _ = st.GetStoredHistory(0)
    # latest trace (id 5) is excluded, as in naive.go:238
    assert st.Search(t0) == [0, 2]
    assert st.SearchWithConverter(hs.SingleTrace(t0.symbols[:3]), lambda t: hs.SingleTrace(t.symbols[:3])) == [0, 2]
    near = st.SearchSimilar(t0, 3, 8)
    assert near[0] == (0, 0) and near[1] == (2, 0)


def test_knn_device_plan_api(ctx):
    import torch
    L = _lib.load()
    ts = make_traces(300, 150, 200, 0.03)
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_ed_plan_create(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), len(ts), 32, ctypes.byref(plan)))
    assert L.nmz_ed_plan_is_fast(plan) == 2  # bit-parallel kernel
    k = 8
    d_keys = torch.empty(len(ts) * k, dtype=torch.int64, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(L.nmz_ed_allpairs_knn_dev(plan, k, ctypes.c_void_p(d_keys.data_ptr()), stream))
    torch.cuda.synchronize()
    keys = d_keys.cpu().numpy().view(np.uint64).reshape(-1, k)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, 32, k)
    assert np.array_equal((keys >> np.uint64(32)).astype(np.uint32), od)
    assert np.array_equal((keys & np.uint64(0xFFFFFFFF)).astype(np.uint32), oi)
    L.nmz_ed_plan_destroy(plan)


@pytest.mark.parametrize("n,lmin,lmax,w,alphabet", [(300, 150, 200, 32, 12),     # host build (small store)
                                                   (700, 1500, 1600, 16, 40),   # device build (>= 2^20 symbols)
                                                   (40, 100, 300, 300, 12)])    # wide kernel (host build)
def test_knn_plan_from_device_symbols(ctx, n, lmin, lmax, w, alphabet):
    """nmz_ed_plan_create_dev (symbols already in HBM: the multi-GPU bench's all_gathered store) gives the same
    k-NN lists as the host-array plan and the oracle, on the device build and on the host builds (which copy the
    symbols back)."""
    import torch
    L = _lib.load()
    rng = np.random.default_rng(n + w)
    ts = make_traces(n, lmin, lmax, 0.03, alphabet=alphabet, rng=rng)
    d_sym = torch.from_numpy(ts.sym.view(np.int64)).to("cuda")
    torch.cuda.synchronize()
    k = 6
    out = []
    for dev in (True, False):
        plan = ctypes.c_void_p()
        if dev:
            _lib.check(L.nmz_ed_plan_create_dev(ctx.handle, _lib.ptr(ts.off), ctypes.c_void_p(d_sym.data_ptr()),
                                                len(ts), w, ctypes.byref(plan)))
        else:
            _lib.check(L.nmz_ed_plan_create(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), len(ts), w,
                                            ctypes.byref(plan)))
        d_keys = torch.empty(len(ts) * k, dtype=torch.int64, device="cuda")
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(L.nmz_ed_allpairs_knn_dev(plan, k, ctypes.c_void_p(d_keys.data_ptr()), stream))
        torch.cuda.synchronize()
        out.append(d_keys.cpu().numpy().view(np.uint64).reshape(-1, k))
        L.nmz_ed_plan_destroy(plan)
    assert np.array_equal(out[0], out[1])
    if n <= 300:
        oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, k)
        assert np.array_equal((out[0] >> np.uint64(32)).astype(np.uint32), od)
        assert np.array_equal((out[0] & np.uint64(0xFFFFFFFF)).astype(np.uint32), oi)


def test_knn_config3_shape_sampled(ctx):
    """configs[2] trace shape (L = 2048, w = 32, k = 8, ZK-style mutations) at
    N = 2048: sampled brute-force parity for a few queries."""
    from namazu_amd.synth import synth_traces
    ts = synth_traces(2048, 2048, seed=7)
    ids, ds = knn(ctx, ts, 32, 8)
    for q in [0, 1, 777, 2047]:
        pairs = np.array([[q, c] for c in range(len(ts)) if c != q], np.uint32)
        d = O.ed_pairs(ts.off, ts.sym, pairs, 32, nthreads=8)
        order = np.lexsort((pairs[:, 1], d))[:8]
        assert ds[q].tolist() == d[order].tolist()
        assert ids[q].tolist() == pairs[order, 1].tolist()


@pytest.mark.parametrize("w", [8, 16, 32])
def test_knn_tile_kernel_mid_alphabet(ctx, w):
    """Alphabet too large for the bit-parallel LDS tables -> packed-u16 tile kernel."""
    ts = make_traces(150, 280, 400, 0.03, alphabet=3000, rng=np.random.default_rng(w))
    from namazu_amd import _lib as L
    plan = ctypes.c_void_p()
    L.check(L.load().nmz_ed_plan_create(ctx.handle, L.ptr(ts.off), L.ptr(ts.sym), len(ts), w, ctypes.byref(plan)))
    kind = L.load().nmz_ed_plan_is_fast(plan)
    L.load().nmz_ed_plan_destroy(plan)
    assert kind == 1
    ids, ds = knn(ctx, ts, w, 6)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, 6)
    assert np.array_equal(ids, oi) and np.array_equal(ds, od)


@pytest.mark.parametrize("n,lmin,lmax,w,mut,alphabet", [
    (300, 0, 300, 32, 0.02, 48), (257, 60, 64, 32, 0.0, 5), (200, 31, 97, 16, 0.04, 20),
    (129, 1, 40, 8, 0.1, 3), (190, 500, 560, 32, 0.01, 100)])
def test_knn_bitparallel_kernel(ctx, n, lmin, lmax, w, mut, alphabet):
    ts = make_traces(n, lmin, lmax, mut, alphabet=alphabet, rng=np.random.default_rng(n + w))
    from namazu_amd import _lib as L
    plan = ctypes.c_void_p()
    L.check(L.load().nmz_ed_plan_create(ctx.handle, L.ptr(ts.off), L.ptr(ts.sym), len(ts), w, ctypes.byref(plan)))
    kind = L.load().nmz_ed_plan_is_fast(plan)
    L.load().nmz_ed_plan_destroy(plan)
    assert kind == 2
    ids, ds = knn(ctx, ts, w, 8)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, 8)
    assert np.array_equal(ids, oi) and np.array_equal(ds, od)


def test_knn_config3_near_duplicates(ctx):
    """L = 2048, w = 32 with low mutation rates, so most distances land inside
    the band (exercises the end-of-trace extraction after 64 column blocks)."""
    from namazu_amd.synth import synth_traces
    ts = synth_traces(192, 2048, seed=11, p_transpose=0.002, p_subst=0.001)
    ids, ds = knn(ctx, ts, 32, 8)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, 32, 8, nthreads=16)
    assert np.array_equal(ids, oi) and np.array_equal(ds, od)
    assert (od[:, 0] <= 32).all()


@pytest.mark.parametrize("n,lmin,lmax,w,mut,alphabet", [
    (12, 2500, 2600, 1024, 0.05, 30),      # distances inside the band, ragged lengths
    (9, 1500, 3400, 1024, 0.02, 8),        # |n - m| > w for some pairs
    (10, 4000, 4100, 2048, 0.3, 20),       # distances past the band: cut-off path
    (7, 9000, 9050, 4096, 0.1, 64),        # configs[4] band, lengths not multiples of 32
    (5, 0, 40, 1024, 0.5, 4),              # short and empty traces
])
def test_knn_wide_kernel(ctx, n, lmin, lmax, w, mut, alphabet):
    ts = make_traces(n, lmin, lmax, mut, alphabet=alphabet, rng=np.random.default_rng(n * 7 + w))
    plan = ctypes.c_void_p()
    L = _lib.load()
    _lib.check(L.nmz_ed_plan_create(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), len(ts), w, ctypes.byref(plan)))
    kind = L.nmz_ed_plan_is_fast(plan)
    L.nmz_ed_plan_destroy(plan)
    assert kind == 3
    k = min(4, max(n - 1, 1))
    ids, ds = knn(ctx, ts, w, k)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, k, nthreads=16)
    assert np.array_equal(ids, oi) and np.array_equal(ds, od)


def test_knn_wide_etcd_shape(ctx):
    """configs[4] trace model (etcd-style, w = 4096) at 16k events, 6 traces."""
    from namazu_amd.synth import etcd_traces
    ts = etcd_traces(6, 16384, seed=3)
    ids, ds = knn(ctx, ts, 4096, 3)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, 4096, 3, nthreads=16)
    assert np.array_equal(ids, oi) and np.array_equal(ds, od)
    assert (od[:, 0] < 4096).all()


@pytest.mark.parametrize("w,alphabet,lmin,lmax,n,kind", [
    (32, 20, 150, 260, 400, 2),     # k_ed_bv
    (16, 3000, 300, 400, 200, 1),   # k_ed_tile (a query pair's symbols exceed the compact tables)
    (1024, 16, 1500, 1700, 12, 3),  # k_ed_wide
    (9000, 12, 10, 60, 90, 0),      # k_ed_generic (beyond the wide kernels)
])
def test_knn_shards_merge_to_full(ctx, w, alphabet, lmin, lmax, n, kind):
    """The multi-GPU path on one device: shard s of 3 into separate partial lists,
    merged by nmz_knn_merge_dev and completed by nmz_ed_knn_fill_dev, equals the oracle's all-pairs k-NN
    (the bit-parallel shards list in-band pairs only; the fill leaves the other kernels' complete lists as they are)."""
    import torch
    L = _lib.load()
    ts = make_traces(n, lmin, lmax, 0.05, alphabet=alphabet, rng=np.random.default_rng(w + n))
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_ed_plan_create(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), n, w, ctypes.byref(plan)))
    assert L.nmz_ed_plan_is_fast(plan) == kind
    k, S = 6, 3
    parts = torch.empty(S * n * k, dtype=torch.int64, device="cuda")
    out = torch.empty(n * k, dtype=torch.int64, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for s in range(S):
        _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, s, S, ctypes.c_void_p(parts.data_ptr() + s * n * k * 8),
                                                   stream))
    _lib.check(L.nmz_knn_merge_dev(ctx.handle, ctypes.c_void_p(parts.data_ptr()), S, n, k,
                                   ctypes.c_void_p(out.data_ptr()), stream))
    _lib.check(L.nmz_ed_knn_fill_dev(plan, k, ctypes.c_void_p(out.data_ptr()), stream))
    torch.cuda.synchronize()
    L.nmz_ed_plan_destroy(plan)
    keys = out.cpu().numpy().view(np.uint64).reshape(n, k)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, k, nthreads=16)
    assert np.array_equal((keys >> np.uint64(32)).astype(np.uint32), od)
    assert np.array_equal((keys & np.uint64(0xFFFFFFFF)).astype(np.uint32), oi)


@pytest.mark.parametrize("w,n,lmin,lmax,mut,alphabet,k", [
    (32, 500, 100, 300, 0.03, 20, 8),     # ragged, most pairs in band
    (16, 300, 0, 80, 0.2, 6, 5),          # short/empty traces, |n - m| > w
    (8, 1200, 50, 60, 0.05, 40, 64),      # k = 64
    (32, 100, 200, 200, 0.01, 48, 8),     # equal lengths, near duplicates
])
def test_similarity_index_queries_vs_oracle(ctx, w, n, lmin, lmax, mut, alphabet, k):
    """SearchSimilar's resident store (nmz_ed_plan_query_knn / k_ed_bv_query): per query the oracle's
    brute-force k-NN over the stored traces. Queries: stored traces themselves (distance 0 to their own id),
    mutated copies, ones holding symbols the store never saw, an empty query."""
    rng = np.random.default_rng(w * n)
    ts = make_traces(n, lmin, lmax, mut, alphabet=alphabet, rng=rng)
    idx = hs.SimilarityIndex(ts, w, ctx=ctx)
    assert idx.bitparallel
    qs = [ts.trace(3), ts.trace(n - 1)]
    t = ts.trace(7).copy()
    if len(t):
        t[rng.random(len(t)) < 0.05] = np.uint64(12345)  # unseen symbol
    qs.append(t)
    t2 = ts.trace(11).copy()
    mm = rng.random(len(t2)) < 0.03
    t2[mm] = ts.sym[rng.integers(0, len(ts.sym), int(mm.sum()))]
    qs.append(t2)
    qs.append(np.zeros(0, np.uint64))
    ids, ds = idx.query(qs, k)
    for r, q in enumerate(qs):
        both = hs.TraceSet([q] + [ts.trace(i) for i in range(n)])
        pairs = np.stack([np.zeros(n, np.uint32), np.arange(1, n + 1, dtype=np.uint32)], 1)
        d = O.ed_pairs(both.off, both.sym, pairs, w)
        order = np.lexsort((np.arange(n), d))[:k]
        assert ds[r, :len(order)].tolist() == d[order].tolist(), r
        assert ids[r, :len(order)].tolist() == order.tolist(), r
    assert ds[0, 0] == 0 and ids[0, 0] in np.nonzero(
        [np.array_equal(ts.trace(i), ts.trace(3)) for i in range(n)])[0]
    idx.close()


def _query_vs_oracle(ts, qs, w, ids, ds, k):
    n = len(ts)
    for r, q in enumerate(qs):
        both = hs.TraceSet([q] + [ts.trace(i) for i in range(n)])
        pairs = np.stack([np.zeros(n, np.uint32), np.arange(1, n + 1, dtype=np.uint32)], 1)
        d = O.ed_pairs(both.off, both.sym, pairs, w, nthreads=16)
        order = np.lexsort((np.arange(n), d))[:k]
        assert ds[r, :len(order)].tolist() == d[order].tolist(), r
        assert ids[r, :len(order)].tolist() == order.tolist(), r


@pytest.mark.parametrize("w", [100, 1024, 4096])
def test_similarity_index_wide_band_queries_vs_oracle(ctx, w):
    """Single queries for bands above 64 against a resident 65,536-event store (16 traces x 4,096 events): the
    wide plan's query kernel (k_ed_wide_query: each query's match table once per call, a wave per (query, stored
    trace)) vs the oracle's brute force. Queries: a stored trace (distance 0 to itself), a shortened one, a
    mutated one with symbols the store never saw, an empty one, and one longer than every stored trace (within
    the band of some of them: the resident generic kernel)."""
    rng = np.random.default_rng(w)
    ts = make_traces(16, 4096, 4096, 0.06, alphabet=30, rng=rng)
    assert int(ts.off[-1]) == 65_536
    idx = hs.SimilarityIndex(ts, w, ctx=ctx)
    assert idx.kind == "wide"
    t = ts.trace(7).copy()
    t[rng.random(len(t)) < 0.05] = np.uint64(12345)  # unseen symbol
    longer = np.concatenate([ts.trace(5), ts.trace(6)[:w // 2 + 10]])
    qs = [ts.trace(3), ts.trace(9)[:4096 - w // 2], t, np.zeros(0, np.uint64), longer]
    k = 8
    ids, ds = idx.query(qs, k)
    idx.close()
    _query_vs_oracle(ts, qs, w, ids, ds, k)
    assert ds[0, 0] == 0


def test_similarity_index_generic_plan_queries_vs_oracle(ctx):
    """A band beyond the wide kernels (9,000 > 8,192) makes a generic plan: its queries run on the resident u64
    symbols (k_ed_query_generic), vs the oracle."""
    rng = np.random.default_rng(5)
    ts = make_traces(40, 150, 260, 0.2, alphabet=9, rng=rng)
    idx = hs.SimilarityIndex(ts, 9000, ctx=ctx)
    assert idx.kind == "generic"
    qs = [ts.trace(2), ts.trace(30)[:100], np.zeros(0, np.uint64),
          np.concatenate([ts.trace(1), ts.trace(1)]), np.full(40, 999, np.uint64)]
    ids, ds = idx.query(qs, 6)
    idx.close()
    _query_vs_oracle(ts, qs, 9000, ids, ds, 6)


def test_similarity_index_long_queries_on_bitparallel_plan(ctx):
    """Queries longer than every stored trace on a bit-parallel plan (band 32): within the band of the longest
    stored traces they have real distances <= 32, so they run on the resident generic kernel over the plan's
    encoded streams instead of being refused."""
    rng = np.random.default_rng(8)
    ts = make_traces(120, 180, 200, 0.02, alphabet=14, rng=rng)
    idx = hs.SimilarityIndex(ts, 32, ctx=ctx)
    assert idx.bitparallel
    L = max(len(ts.trace(i)) for i in range(len(ts)))
    longest = [i for i in range(len(ts)) if len(ts.trace(i)) == L][0]
    qs = [np.concatenate([ts.trace(longest), ts.trace(0)[:10]]), ts.trace(4), np.full(L + 40, 7, np.uint64)]
    ids, ds = idx.query(qs, 5)
    idx.close()
    _query_vs_oracle(ts, qs, 32, ids, ds, 5)
    assert ds[0, 0] <= 32


def test_search_similar_on_storage_uses_resident_index(ctx, tmp_path):
    from namazu_amd.signal import Event
    from tests.test_host import _make_storage
    evs = [Event.packet(f"entity-{i % 3}", "a", "b", {"n": i}) for i in range(40)]
    runs = [evs[i:i + 30] for i in range(8)]
    _make_storage(str(tmp_path), runs)
    st = hs.LoadStorage(str(tmp_path))
    t3, _ = st.GetStoredHistory(3)
    near = st.SearchSimilar(t3, 3, 8)
    assert near[0] == (3, 0) and [d for _, d in near] == sorted(d for _, d in near)
    assert st._index.bitparallel
    first = st._index
    assert st.SearchSimilar(t3, 2, 8)[0] == (3, 0) and st._index is first  # reused, not rebuilt


def test_device_and_host_plan_builds_agree(ab_knobs, ctx, monkeypatch):
    """Stores of >= 2^20 symbols build the bit-parallel plan on the device (sort/unique + binary-search remap);
    NMZ_ED_HOST_REMAP forces the host build. Both give the oracle's k-NN lists and the same single-query answers
    (the query dictionary comes from the device's sorted symbols)."""
    rng = np.random.default_rng(77)
    ts = make_traces(600, 1700, 2000, 0.01, alphabet=40, rng=rng)
    assert int(ts.off[-1]) >= 1 << 20
    ids_d, ds_d = knn(ctx, ts, 32, 5)
    qs = [ts.trace(5), ts.trace(9)[:1500]]
    qi_d, qd_d = hs.SimilarityIndex(ts, 32, ctx=ctx).query(qs, 4)
    monkeypatch.setenv("NMZ_ED_HOST_REMAP", "1")
    ids_h, ds_h = knn(ctx, ts, 32, 5)
    qi_h, qd_h = hs.SimilarityIndex(ts, 32, ctx=ctx).query(qs, 4)
    assert np.array_equal(ids_d, ids_h) and np.array_equal(ds_d, ds_h)
    assert np.array_equal(qi_d, qi_h) and np.array_equal(qd_d, qd_h)
    for q in [0, 299, 599]:
        pairs = np.array([[q, c] for c in range(len(ts)) if c != q], np.uint32)
        d = O.ed_pairs(ts.off, ts.sym, pairs, 32, nthreads=16)
        order = np.lexsort((pairs[:, 1], d))[:5]
        assert ds_d[q].tolist() == d[order].tolist() and ids_d[q].tolist() == pairs[order, 1].tolist()


def test_device_plan_symbols_zero_and_all_ones(ab_knobs, ctx, monkeypatch):
    """The device plan's distinct-symbol set (an LDS + global hash set, csrc/unique.hip) keeps 0 and 2^64 - 1 (its
    free-slot value) as symbols like any other: same k-NN lists as the host build and the oracle."""
    rng = np.random.default_rng(78)
    base = make_traces(600, 1700, 2000, 0.01, alphabet=40, rng=rng)
    m = {np.uint64(3): np.uint64(0), np.uint64(0x9E3779B97F4A7C15 + 3): np.uint64(2**64 - 1)}
    trs = []
    for i in range(len(base)):
        t = base.trace(i).copy()
        for a, b in m.items():
            t[t == a] = b
        trs.append(t)
    ts = hs.TraceSet(trs)
    assert int(ts.off[-1]) >= 1 << 20 and (ts.sym == 0).any() and (ts.sym == np.uint64(2**64 - 1)).any()
    ids_d, ds_d = knn(ctx, ts, 32, 5)
    monkeypatch.setenv("NMZ_ED_HOST_REMAP", "1")
    ids_h, ds_h = knn(ctx, ts, 32, 5)
    assert np.array_equal(ids_d, ids_h) and np.array_equal(ds_d, ds_h)
    for q in [0, 411]:
        pairs = np.array([[q, c] for c in range(len(ts)) if c != q], np.uint32)
        d = O.ed_pairs(ts.off, ts.sym, pairs, 32, nthreads=16)
        order = np.lexsort((pairs[:, 1], d))[:5]
        assert ds_d[q].tolist() == d[order].tolist() and ids_d[q].tolist() == pairs[order, 1].tolist()


def test_wide_device_and_host_plan_builds_agree(ab_knobs, ctx, monkeypatch):
    """Wide-band stores of >= 2^20 symbols build k_ed_wide's plan on the device (hash-set alphabet + remap kernel,
    ids by sorted rank instead of first appearance); NMZ_ED_HOST_REMAP forces the host build. Same k-NN lists,
    and the oracle's for sampled queries."""
    rng = np.random.default_rng(80)
    ts = make_traces(300, 3600, 3900, 0.02, alphabet=40, rng=rng)
    assert int(ts.off[-1]) >= 1 << 20
    ids_d, ds_d = knn(ctx, ts, 1500, 4)
    monkeypatch.setenv("NMZ_ED_HOST_REMAP", "1")
    ids_h, ds_h = knn(ctx, ts, 1500, 4)
    assert np.array_equal(ids_d, ids_h) and np.array_equal(ds_d, ds_h)
    for q in [0, 157]:
        pairs = np.array([[q, c] for c in range(len(ts)) if c != q], np.uint32)
        d = O.ed_pairs(ts.off, ts.sym, pairs, 1500, nthreads=16)
        order = np.lexsort((pairs[:, 1], d))[:4]
        assert ds_d[q].tolist() == d[order].tolist() and ids_d[q].tolist() == pairs[order, 1].tolist()


def test_device_plan_too_many_symbols_falls_back(ctx):
    """A store of >= 2^20 symbols with ~10^6 distinct values: the device distinct set passes its cap (65,533), the
    plan falls back to the host build and the exact generic kernel. All symbols distinct except one copied trace,
    so every distance is beyond the band except the copy's (0)."""
    rng = np.random.default_rng(79)
    trs = [rng.integers(0, 2**64, size=7200, dtype=np.uint64) for _ in range(150)]
    trs[111] = trs[17].copy()
    ts = hs.TraceSet(trs)
    assert int(ts.off[-1]) >= 1 << 20
    ids, ds = knn(ctx, ts, 32, 3)
    assert ds[111][0] == 0 and ids[111][0] == 17 and ds[17][0] == 0 and ids[17][0] == 111
    others = np.ones(len(ts), bool)
    others[[17, 111]] = False
    assert (ds[others] == 33).all() and (ds[[17, 111], 1:] == 33).all()
    # neighbours beyond the band are listed by index (the reference's stable order)
    assert ids[0].tolist() == [1, 2, 3] and ids[17][1:].tolist() == [0, 1]


def _edited_family(n, length, alphabet, max_edits, rng):
    """Traces = one base with 0..max_edits random edits each (adjacent transpositions, substitutions,
    insertions, deletions), so pair distances spread across the band edge and the q-gram bound's edge."""
    base = rng.integers(0, alphabet, size=length)
    out = []
    for _ in range(n):
        t = list(base)
        for _ in range(int(rng.integers(0, max_edits + 1))):
            op, p = int(rng.integers(0, 4)), int(rng.integers(0, max(len(t) - 1, 1)))
            if op == 0 and len(t) > 1:
                t[p], t[p + 1] = t[p + 1], t[p]
            elif op == 1:
                t[p] = int(rng.integers(0, alphabet))
            elif op == 2:
                t.insert(p, int(rng.integers(0, alphabet)))
            elif len(t) > 1:
                del t[p]
        out.append(np.array(t, np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(11))
    return hs.TraceSet(out)


@pytest.mark.parametrize("recompute", [False, True])
@pytest.mark.parametrize("w,alphabet,max_edits", [(32, 48, 90), (16, 6, 40), (8, 200, 25)])
def test_knn_qgram_filter_exact(ab_knobs, ctx, monkeypatch, w, alphabet, max_edits, recompute):
    """The q-gram lower bound (bigram profiles > 4w apart => ED_w = w + 1 without a DP) and the in-band-only
    publishing + k_knn_fill: the all-pairs k-NN equals the oracle's and the run with the filter off, the counters
    show pairs settled by the bound and pairs that ran the DP, and the shard path (merge + fill) agrees too. The
    write pass runs from the count pass's survivor records, or (recompute) re-runs the filter."""
    import torch
    if recompute:
        monkeypatch.setenv("NMZ_ED_QG_RECOMPUTE", "1")
    L = _lib.load()
    rng = np.random.default_rng(w * 1000 + alphabet)
    ts = _edited_family(400, 300, alphabet, max_edits, rng)
    n, k = len(ts), 8
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def make_plan(qgram):  # the filter switch is plan state, fixed at creation (NMZ_ED_QGRAM read then)
        monkeypatch.setenv("NMZ_ED_QGRAM", "1" if qgram else "0")
        plan = ctypes.c_void_p()
        _lib.check(L.nmz_ed_plan_create(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), n, w, ctypes.byref(plan)))
        assert L.nmz_ed_plan_is_fast(plan) == 2
        return plan

    def run(qgram):
        plan = make_plan(qgram)
        monkeypatch.setenv("NMZ_ED_QGRAM", "0" if qgram else "1")  # a later change does not reach the plan
        d = torch.empty(n * k, dtype=torch.int64, device="cuda")
        _lib.check(L.nmz_ed_allpairs_knn_dev(plan, k, ctypes.c_void_p(d.data_ptr()), stream))
        cnt = np.zeros(_lib.NMZ_ED_NCOUNTERS, np.uint64)
        _lib.check(L.nmz_ed_plan_counters(plan, _lib.ptr(cnt), stream))
        L.nmz_ed_plan_destroy(plan)
        return d.cpu().numpy().view(np.uint64).reshape(n, k), cnt

    on, c_on = run(True)
    off, c_off = run(False)
    S = 3
    parts = torch.empty(S * n * k, dtype=torch.int64, device="cuda")
    out = torch.empty(n * k, dtype=torch.int64, device="cuda")
    plan = make_plan(True)
    for s in range(S):
        _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, s, S, ctypes.c_void_p(parts.data_ptr() + s * n * k * 8),
                                                   stream))
    _lib.check(L.nmz_knn_merge_dev(ctx.handle, ctypes.c_void_p(parts.data_ptr()), S, n, k,
                                   ctypes.c_void_p(out.data_ptr()), stream))
    _lib.check(L.nmz_ed_knn_fill_dev(plan, k, ctypes.c_void_p(out.data_ptr()), stream))
    torch.cuda.synchronize()  # the default torch stream is NULL here: the calls ran on the context's stream
    sharded = out.cpu().numpy().view(np.uint64).reshape(n, k)
    L.nmz_ed_plan_destroy(plan)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, k, nthreads=16)
    ref = (od.astype(np.uint64) << np.uint64(32)) | oi.astype(np.uint64)
    assert np.array_equal(on, ref) and np.array_equal(off, ref) and np.array_equal(sharded, ref)
    assert c_on[5] > 0 and c_on[0] > 0 and c_off[5] == 0
    assert c_on[1] == c_off[1]  # the same in-band pairs
    assert c_on[0] + c_on[5] == c_off[0]  # every pair the bound settles would have run the DP


@pytest.mark.parametrize("limit", [0, 1, 500, "mid"])
def test_knn_two_phase_entry_limit_batches(ab_knobs, ctx, monkeypatch, limit):
    """Entry lists beyond the two-phase limit (2^30 entries; NMZ_ED_TP_MAX_ENTRIES lowers it) run in batches of
    whole query blocks after the count pass (csrc/ed.hip ed_bv_two_phase). The count pass lists pairs with an empty
    trace before the total is known, so the batches must start from empty lists: near-duplicates with empty traces
    in the store (n + m <= w pairs), vs the oracle, through the one-shard and the 3-shard (merge + fill) paths.
    "mid" puts the limit between the shards' own entry totals, so some shards of one search split into batches and
    others do not: each must still cover exactly its own query blocks (no pair dropped or doubled)."""
    import torch
    if limit != "mid":
        monkeypatch.setenv("NMZ_ED_TP_MAX_ENTRIES", str(limit))
    L = _lib.load()
    rng = np.random.default_rng(77 + (limit if limit != "mid" else 3))
    ts0 = _edited_family(500, 120, 16, 30, rng)
    trs = [ts0.trace(i) for i in range(len(ts0))]
    for i in (3, 40, 41, 333):
        trs[i] = np.zeros(0, np.uint64)
    trs[100] = trs[100][:5]
    ts = hs.TraceSet(trs)
    n, k, w = len(ts), 8, 32
    ids, ds = knn(ctx, ts, w, k)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, k, nthreads=16)
    assert np.array_equal(ids, oi) and np.array_equal(ds, od)
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_ed_plan_create(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), n, w, ctypes.byref(plan)))
    assert L.nmz_ed_plan_is_fast(plan) == 2
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    S = 3
    parts = torch.empty(S * n * k, dtype=torch.int64, device="cuda")
    out = torch.empty(n * k, dtype=torch.int64, device="cuda")
    if limit == "mid":  # the shards' DP pairs (= their entries) under the default limit, then a limit between them
        per = []
        for s in range(S):
            _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, s, S, ctypes.c_void_p(parts.data_ptr()), stream))
            cnt = np.zeros(6, np.uint64)
            _lib.check(L.nmz_ed_plan_counters(plan, _lib.ptr(cnt), stream))
            per.append(int(cnt[0]))
        assert min(per) < max(per), per
        monkeypatch.setenv("NMZ_ED_TP_MAX_ENTRIES", str((min(per) + max(per)) // 2))
    for s in range(S):
        _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, s, S, ctypes.c_void_p(parts.data_ptr() + s * n * k * 8),
                                                   stream))
    _lib.check(L.nmz_knn_merge_dev(ctx.handle, ctypes.c_void_p(parts.data_ptr()), S, n, k,
                                   ctypes.c_void_p(out.data_ptr()), stream))
    _lib.check(L.nmz_ed_knn_fill_dev(plan, k, ctypes.c_void_p(out.data_ptr()), stream))
    torch.cuda.synchronize()
    sharded = out.cpu().numpy().view(np.uint64).reshape(n, k)
    L.nmz_ed_plan_destroy(plan)
    ref = (od.astype(np.uint64) << np.uint64(32)) | oi.astype(np.uint64)
    assert np.array_equal(sharded, ref)


def _family_store(n, family, per_family, alphabet_total, seed, length=2048):
    from namazu_amd.synth import clustered_traces
    return clustered_traces(n, length, seed=seed, n_symbols=per_family, family=family,
                            alphabet_total=alphabet_total, edits_mean=10.0)


def test_knn_compact_tables_5000_symbol_store(ctx):
    """A store whose alphabet (>= 5,000 distinct events, L = 2,048) is far beyond the direct LDS tables (117
    symbols) stays on the bit-parallel kernels with compact tables (each workgroup's rows = its query pair's own
    symbols): all-pairs k-NN vs the oracle, the 3-shard merge path, and single queries (nmz_ed_plan_query_knn)
    vs brute force."""
    import torch
    ts = _family_store(520, 4, 40, 200_000, seed=9)
    assert len(np.unique(ts.sym)) >= 5000
    n, k, w = len(ts), 8, 32
    assert _plan_kind(ctx, ts, w) == 2
    ids, ds = knn(ctx, ts, w, k)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, k, nthreads=16)
    assert np.array_equal(ids, oi) and np.array_equal(ds, od)
    assert (od[:, 0] <= w).mean() > 0.8  # most traces have family members inside the band
    L = _lib.load()
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_ed_plan_create(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), n, w, ctypes.byref(plan)))
    S = 3
    parts = torch.empty(S * n * k, dtype=torch.int64, device="cuda")
    out = torch.empty(n * k, dtype=torch.int64, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for sh in range(S):
        _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, sh, S, ctypes.c_void_p(parts.data_ptr() + sh * n * k * 8),
                                                   stream))
    _lib.check(L.nmz_knn_merge_dev(ctx.handle, ctypes.c_void_p(parts.data_ptr()), S, n, k,
                                   ctypes.c_void_p(out.data_ptr()), stream))
    _lib.check(L.nmz_ed_knn_fill_dev(plan, k, ctypes.c_void_p(out.data_ptr()), stream))
    torch.cuda.synchronize()
    L.nmz_ed_plan_destroy(plan)
    keys = out.cpu().numpy().view(np.uint64).reshape(n, k)
    assert np.array_equal((keys >> np.uint64(32)).astype(np.uint32), od)
    assert np.array_equal((keys & np.uint64(0xFFFFFFFF)).astype(np.uint32), oi)
    idx = hs.SimilarityIndex(ts, w, ctx=ctx)
    assert idx.bitparallel
    rng = np.random.default_rng(4)
    t = ts.trace(101).copy()
    t[rng.random(len(t)) < 0.004] = np.uint64(77777)  # a symbol the store never saw
    qs = [ts.trace(17), t, ts.trace(400)[:2000]]
    qi, qd = idx.query(qs, 6)
    idx.close()
    for r, q in enumerate(qs):
        both = hs.TraceSet([q] + [ts.trace(i) for i in range(n)])
        pairs = np.stack([np.zeros(n, np.uint32), np.arange(1, n + 1, dtype=np.uint32)], 1)
        d = O.ed_pairs(both.off, both.sym, pairs, w, nthreads=16)
        order = np.lexsort((np.arange(n), d))[:6]
        assert qd[r].tolist() == d[order].tolist() and qi[r].tolist() == order.tolist(), r


@pytest.mark.parametrize("w", [8, 21, 32, 64])
def test_knn_compact_tables_forced(ab_knobs, ctx, monkeypatch, w):
    """NMZ_ED_COMPACT forces the compact tables on a small-alphabet store: the same lists as the direct tables
    and the oracle, through the two-phase search, the single-kernel search (NMZ_ED_TWO_PHASE=0) and both plan
    builds (device: >= 2^20 symbols; NMZ_ED_HOST_REMAP: host)."""
    ts = make_traces(560, 1850, 2000, 0.004, alphabet=30, rng=np.random.default_rng(w))
    assert int(ts.off[-1]) >= 1 << 20
    k = 5
    ref_i, ref_d = knn(ctx, ts, w, k)
    monkeypatch.setenv("NMZ_ED_COMPACT", "1")
    for env in ({}, {"NMZ_ED_TWO_PHASE": "0"}, {"NMZ_ED_HOST_REMAP": "1"}):
        for key, v in env.items():
            monkeypatch.setenv(key, v)
        assert _plan_kind(ctx, ts, w) == 2
        ci, cd = knn(ctx, ts, w, k)
        assert np.array_equal(ci, ref_i) and np.array_equal(cd, ref_d), env
        for key in env:
            monkeypatch.delenv(key)
    for q in [0, 301, 559]:
        pairs = np.array([[q, c] for c in range(len(ts)) if c != q], np.uint32)
        d = O.ed_pairs(ts.off, ts.sym, pairs, w, nthreads=16)
        order = np.lexsort((pairs[:, 1], d))[:k]
        assert ref_d[q].tolist() == d[order].tolist() and ref_i[q].tolist() == pairs[order, 1].tolist()


def _fp(L, plan):
    fp = np.zeros(_lib.NMZ_ED_FP_WORDS, np.uint64)
    _lib.check(L.nmz_ed_plan_fingerprint(plan, _lib.ptr(fp)))
    return fp


@pytest.mark.parametrize("S", [3, 4, 8])
def test_shards_partition_across_search_forms(ctx, S):
    """A shard owns whole 64-query blocks (nmz_ed_block_shard) whichever form of the bit-parallel search its plan
    took -- two-phase, single kernel, no q-gram filter, compact tables (NMZ_ED_OPT_*) -- so shards of one search
    run with different forms still partition the pairs exactly: shard s here runs on plan s mod 4, and the merged,
    filled lists equal the oracle's (a pair dropped or doubled would change them). The plans' fingerprints differ,
    which is what the multi-rank paths check before a search (dist.check_ed_plans, nmz_ed_group_plan_create)."""
    import torch
    L = _lib.load()
    rng = np.random.default_rng(S)
    ts = _edited_family(700, 150, 24, 30, rng)
    n, k, w = len(ts), 6, 32
    forms = [0, _lib.NMZ_ED_OPT_SINGLE_KERNEL, _lib.NMZ_ED_OPT_NO_QGRAM, _lib.NMZ_ED_OPT_COMPACT]
    plans = []
    for o in forms:
        p = ctypes.c_void_p()
        _lib.check(L.nmz_ed_plan_create_opts(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), None, n, w, o,
                                             ctypes.byref(p)))
        assert L.nmz_ed_plan_is_fast(p) == 2
        plans.append(p)
    fps = [_fp(L, p) for p in plans]
    assert all(not np.array_equal(fps[0], f) for f in fps[1:])
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    parts = torch.empty(S * n * k, dtype=torch.int64, device="cuda")
    out = torch.empty(n * k, dtype=torch.int64, device="cuda")
    for s in range(S):
        _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plans[s % 4], k, s, S,
                                                   ctypes.c_void_p(parts.data_ptr() + s * n * k * 8), stream))
    _lib.check(L.nmz_knn_merge_dev(ctx.handle, ctypes.c_void_p(parts.data_ptr()), S, n, k,
                                   ctypes.c_void_p(out.data_ptr()), stream))
    _lib.check(L.nmz_ed_knn_fill_dev(plans[0], k, ctypes.c_void_p(out.data_ptr()), stream))
    torch.cuda.synchronize()
    for p in plans:
        L.nmz_ed_plan_destroy(p)
    keys = out.cpu().numpy().view(np.uint64).reshape(n, k)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, k, nthreads=16)
    assert np.array_equal((keys >> np.uint64(32)).astype(np.uint32), od)
    assert np.array_equal((keys & np.uint64(0xFFFFFFFF)).astype(np.uint32), oi)


def test_knobs_need_nmz_ab(ctx, monkeypatch):
    """NMZ_* A/B knobs reach the library only under NMZ_AB=1: without it NMZ_ED_TWO_PHASE=0 / NMZ_ED_QGRAM=0 leave
    the plan as the product builds it (same fingerprint), with it they change the plan."""
    L = _lib.load()
    ts = _edited_family(200, 100, 16, 20, np.random.default_rng(5))

    def fp():
        p = ctypes.c_void_p()
        _lib.check(L.nmz_ed_plan_create(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), len(ts), 32, ctypes.byref(p)))
        f = _fp(L, p)
        L.nmz_ed_plan_destroy(p)
        return f

    monkeypatch.delenv("NMZ_AB", raising=False)
    monkeypatch.delenv("NMZ_ED_TWO_PHASE", raising=False)
    monkeypatch.delenv("NMZ_ED_QGRAM", raising=False)
    base = fp()
    monkeypatch.setenv("NMZ_ED_TWO_PHASE", "0")
    monkeypatch.setenv("NMZ_ED_QGRAM", "0")
    assert np.array_equal(fp(), base)
    monkeypatch.setenv("NMZ_AB", "1")
    f = fp()
    assert not np.array_equal(f, base) and int(f[4]) & 3 == 0 and int(base[4]) & 3 == 3


def test_similarity_index_k_beyond_64(ctx):
    """SimilarityIndex.query with k > 64 (the reference's search has no cap, naive.go:235): every pair distance on
    the GPU (nmz_ed_pairs), ordered by (distance, id), equal to the oracle's brute force; k <= 64 answers agree with
    its prefix."""
    ts = _edited_family(150, 80, 12, 20, np.random.default_rng(8))
    idx = hs.SimilarityIndex(ts, 16, ctx=ctx)
    qs = [ts.trace(3), ts.trace(77)[:60]]
    qi, qd = idx.query(qs, 100)
    si, sd = idx.query(qs, 40)
    idx.close()
    n = len(ts)
    for r, q in enumerate(qs):
        both = hs.TraceSet([q] + [ts.trace(i) for i in range(n)])
        pairs = np.stack([np.zeros(n, np.uint32), np.arange(1, n + 1, dtype=np.uint32)], 1)
        d = O.ed_pairs(both.off, both.sym, pairs, 16)
        order = np.lexsort((np.arange(n), d))[:100]
        assert qi[r].tolist() == order.tolist() and qd[r].tolist() == d[order].tolist()
        assert si[r].tolist() == qi[r, :40].tolist() and sd[r].tolist() == qd[r, :40].tolist()


def test_repeated_shard_searches_use_cached_sizes(ctx):
    """A shard's second and later two-phase searches enqueue every kernel with the sizes its first search read
    back (no host round trip); the kernels still run in full, so the lists equal the first search's and the
    oracle's, and a device check of this search's own totals against the cached ones passes
    (nmz_ed_plan_counters raises otherwise)."""
    import torch
    L = _lib.load()
    ts = _edited_family(600, 160, 20, 30, np.random.default_rng(31))
    n, k, w, S = len(ts), 6, 32, 3
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_ed_plan_create(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), n, w, ctypes.byref(plan)))
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    parts = torch.empty(S * n * k, dtype=torch.int64, device="cuda")
    out = torch.empty(n * k, dtype=torch.int64, device="cuda")
    runs = []
    cnt = np.zeros(_lib.NMZ_ED_NCOUNTERS, np.uint64)
    for rep in range(3):
        for s in range(S):
            _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, s, S,
                                                       ctypes.c_void_p(parts.data_ptr() + s * n * k * 8), stream))
        _lib.check(L.nmz_knn_merge_dev(ctx.handle, ctypes.c_void_p(parts.data_ptr()), S, n, k,
                                       ctypes.c_void_p(out.data_ptr()), stream))
        _lib.check(L.nmz_ed_knn_fill_dev(plan, k, ctypes.c_void_p(out.data_ptr()), stream))
        _lib.check(L.nmz_ed_plan_counters(plan, _lib.ptr(cnt), stream))
        runs.append(out.cpu().numpy().view(np.uint64).reshape(n, k).copy())
    L.nmz_ed_plan_destroy(plan)
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, k, nthreads=16)
    ref = (od.astype(np.uint64) << np.uint64(32)) | oi.astype(np.uint64)
    for r in runs:
        assert np.array_equal(r, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("n,item,big", [(1, 128, False), (2047, 128, False), (2048, 4096, False),
                                         (2049, 256, False), (256 * 2048 + 5, 128, False),
                                         (3_000_001, 1024, False), (20, 128, True)])
def test_two_phase_offset_kernels(ctx, n, item, big):
    """k_tp_reduce + k_tp_scan (the two-phase search's offsets after its count pass) against numpy: entry offsets and
    work-item offsets as exclusive sums mod 2^32, the 64-bit entry total. n past 256 x 2,048 pairs makes every block
    scan several 2,048-pair tiles; `big` counts push the total past 2^32 (the offsets wrap, the total must not)."""
    import ctypes

    import torch
    L = _lib.load()
    rng = np.random.default_rng(n + item)
    cnt = (rng.integers(2**28, 2**30, n) if big else rng.integers(0, 40, n)).astype(np.uint32)
    cnt[rng.random(n) < 0.3] = 0
    d_cnt = torch.from_numpy(cnt.view(np.int32)).cuda()
    d_poff = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
    d_ioff = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
    d_tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    _lib.check(L.nmz_debug_tp_offsets(ctx.handle, ctypes.c_void_p(d_cnt.data_ptr()), n, item,
                                      ctypes.c_void_p(d_poff.data_ptr()), ctypes.c_void_p(d_ioff.data_ptr()),
                                      ctypes.c_void_p(d_tot.data_ptr()), None))
    c64 = cnt.astype(np.uint64)
    exp_p = np.concatenate([[0], np.cumsum(c64)]).astype(np.uint64)
    exp_i = np.concatenate([[0], np.cumsum((c64 + item - 1) // item)]).astype(np.uint64)
    assert np.array_equal(d_poff.cpu().numpy().view(np.uint32), (exp_p & 0xFFFFFFFF).astype(np.uint32))
    assert np.array_equal(d_ioff.cpu().numpy().view(np.uint32), (exp_i & 0xFFFFFFFF).astype(np.uint32))
    assert int(d_tot.cpu().numpy().view(np.uint64)[0]) == int(exp_p[-1])


def test_cached_searches_back_to_back_then_destroy(ctx):
    """Cached searches publish their mismatch flag from the offsets scan into pinned host words (csrc/ed.hip
    ed_tp_flag_*: a sequence number, then the flag; no copy or event on the queue). Enqueued back to back without a
    synchronisation, none reports a mismatch (a number not yet landed is read later) and the last one's lists equal
    the oracle; destroying the plan right after a burst waits for the last scan's words before freeing them."""
    import torch
    L = _lib.load()
    ts = _edited_family(300, 150, 16, 30, np.random.default_rng(23))
    n, k, w = len(ts), 8, 32
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, k, nthreads=16)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    keys = torch.empty(n * k, dtype=torch.int64, device="cuda")
    for destroy_in_flight in (False, True):
        plan = ctypes.c_void_p()
        _lib.check(L.nmz_ed_plan_create(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), n, w, ctypes.byref(plan)))
        try:
            assert L.nmz_ed_plan_is_fast(plan) == 2
            _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, 0, 1, ctypes.c_void_p(keys.data_ptr()), stream))
            torch.cuda.synchronize()  # sizes read back: the searches below run from the cache
            for _ in range(8):
                _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, 0, 1, ctypes.c_void_p(keys.data_ptr()), stream))
            if destroy_in_flight:  # the burst is still running: destroy waits for its last scan's words
                L.nmz_ed_plan_destroy(plan)
                plan = None
                torch.cuda.synchronize()
                continue
            torch.cuda.synchronize()
            out = keys.clone()
            torch.cuda.synchronize()
            _lib.check(L.nmz_ed_knn_fill_dev(plan, k, ctypes.c_void_p(out.data_ptr()), stream))
            torch.cuda.synchronize()
            kk = out.cpu().numpy().view(np.uint64).reshape(n, k)
            ids, ds = (kk & np.uint64(0xFFFFFFFF)).astype(np.uint32), (kk >> np.uint64(32)).astype(np.uint32)
            assert np.array_equal(ids, oi) and np.array_equal(ds, od)
            cnt = np.zeros(_lib.NMZ_ED_NCOUNTERS, np.uint64)
            _lib.check(L.nmz_ed_plan_counters(plan, _lib.ptr(cnt), stream))  # no mismatch pending
        finally:
            if plan is not None:
                L.nmz_ed_plan_destroy(plan)


def test_cached_size_mismatch_skips_writes_and_surfaces(ab_knobs, ctx, monkeypatch):
    """A shard's later searches run with the sizes its first search read back (csrc/ed.hip ed_bv_two_phase); a
    one-thread check flags a search whose own totals differ. NMZ_ED_TP_FAKE_MISMATCH forces the flag on a cached
    search: that search writes no entry and runs no DP (nothing past the lists sized for the cached totals), the
    shard's next search reports it (NMZ_EHIP) and drops the cache, and the search after that is whole again and
    equals the oracle. nmz_ed_plan_counters reports a pending flag too."""
    import torch
    L = _lib.load()
    ts = _edited_family(300, 150, 16, 30, np.random.default_rng(21))
    n, k, w = len(ts), 8, 32
    oi, od = O.ed_allpairs_knn(ts.off, ts.sym, w, k, nthreads=16)
    plan = ctypes.c_void_p()
    _lib.check(L.nmz_ed_plan_create(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), n, w, ctypes.byref(plan)))
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    keys = torch.empty(n * k, dtype=torch.int64, device="cuda")

    def search():
        rc = L.nmz_ed_allpairs_knn_shard_dev(plan, k, 0, 1, ctypes.c_void_p(keys.data_ptr()), stream)
        torch.cuda.synchronize()
        return rc

    def lists():
        out = torch.empty_like(keys)
        out.copy_(keys)
        torch.cuda.synchronize()  # the copy (torch's stream) before the fill (the context's stream)
        _lib.check(L.nmz_ed_knn_fill_dev(plan, k, ctypes.c_void_p(out.data_ptr()), stream))
        torch.cuda.synchronize()
        kk = out.cpu().numpy().view(np.uint64).reshape(n, k)
        return (kk & np.uint64(0xFFFFFFFF)).astype(np.uint32), (kk >> np.uint64(32)).astype(np.uint32)

    try:
        assert L.nmz_ed_plan_is_fast(plan) == 2
        for _ in range(2):  # the first search reads its sizes back, the second runs from the cache
            assert search() == _lib.NMZ_OK
            ids, ds = lists()
            assert np.array_equal(ids, oi) and np.array_equal(ds, od)
        monkeypatch.setenv("NMZ_ED_TP_FAKE_MISMATCH", "1")
        assert search() == _lib.NMZ_OK  # enqueued with the cached sizes; the check flags it on the device
        monkeypatch.delenv("NMZ_ED_TP_FAKE_MISMATCH")
        ids, ds = lists()
        assert not (np.array_equal(ids, oi) and np.array_equal(ds, od))  # the flagged search ran no DP
        cnt = np.zeros(_lib.NMZ_ED_NCOUNTERS, np.uint64)
        assert L.nmz_ed_plan_counters(plan, _lib.ptr(cnt), stream) == _lib.NMZ_EHIP
        assert "cached sizes" in _lib.last_error()
        _lib.check(L.nmz_ed_plan_counters(plan, _lib.ptr(cnt), stream))  # reported once, then clear
        for _ in range(2):  # recounted (the cache was dropped), then cached again
            assert search() == _lib.NMZ_OK
            ids, ds = lists()
            assert np.array_equal(ids, oi) and np.array_equal(ds, od)
        # the non-waiting report: the shard's next search fails with the flag of the previous one
        monkeypatch.setenv("NMZ_ED_TP_FAKE_MISMATCH", "1")
        assert search() == _lib.NMZ_OK
        monkeypatch.delenv("NMZ_ED_TP_FAKE_MISMATCH")
        assert search() == _lib.NMZ_EHIP
        assert search() == _lib.NMZ_OK
        ids, ds = lists()
        assert np.array_equal(ids, oi) and np.array_equal(ds, od)
    finally:
        L.nmz_ed_plan_destroy(plan)
