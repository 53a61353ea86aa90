"""CPU: pin the oracle against published KATs, the golden fixtures and
independent pure-Python restatements (no GPU)."""
import os
import re
import sys

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from gen_go_rng_cooked import GoRand as PyGoRand  # noqa: E402  (pure-Python rngSource)

M64 = (1 << 64) - 1


def test_fnv_kat(golden):
    for s, h in golden("fnv_kat.json")["vectors"]:
        assert O.fnv1a64(s.encode()) == int(h, 16)
        assert O.fnv1a64_py(s.encode()) == int(h, 16)


def test_fnv_c_vs_python():
    rng = np.random.default_rng(0)
    for n in [0, 1, 7, 8, 19, 64]:
        b = bytes(rng.integers(0, 256, n, dtype=np.uint8))
        assert O.fnv1a64(b) == O.fnv1a64_py(b)


def test_go_rand_kat(golden):
    k = golden("go_rand_kat.json")
    r = O.GoRand(k["seed"])
    assert [r.int63() for _ in k["int63"]] == k["int63"]
    r = O.GoRand(k["seed"])
    assert [r.intn(100) for _ in k["intn100"]] == k["intn100"]
    r = O.GoRand(k["seed"])
    assert [r.intn(10) for _ in k["intn10"]] == k["intn10"]
    assert list(O.go_rng_cooked()[:3]) == k["rng_cooked_head"]


def test_cooked_table_matches_product_header():
    """The oracle derives rngCooked itself; the product ships a generated copy."""
    hdr = open(os.path.join(ROOT, "namazu_amd", "csrc", "go_rng_cooked.h")).read()
    vals = [int(x, 16) for x in re.findall(r"0x([0-9a-f]{16})ULL", hdr)]
    assert len(vals) == 607
    assert [v & M64 for v in O.go_rng_cooked().tolist()] == vals


@pytest.mark.parametrize("seed", [1, 0, -1, 2147483647, -2147483647, 2**62 + 12345, -(2**63), 89482311,
                                  4294967294, 123456789])
def test_go_rand_c_vs_python(seed):
    cooked = O.go_rng_cooked().tolist()
    py = PyGoRand(cooked, _go_mod_seed(seed))
    c = O.GoRand(seed)
    for _ in range(700):  # crosses the 607/273 lag boundaries
        assert c.uint64() == py.uint64()


def _go_mod_seed(seed):
    """The Python KAT helper reduces with Python's %, matching Go's result."""
    s = seed % (2**31 - 1) if seed >= 0 else -((-seed) % (2**31 - 1))
    if s < 0:
        s += 2**31 - 1
    return s


def test_int63n_int31n_ranges_and_intn_dispatch():
    r1 = O.GoRand(42)
    for n in [1, 2, 1024, 999, 70_000_000, 2**62 + 1]:
        v = r1.int63n(n)
        assert 0 <= v < n
    # Intn(n) for n < 2^31 is Int31n(n) on the same stream (rand.go Intn)
    a, b = O.GoRand(7), O.GoRand(7)
    assert [a.intn(999) for _ in range(50)] == [b.int31n(999) for _ in range(50)]
    # power of two: mask, no rejection draw
    c, d = O.GoRand(9), O.GoRand(9)
    assert c.int63n(1 << 20) == d.int63() & ((1 << 20) - 1)


def test_replayable_golden(golden):
    for case in golden("replayable_foobar.json")["cases"]:
        m = case["max_interval_ns"]
        if "seed" in case:
            got = [O.replayable_interval(case["seed"], h, m) for h in case["hints"]]
            assert got == case["delays_ns"]
        else:
            for s, row in zip(case["seed_list"], case["delays_ns"]):
                assert [O.replayable_interval(s, h, m) for h in case["hints"]] == row


def test_replayable_vs_python():
    rng = np.random.default_rng(1)
    for _ in range(200):
        seed = "".join(chr(c) for c in rng.integers(32, 127, rng.integers(0, 12)))
        hint = "".join(chr(c) for c in rng.integers(32, 127, rng.integers(0, 25)))
        m = int(rng.choice([1, 10_000_000, 2**30 + 1, 2**63 - 1]))
        h = O.fnv1a64_py((seed + hint).encode())
        assert O.replayable_interval(seed, hint, m) == h % m
    assert O.replayable_interval("x", "y", 0) == 0  # replayablepolicy.go:101-104


def test_replayable_negative_interval():
    """uint64(negative Duration) as the modulus; the result may be a negative Duration."""
    h = O.fnv1a64_py(b"ab")
    m = -5
    exp = h % ((m + 2**64) % 2**64)
    exp = exp - 2**64 if exp >= 2**63 else exp
    assert O.replayable_interval("a", "b", m) == exp


def _py_random_decide(seed, evhash, cls, mn, mx, thr, cooked):
    buf = seed.to_bytes(8, "little") + evhash.to_bytes(8, "little")
    es = O.fnv1a64_py(buf)
    es = es - 2**64 if es >= 2**63 else es
    r = PyGoRand(cooked, _go_mod_seed(es))
    if cls & 1:
        mn, mx = int(float(mn) * 0.8), int(float(mx) * 0.8)
    if mn == mx:
        d = mn
    else:
        n = mx - mn
        if n & (n - 1) == 0:
            d = (r.uint64() & (2**63 - 1)) & (n - 1)
        else:
            mxa = 2**63 - 1 - (2**63 % n)
            v = r.uint64() & (2**63 - 1)
            while v > mxa:
                v = r.uint64() & (2**63 - 1)
            d = v % n
        d += mn
    f = False
    if cls & 2:
        f = r.int31n(999) < thr
    return d, f


def test_random_golden_and_python(golden):
    cooked = O.go_rng_cooked().tolist()
    for rec in golden("random_decisions.json")["decisions"]:
        p = O.random_params(rec["min_ns"], rec["max_ns"], rec["p"])
        d, f, n = O.random_decide(rec["seed"], rec["evhash"], rec["evclass"], p)
        assert (d, f, n) == (rec["delay_ns"], rec["fault"], rec["rng_outputs"])
        assert O.random_event_seed(rec["seed"], rec["evhash"]) == rec["event_seed"]
        assert _py_random_decide(rec["seed"], rec["evhash"], rec["evclass"], rec["min_ns"], rec["max_ns"],
                                 p.fault_threshold, cooked) == (d, f)


def test_random_params_semantics():
    p = O.random_params(30_000_000, 100_000_000, 0.1)
    assert list(p.min_ns) == [30_000_000, 24_000_000]
    assert list(p.max_ns) == [100_000_000, 80_000_000]
    assert p.fault_threshold == 100
    assert O.random_params(0, 0, 0.999).fault_threshold == 999
    with pytest.raises(ValueError):
        O.random_params(0, 0, 1.5)
    with pytest.raises(ValueError):
        O.random_params(10, 5, 0.1)


def test_ed_kat(golden):
    for p in golden("ed_kat.json")["pairs"]:
        a, b = list(p["a"].encode()), list(p["b"].encode())
        assert O.levenshtein(a, b) == p["d"]
        assert O.levenshtein_py(a, b) == p["d"]
        for w in range(0, 10):
            assert O.levenshtein_banded(a, b, w) == min(p["d"], w + 1)


def test_banded_equals_clamped_full():
    """ED_w = min(D_band, w+1) == min(Levenshtein, w+1) (a path of cost <= w stays in band)."""
    rng = np.random.default_rng(2)
    for _ in range(300):
        a = rng.integers(0, 4, rng.integers(0, 30)).astype(np.uint64)
        b = rng.integers(0, 4, rng.integers(0, 30)).astype(np.uint64)
        full = O.levenshtein_py(list(a), list(b))
        assert O.levenshtein(a, b) == full
        for w in [0, 1, 2, 5, 16]:
            assert O.levenshtein_banded(a, b, w) == min(full, w + 1)


def test_zk_traces_golden(golden):
    z = golden("zk_traces.json")
    seqs = [np.array([int(h, 16) for h in t["evhash"]], np.uint64) for t in z["traces"]]
    assert [len(s) for s in seqs] == [48, 41, 26, 36]
    assert z["distinct_events"] == 38
    n = len(seqs)
    for i in range(n):
        for j in range(n):
            assert O.levenshtein(seqs[i], seqs[j]) == z["levenshtein"][i][j]
            for w, mat in z["banded"].items():
                assert O.levenshtein_banded(seqs[i], seqs[j], int(w)) == mat[i][j]
    # distance 0 <=> equal (SingleTrace.Equals)
    assert all(z["levenshtein"][i][i] == 0 for i in range(n))


def test_knn_bruteforce():
    rng = np.random.default_rng(3)
    traces = [rng.integers(0, 3, rng.integers(0, 12)).astype(np.uint64) for _ in range(15)]
    off = np.zeros(16, np.uint64)
    off[1:] = np.cumsum([len(t) for t in traces])
    sym = np.concatenate(traces)
    for w, k in [(3, 4), (16, 20)]:
        ids, ds = O.ed_allpairs_knn(off, sym, w, k)
        for q in range(15):
            cand = sorted((min(O.levenshtein_py(list(traces[q]), list(traces[c])), w + 1), c)
                          for c in range(15) if c != q)[:k]
            cand += [(0xFFFFFFFF, 0xFFFFFFFF)] * (k - len(cand))
            assert [(int(d), int(i)) for d, i in zip(ds[q], ids[q])] == cand


def test_topk_order():
    st = np.zeros(6, O.SCHED_STATS_DTYPE)
    st["n_fault"] = [1, 3, 3, 0, 3, 1]
    st["sum_delay_ns"] = [5, 7, 9, 100, 9, 5]
    tk = O.topk_from_stats(st, 100, 4)
    assert list(tk["seed"]) == [102, 104, 101, 100]
    tk = O.topk_from_stats(st, 0, 8)
    assert list(tk["seed"][6:]) == [2**64 - 1] * 2


def test_random_rejection_vectors(golden):
    """tests/golden/random_rejections.json: each vector's fault draw is rejected and re-drawn (Go Int31n), after
    one Int63n delay draw (ranged) or none (fixed duration); for any ranged or fixed parameters."""
    g = golden("random_rejections.json")
    for mn, mx in [(30_000_000, 100_000_000), (0, 3_000_000_000)]:
        p = O.random_params(mn, mx, 0.1)
        for eh in g["ranged"]:
            for cls in (2, 3):
                assert O.random_decide(g["seed"], eh, cls, p)[2] == 3
    for mn in [5_000_000, 3_000_000_000]:
        p = O.random_params(mn, mn, 0.1)
        for eh in g["fixed"]:
            for cls in (2, 3):
                assert O.random_decide(g["seed"], eh, cls, p)[2] == 2
