"""Quick GPU parity smoke for K1/K2 against the CPU oracle (dev tool)."""
import sys, time
import numpy as np
sys.path.insert(0, ".")
from oracle import oracle as O
from namazu_amd import _lib
from namazu_amd.explorepolicy import Replayable, Random, to_csr

rng = np.random.default_rng(5)
def hints(n):
    v = rng.integers(-2**63, 2**63 - 1, size=n, dtype=np.int64)
    return [str(int(x)) for x in v]

ok = True
for m in [10**8, 10**9, 0, 2**30 + 5, 2**62 + 11, -5_000_000, 1]:
    p = Replayable(); p.MaxInterval = m
    seeds = [str(i) for i in range(3000)] + ["", "foobar"]
    hs = hints(300) + ["", "a", "hint-entity-0-0"]
    t = time.time(); r = p.Sweep(seeds, hs, n_dump=40, k=8); dt = time.time() - t
    so, sb = O.to_csr(seeds); ho, hb = O.to_csr(hs)
    st, dl = O.replayable_sweep(so, sb, ho, hb, m, n_dump=40)
    eq_s = np.array_equal(r.stats, st); eq_d = np.array_equal(r.delays, dl)
    tk = O.topk_from_stats(st, 0, 8); eq_t = np.array_equal(r.topk, tk)
    print(f"replayable m={m}: stats {eq_s} dump {eq_d} topk {eq_t} ({dt*1e3:.1f} ms)")
    if not (eq_s and eq_d and eq_t):
        ok = False
        bad = np.nonzero(r.stats != st)[0][:3]
        print(" gpu", r.stats[bad], "\n cpu", st[bad])

for (mn, mx, pr) in [(30_000_000, 100_000_000, 0.1), (5_000_000, 5_000_000, 0.5), (0, 2**20, 1.0), (80_000_000, 3_000_000_000, 0.999)]:
    rp = Random(); rp.MinInterval, rp.MaxInterval, rp.FaultActionProbability = mn, mx, pr
    E = 500
    eh = rng.integers(0, 2**64, size=E, dtype=np.uint64)
    ec = rng.integers(0, 4, size=E, dtype=np.uint8)
    t = time.time(); r = rp.Sweep(12345, 700, eh, ec, n_dump=20, k=16); dt = time.time() - t
    params = O.random_params(mn, mx, pr)
    st, dl, fl = O.random_sweep(12345, 700, eh, ec, params, n_dump=20)
    eq_s = np.array_equal(r.stats, st); eq_d = np.array_equal(r.delays, dl) and np.array_equal(r.faults, fl)
    tk = O.topk_from_stats(st, 12345, 16); eq_t = np.array_equal(r.topk, tk)
    print(f"random ({mn},{mx},{pr}): stats {eq_s} dump {eq_d} topk {eq_t} ({dt*1e3:.1f} ms)")
    if not (eq_s and eq_d and eq_t):
        ok = False
        bad = np.nonzero(r.stats != st)[0][:3]
        print(" gpu", r.stats[bad], "\n cpu", st[bad])
        bd = np.argwhere(r.delays != dl)[:3]
        print(" dump mismatch", bd, r.delays[tuple(bd.T)] if len(bd) else None, dl[tuple(bd.T)] if len(bd) else None)

# ---- ED
import ctypes
L = _lib.load(); ctx = _lib.default_context(0)
def ed_allpairs(off, sym, w, k):
    n = len(off) - 1
    ids = np.zeros((n, k), np.uint32); ds = np.zeros((n, k), np.uint32)
    _lib.check(L.nmz_ed_allpairs_knn(ctx.handle, _lib.ptr(off), _lib.ptr(sym), n, w, k, _lib.ptr(ids), _lib.ptr(ds)))
    return ids, ds
def ed_pairs(off, sym, pairs, w):
    d = np.zeros(len(pairs), np.uint32)
    _lib.check(L.nmz_ed_pairs(ctx.handle, _lib.ptr(off), _lib.ptr(sym), len(off) - 1, _lib.ptr(pairs), len(pairs), w, _lib.ptr(d)))
    return d
for (N, Lmin, Lmax, w, mut) in [(70, 0, 40, 8, 0.3), (150, 180, 260, 32, 0.05), (130, 100, 300, 16, 0.02), (97, 1, 70, 32, 0.5)]:
    base = rng.integers(0, 12, size=Lmax)
    traces = []
    for i in range(N):
        l = int(rng.integers(Lmin, Lmax + 1))
        t = base[:l].copy()
        msk = rng.random(l) < mut
        t[msk] = rng.integers(0, 12, size=int(msk.sum()))
        traces.append(t.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(7))
    off = np.zeros(N + 1, np.uint64); off[1:] = np.cumsum([len(t) for t in traces])
    sym = np.concatenate(traces).astype(np.uint64) if off[-1] else np.zeros(1, np.uint64)
    k = 6
    t0 = time.time(); ids, ds = ed_allpairs(off, sym, w, k); dt = time.time() - t0
    oi, od = O.ed_allpairs_knn(off, sym, w, k)
    pairs = rng.integers(0, N, size=(500, 2)).astype(np.uint32)
    dg = ed_pairs(off, sym, pairs, w); dc = O.ed_pairs(off, sym, pairs, w)
    e1 = np.array_equal(ids, oi) and np.array_equal(ds, od); e2 = np.array_equal(dg, dc)
    print(f"ED N={N} L=[{Lmin},{Lmax}] w={w}: knn {e1} pairs {e2} ({dt*1e3:.1f} ms)")
    if not (e1 and e2):
        ok = False
        bad = np.nonzero((ids != oi).any(1) | (ds != od).any(1))[0][:3]
        for b in bad: print("  q", b, "gpu", list(zip(ids[b], ds[b])), "cpu", list(zip(oi[b], od[b])))
        bp = np.nonzero(dg != dc)[0][:5]
        print("  pairs bad", pairs[bp].tolist(), dg[bp], dc[bp])
print("ALL OK" if ok else "MISMATCH")
sys.exit(0 if ok else 1)
