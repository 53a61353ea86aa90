"""CPU ORACLE -- test infrastructure only.

ctypes front end to oracle/nmz_oracle.c plus tiny pure-Python restatements used
to cross-check it. Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker / baseline,
never as the thing measured or shipped. The product (namazu_amd/) must not
import it.

Reference semantics followed (paths relative to the reference's nmz/):
  replayable   explorepolicy/replayable/replayablepolicy.go:100-114
  random       explorepolicy/random/randompolicy.go:300-316,332-346,
               util/queue/impl.go:35-46,94-128
  fnv          Go 1.10 hash/fnv New64a (not vendored; pinned by KATs)
  math/rand    Go 1.10 math/rand rng.go / rand.go (not vendored; pinned by
               the published seed-1 KATs in tests/test_oracle.py)
  trace eq.    util/trace/trace.go:29-31, util/signal/misc.go:22-35
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libnmz_oracle.so")

NONE32 = 0xFFFFFFFF

SCHED_STATS_DTYPE = np.dtype([
    ("sum_delay_ns", "<u8"), ("max_delay_ns", "<i8"), ("argmax_event", "<u4"),
    ("n_fault", "<u4"), ("first_fault", "<u4"), ("flags", "<u4")])
TOPK_DTYPE = np.dtype([("seed", "<u8"), ("sum_delay_ns", "<i8"), ("n_fault", "<u4"),
                       ("first_fault", "<u4")])


class RandomParams(ctypes.Structure):
    _fields_ = [("min_ns", ctypes.c_int64 * 2), ("max_ns", ctypes.c_int64 * 2),
                ("fault_threshold", ctypes.c_int32), ("reserved", ctypes.c_uint32)]


class GoRng(ctypes.Structure):
    _fields_ = [("tap", ctypes.c_int), ("feed", ctypes.c_int), ("n_out", ctypes.c_int64),
                ("vec", ctypes.c_uint64 * 607)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        u64, i64, u32, i32 = ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint32, ctypes.c_int32
        sz = ctypes.c_size_t
        L.nmzo_fnv1a64.restype = u64
        L.nmzo_fnv1a64.argtypes = [P, sz]
        L.nmzo_fnv1a64_update.restype = u64
        L.nmzo_fnv1a64_update.argtypes = [u64, P, sz]
        L.nmzo_init.argtypes = []
        L.nmzo_go_rng_cooked.argtypes = [P]
        L.nmzo_go_seed.argtypes = [P, i64]
        L.nmzo_go_uint64.restype = u64
        L.nmzo_go_uint64.argtypes = [P]
        L.nmzo_go_int63.restype = i64
        L.nmzo_go_int63.argtypes = [P]
        L.nmzo_go_int63n.restype = i64
        L.nmzo_go_int63n.argtypes = [P, i64]
        L.nmzo_go_int31n.restype = i32
        L.nmzo_go_int31n.argtypes = [P, i32]
        L.nmzo_go_intn.restype = i64
        L.nmzo_go_intn.argtypes = [P, i64]
        L.nmzo_replayable_interval.restype = i64
        L.nmzo_replayable_interval.argtypes = [P, sz, P, sz, i64]
        L.nmzo_replayable_sweep.argtypes = [P, P, u64, P, P, u32, i64, P, P, u64, ctypes.c_int]
        L.nmzo_random_params.restype = ctypes.c_int
        L.nmzo_random_params.argtypes = [i64, i64, ctypes.c_double, P]
        L.nmzo_random_event_seed.restype = i64
        L.nmzo_random_event_seed.argtypes = [u64, u64]
        L.nmzo_random_decide.restype = ctypes.c_int
        L.nmzo_random_decide.argtypes = [u64, u64, ctypes.c_uint8, P, P, P]
        L.nmzo_random_sweep.argtypes = [u64, u64, P, P, u32, P, P, P, P, u64, ctypes.c_int]
        L.nmzo_topk_from_stats.argtypes = [P, u64, u64, u32, P]
        L.nmzo_levenshtein.restype = u64
        L.nmzo_levenshtein.argtypes = [P, u64, P, u64]
        L.nmzo_levenshtein_banded.restype = u32
        L.nmzo_levenshtein_banded.argtypes = [P, u64, P, u64, u32]
        L.nmzo_ed_pairs.argtypes = [P, P, P, u64, u32, P, ctypes.c_int]
        L.nmzo_ed_allpairs_knn.argtypes = [P, P, u32, u32, u32, P, P, ctypes.c_int]
        L.nmzo_init()
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------- primitives
def fnv1a64(data: bytes) -> int:
    buf = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, np.uint8)
    return lib().nmzo_fnv1a64(_p(buf), len(data))


def fnv1a64_py(data: bytes) -> int:
    """Pure-Python restatement (cross-check of the C oracle)."""
    h = 0xCBF29CE484222325
    for b in data:
        h = ((h ^ b) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def go_rng_cooked():
    out = np.zeros(607, np.int64)
    lib().nmzo_go_rng_cooked(_p(out))
    return out


class GoRand:
    """rand.New(rand.NewSource(seed)) restated in C."""

    def __init__(self, seed: int):
        self._r = GoRng()
        lib().nmzo_go_seed(ctypes.byref(self._r), seed)

    def uint64(self):
        return lib().nmzo_go_uint64(ctypes.byref(self._r))

    def int63(self):
        return lib().nmzo_go_int63(ctypes.byref(self._r))

    def int63n(self, n):
        return lib().nmzo_go_int63n(ctypes.byref(self._r), n)

    def int31n(self, n):
        return lib().nmzo_go_int31n(ctypes.byref(self._r), n)

    def intn(self, n):
        return lib().nmzo_go_intn(ctypes.byref(self._r), n)

    @property
    def n_out(self):
        return self._r.n_out


# ---------------------------------------------------------------- CSR helpers
def to_csr(strings):
    bs = [s.encode() if isinstance(s, str) else bytes(s) for s in strings]
    off = np.zeros(len(bs) + 1, np.uint32)
    off[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    data = np.frombuffer(b"".join(bs), np.uint8).copy() if off[-1] else np.zeros(1, np.uint8)
    return off, data


# ---------------------------------------------------------------- replayable
def replayable_interval(seed: str, hint: str, max_interval_ns: int) -> int:
    s, h = seed.encode(), hint.encode()
    sb = np.frombuffer(s, np.uint8) if s else np.zeros(1, np.uint8)
    hb = np.frombuffer(h, np.uint8) if h else np.zeros(1, np.uint8)
    return lib().nmzo_replayable_interval(_p(sb), len(s), _p(hb), len(h), max_interval_ns)


def replayable_sweep(seed_off, seed_bytes, hint_off, hint_bytes, max_interval_ns, n_dump=0,
                     nthreads=0):
    n_seeds, n_events = len(seed_off) - 1, len(hint_off) - 1
    stats = np.zeros(n_seeds, SCHED_STATS_DTYPE)
    delays = np.zeros((max(n_dump, 0), n_events), np.int64) if n_dump else None
    lib().nmzo_replayable_sweep(_p(seed_off), _p(seed_bytes), n_seeds, _p(hint_off),
                                _p(hint_bytes), n_events, max_interval_ns, _p(stats),
                                _p(delays), n_dump, nthreads)
    return stats, delays


# ---------------------------------------------------------------- random
def random_params(min_ns, max_ns, probability):
    p = RandomParams()
    rc = lib().nmzo_random_params(min_ns, max_ns, probability, ctypes.byref(p))
    if rc != 0:
        raise ValueError("bad random-policy parameters")
    return p


def random_event_seed(seed, evhash):
    return lib().nmzo_random_event_seed(seed, evhash)


def random_decide(seed, evhash, evclass, params):
    d = ctypes.c_int64()
    f = ctypes.c_int()
    n = lib().nmzo_random_decide(seed, evhash, evclass, ctypes.byref(params), ctypes.byref(d),
                                 ctypes.byref(f))
    return d.value, bool(f.value), n


def random_sweep(seed0, n_seeds, evhash, evclass, params, n_dump=0, nthreads=0):
    evhash = np.ascontiguousarray(evhash, np.uint64)
    evclass = np.ascontiguousarray(evclass, np.uint8)
    n_events = len(evhash)
    stats = np.zeros(n_seeds, SCHED_STATS_DTYPE)
    delays = np.zeros((n_dump, n_events), np.int64) if n_dump else None
    faults = np.zeros((n_dump, n_events), np.uint8) if n_dump else None
    lib().nmzo_random_sweep(seed0, n_seeds, _p(evhash), _p(evclass), n_events,
                            ctypes.byref(params), _p(stats), _p(delays), _p(faults), n_dump,
                            nthreads)
    return stats, delays, faults


def topk_from_stats(stats, seed0, k):
    out = np.zeros(k, TOPK_DTYPE)
    lib().nmzo_topk_from_stats(_p(np.ascontiguousarray(stats)), len(stats), seed0, k, _p(out))
    return out


# ---------------------------------------------------------------- trace distance
def levenshtein(a, b):
    a = np.ascontiguousarray(a, np.uint64)
    b = np.ascontiguousarray(b, np.uint64)
    return lib().nmzo_levenshtein(_p(a), len(a), _p(b), len(b))


def levenshtein_banded(a, b, w):
    a = np.ascontiguousarray(a, np.uint64)
    b = np.ascontiguousarray(b, np.uint64)
    return lib().nmzo_levenshtein_banded(_p(a), len(a), _p(b), len(b), w)


def levenshtein_py(a, b):
    """Pure-Python full Levenshtein (small cases only)."""
    prev = list(range(len(b) + 1))
    for i in range(1, len(a) + 1):
        cur = [i] + [0] * len(b)
        for j in range(1, len(b) + 1):
            cur[j] = min(prev[j - 1] + (a[i - 1] != b[j - 1]), prev[j] + 1, cur[j - 1] + 1)
        prev = cur
    return prev[-1]


def ed_pairs(off, sym, pairs, w, nthreads=0):
    pairs = np.ascontiguousarray(pairs, np.uint32).reshape(-1, 2)
    dist = np.zeros(len(pairs), np.uint32)
    lib().nmzo_ed_pairs(_p(np.ascontiguousarray(off, np.uint64)),
                        _p(np.ascontiguousarray(sym, np.uint64)), _p(pairs), len(pairs), w,
                        _p(dist), nthreads)
    return dist


def ed_allpairs_knn(off, sym, w, k, nthreads=0):
    n = len(off) - 1
    ids = np.zeros((n, k), np.uint32)
    ds = np.zeros((n, k), np.uint32)
    lib().nmzo_ed_allpairs_knn(_p(np.ascontiguousarray(off, np.uint64)),
                               _p(np.ascontiguousarray(sym, np.uint64)), n, w, k, _p(ids),
                               _p(ds), nthreads)
    return ids, ds


# ---------------------------------------------------------------- visualize uniqueness (pure Python, literal)
def unique_curve_exact(traces):
    """`nmz tools visualize` without PO reduction (cli/tools/visualize.go:51-60,138-172): for i in order,
    seenBefore(uniqueTraces, trace_i) = any stored unique trace Equals it (SingleTrace.Equals ->
    AreActionsSliceEqual: equal length + element-wise Action.Equals, util/signal/misc.go:22-35).
    traces: sequences of action symbols (equal symbols <=> Action.Equals). Returns the printed
    nrUniques column, one entry per trace."""
    uniques, out = [], []
    for t in traces:
        t = [int(x) for x in t]
        seen = False
        for u in uniques:  # seenBefore
            if len(u) == len(t) and all(a == b for a, b in zip(u, t)):
                seen = True
                break
        if not seen:
            uniques.append(t)
        out.append(len(uniques))
    return out


def unique_curve_po(traces):
    """`nmz tools visualize` with PO reduction, the default (visualize.go:42,62-136,158-159).
    traces: sequences of (entity, event_symbol) per action, entity None for an action without an event
    (act.Event() == nil: skipped by createTracesPerEntity). Equal event symbols <=> Event.Equals."""
    def per_entity(t):  # createTracesPerEntity (:62-79)
        m = {}
        for ent, ev in t:
            if ent is not None:
                m.setdefault(ent, []).append(int(ev))
        return m

    def equal_in_po(a, b):  # tracesEqualInPO (:81-124)
        ea, eb = sorted(a), sorted(b)
        if len(ea) != len(eb):
            return False
        for x, y in zip(ea, eb):
            if x != y:
                return False
        for ent in ea:
            if len(a[ent]) != len(b[ent]):
                return False
            for x, y in zip(a[ent], b[ent]):
                if x != y:
                    return False
        return True

    uniques, out = [], []
    for t in traces:
        u = per_entity(t)
        if not any(equal_in_po(v, u) for v in uniques):  # seenBeforePOR (:126-136)
            uniques.append(u)
        out.append(len(uniques))
    return out
