"""Synthetic inputs shaped like BASELINE.json's configs (no datasets here).

* zk_hints: replay hints in pynmz's format (misc/pynmz/inspector/zookeeper.py:113,
  str(hash(frozenset(...))) = decimal signed int64), from SplitMix64.
* etcd_traces: configs[4] long traces -- 64 event symbols (etcd raft
  messages x members), transpositions 1%, substitutions 0.3%, so pair
  distances (~0.046 per event, ~3000 at 65,536 events) stay inside w = 4096.
* synth_traces: SURVEY 8(d) config 3 -- a ZooKeeper-style Markov base sequence
  over 48 event symbols (the stored example traces hold 38 distinct events),
  each trace = base + adjacent transpositions at 2% + substitutions at 0.5%,
  fixed length; symbols are 64-bit event hashes. Independent mutations at these
  rates put every pair ~150-175 edits apart, past w = 32: a search workload in
  which nothing is near anything else.
* clustered_traces: configs[2] as a search workload -- the same base, split
  into families. A family's parent is the base mutated at the survey rates;
  each member is its parent plus a few edits (Poisson-many adjacent
  transpositions and substitutions), as repeated runs of one schedule differ
  by a few reordered or changed events. Members of one family are a few edits
  apart (inside w = 32), families ~150 edits apart, so with families of
  `family` traces about (family-1)/(n-1) of all pairs fall inside the band.
"""
import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(seed, n):
    """Vectorised SplitMix64 stream (state += golden; finalize)."""
    with np.errstate(over="ignore"):
        s = np.uint64(seed) + GOLDEN * np.arange(1, n + 1, dtype=np.uint64)
        z = (s ^ (s >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def zk_hints(n, seed=0x5EED):
    return [str(int(x)) for x in splitmix64(seed, n).view(np.int64)]


def _markov_base(length, n_symbols, rng):
    succ = rng.integers(0, n_symbols, size=(n_symbols, 4))
    out = np.empty(length, np.int64)
    s = int(rng.integers(0, n_symbols))
    for i in range(length):
        out[i] = s
        s = int(succ[s, rng.integers(0, 4)]) if rng.random() < 0.9 else int(rng.integers(0, n_symbols))
    return out


def synth_traces(n, length, seed=0x5EED, n_symbols=48, p_transpose=0.02, p_subst=0.005):
    """Returns a historystorage.TraceSet of n traces of `length` event hashes."""
    from .historystorage import TraceSet
    rng = np.random.default_rng(seed)
    base = _markov_base(length, n_symbols, rng)
    sym_hash = splitmix64(seed ^ 0xABCDEF, n_symbols)
    ts = TraceSet([])
    ts.off = np.arange(n + 1, dtype=np.uint64) * np.uint64(length)
    ids = np.empty((n, length), np.int64)
    chunk = 4096
    for c0 in range(0, n, chunk):
        c = min(chunk, n - c0)
        t = np.broadcast_to(base, (c, length)).copy()
        # adjacent transpositions (non-overlapping: drop a swap right after another)
        sw = rng.random((c, length - 1)) < p_transpose
        sw[:, 1:] &= ~sw[:, :-1]
        r, i = np.nonzero(sw)
        a = t[r, i].copy()
        t[r, i] = t[r, i + 1]
        t[r, i + 1] = a
        sub = rng.random((c, length)) < p_subst
        t[sub] = rng.integers(0, n_symbols, size=int(sub.sum()))
        ids[c0:c0 + c] = t
    ts.sym = sym_hash[ids.reshape(-1)]
    return ts


def etcd_traces(n, length, seed=0xE7CD):
    """configs[4]: n etcd-style traces of `length` events (see module docstring)."""
    return synth_traces(n, length, seed=seed, n_symbols=64, p_transpose=0.01, p_subst=0.003)


def clustered_traces(n, length, seed=0x5EED, n_symbols=48, family=1024, edits_mean=6.0,
                     p_transpose=0.02, p_subst=0.005, alphabet_total=None):
    """configs[2] search workload: n traces in families of `family` near-duplicates (module docstring).
    Trace i belongs to family i // family (contiguous ids). Returns a historystorage.TraceSet.
    alphabet_total: each family's events are its own `n_symbols` symbols drawn from a store-wide alphabet of
    that many (different scenarios record different event maps, SURVEY A11: every distinct event map is a
    symbol), so the store holds thousands of distinct symbols while a trace holds at most n_symbols."""
    from .historystorage import TraceSet
    rng = np.random.default_rng(seed)
    base = _markov_base(length, n_symbols, rng)
    n_fam0 = max(1, -(-n // family))
    if alphabet_total:
        fmap = np.stack([rng.choice(alphabet_total, n_symbols, replace=False) for _ in range(n_fam0)])
        sym_hash = splitmix64(seed ^ 0xABCDEF, alphabet_total)
    else:
        fmap = None
        sym_hash = splitmix64(seed ^ 0xABCDEF, n_symbols)
    n_fam = max(1, -(-n // family))
    parents = np.broadcast_to(base, (n_fam, length)).copy()
    _mutate(parents, rng, n_symbols, p_transpose, p_subst)
    ids = np.empty((n, length), np.int64)
    chunk = 4096
    for c0 in range(0, n, chunk):
        c = min(chunk, n - c0)
        t = parents[np.arange(c0, c0 + c) // family].copy()
        # a few edits per member: Poisson(edits_mean) events, each an adjacent transposition or a substitution
        k = rng.poisson(edits_mean, c)
        rows = np.repeat(np.arange(c), k)
        pos = rng.integers(0, max(length - 1, 1), rows.size)
        swap = rng.random(rows.size) < 0.5
        r, i = rows[swap], pos[swap]
        if length > 1:
            a = t[r, i].copy()
            t[r, i] = t[r, i + 1]
            t[r, i + 1] = a
        r, i = rows[~swap], pos[~swap]
        t[r, i] = rng.integers(0, n_symbols, size=r.size)
        if fmap is not None:  # local symbols -> the family's store-wide ids
            t = fmap[(np.arange(c0, c0 + c) // family)[:, None], t]
        ids[c0:c0 + c] = t
    ts = TraceSet([])
    ts.off = np.arange(n + 1, dtype=np.uint64) * np.uint64(length)
    ts.sym = sym_hash[ids.reshape(-1)]
    return ts


def _mutate(t, rng, n_symbols, p_transpose, p_subst):
    """In place: non-overlapping adjacent transpositions at p_transpose, then substitutions at p_subst."""
    c, length = t.shape
    if length > 1:
        sw = rng.random((c, length - 1)) < p_transpose
        sw[:, 1:] &= ~sw[:, :-1]
        r, i = np.nonzero(sw)
        a = t[r, i].copy()
        t[r, i] = t[r, i + 1]
        t[r, i + 1] = a
    sub = rng.random((c, length)) < p_subst
    t[sub] = rng.integers(0, n_symbols, size=int(sub.sum()))


def po_store(n, length, n_entities=16, p_reorder=0.5, p_new=0.3, seed=0x5EED):
    """`nmz tools visualize` workload: n stored runs of `length` events over `n_entities` entities (each entity
    `length // n_entities` events).

    A run is either new (probability p_new: fresh per-entity event sequences) or a repeat of an earlier run's
    per-entity sequences, re-interleaved across entities with probability p_reorder (partial-order equal,
    not exactly equal) or in the same interleaving (exactly equal). Returns (TraceSet of event symbols,
    entity ids uint32 per element (dense per trace), number of distinct runs by construction)."""
    from .historystorage import TraceSet
    rng = np.random.default_rng(seed)
    per = length // n_entities
    length = per * n_entities
    ent_of = np.repeat(np.arange(n_entities, dtype=np.uint16), per)
    base_of = np.empty(n, np.int64)
    orders = np.empty((n, length), np.int64)
    n_bases = 0
    first_order = {}
    for i in range(n):
        if n_bases == 0 or rng.random() < p_new:
            base_of[i] = n_bases
            n_bases += 1
            orders[i] = rng.permutation(length)
            first_order[int(base_of[i])] = i
        else:
            base_of[i] = rng.integers(n_bases)
            orders[i] = rng.permutation(length) if rng.random() < p_reorder else orders[first_order[int(base_of[i])]]
    ev = rng.integers(0, 64, (n_bases, n_entities, per)).astype(np.uint64)
    slot_ent = ent_of[orders].astype(np.uint16)                 # (n, length) entity of each slot
    srt = np.argsort(slot_ent, axis=1, kind="stable")           # slots grouped by entity, in slot order (radix)
    rank = np.empty_like(srt)
    np.put_along_axis(rank, srt, np.tile(np.arange(length) % per, (n, 1)), axis=1)
    sym = ev[base_of[:, None], slot_ent, rank] * np.uint64(0x9E3779B97F4A7C15) + \
        slot_ent.astype(np.uint64) * np.uint64(0xBF58476D1CE4E5B9) + np.uint64(1)
    ts = TraceSet([])
    ts.off = np.arange(n + 1, dtype=np.uint64) * np.uint64(length)
    ts.sym = sym.reshape(-1)
    return ts, slot_ent.astype(np.uint32).reshape(-1), n_bases
