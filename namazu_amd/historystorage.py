"""HistoryStorage surface with GPU similarity search behind it.

Mirrors nmz/historystorage:
  * HistoryStorage interface, New(name, dir), LoadStorage(dir)
        historystorage/historystorage.go:33-83
  * Naive storage layout %08x/actions/N.{action,event}.json, result.json
        historystorage/naive/naive.go:82-233, naive/common.go:24-40
  * Search / SearchWithConverter (exact equality of the converted sequence,
    the latest trace excluded)         naive/naive.go:235-257
and adds the optional SimilaritySearcher interface: banded edit
distance k-NN over event-hash sequences, plus the `nmz tools visualize`
unique-trace count (cli/tools/visualize.go:51-172), exact and partial-order
reduced. The gob-encoded `history`/`SearchModeInfo` files are not read; the
per-action JSON files (naive.go:65-80) carry the same actions and events.

Two symbol streams per stored trace (build-defined), each the FNV-1a
64 of a canonical JSON (Go encoding/json form, namazu_amd/signal.py):
  * action symbols: the action's map without "uuid" -- Action.Equals
    (BasicSignal.EqualsSignal ignores only uuid and arrival time, signal.go:174-186),
    so "event_uuid" counts wherever the layout puts it (top level since
    action_accept_event.go:40; under "option" in the 2015 example traces).
    Search / SearchWithConverter and the exact unique count compare these
    (AreActionsSliceEqual, util/signal/misc.go:22-35). Actions of different runs
    carry different event uuids, so -- as in the reference -- they never match.
  * event symbols: the action's event without "uuid" -- Event.Equals. The
    similarity search (SearchSimilar, AllPairsKNN) and the partial-order unique
    count compare these; an action without an event file uses its action symbol
    there, and has no entity (skipped by the PO projection, visualize.go:67-76).
Every comparison runs in libnmz_gpu.so.
"""
import ctypes
import glob
import json
import os
import re

import numpy as np

from . import _lib
from .config import Config
from .signal import Event, fnv1a64, go_json

STORAGE_TOML = "config.toml"  # historystorage.go:28


class SingleTrace:
    """util/trace.SingleTrace: the stored action sequence.

    symbols         event symbols (Event.Equals; SimilaritySearcher)
    action_symbols  action symbols (Action.Equals; Equals, Search) -- default: symbols
    entities        EntityID() of each action's event, None for an action without one
    events          the events (signal.Event) or None"""

    def __init__(self, symbols, events=None, action_symbols=None, entities=None):
        self.symbols = np.asarray(symbols, np.uint64)
        self.events = events or []
        self.action_symbols = self.symbols if action_symbols is None else np.asarray(action_symbols, np.uint64)
        self.entities = entities if entities is not None else [None] * len(self.symbols)

    def __len__(self):
        return len(self.symbols)

    def Equals(self, other):
        """trace.go:29-31 -> AreActionsSliceEqual (misc.go:22-35): equal length, element-wise Action.Equals."""
        return len(self.action_symbols) == len(other.action_symbols) and \
            bool(np.array_equal(self.action_symbols, other.action_symbols))


def action_symbol(action_json):
    """Symbol of an action map: FNV-1a 64 of its canonical JSON without "uuid" (EqualsSignal keeps every
    other key, including "event_uuid" at whichever level it is stored)."""
    return fnv1a64(go_json({k: v for k, v in action_json.items() if k != "uuid"}).encode())


def action_symbols(actions):
    """[]Action (signal.Action objects or JSON maps) -> uint64 action symbols."""
    return np.array([action_symbol(a.JSONMap() if hasattr(a, "JSONMap") else a) for a in actions], np.uint64)


class TraceSet:
    """CSR of event-hash sequences, the layout the GPU kernels consume."""

    def __init__(self, traces):
        self.off = np.zeros(len(traces) + 1, np.uint64)
        if traces:
            self.off[1:] = np.cumsum([len(t) for t in traces])
        self.sym = (np.concatenate([np.asarray(t, np.uint64) for t in traces])
                    if self.off[-1] else np.zeros(1, np.uint64))

    def __len__(self):
        return len(self.off) - 1

    def trace(self, i):
        return self.sym[int(self.off[i]):int(self.off[i + 1])]


class HistoryStorage:
    def Name(self):
        raise NotImplementedError


class Naive(HistoryStorage):
    """Reader for the naive storage directory layout."""

    def __init__(self, dir_path):
        self.dir = dir_path
        self._ids = None

    def Name(self):
        return "naive"

    def Init(self):
        ids = []
        for p in glob.glob(os.path.join(self.dir, "*")):
            b = os.path.basename(p)
            if os.path.isdir(p) and re.fullmatch(r"[0-9a-f]{8}", b):
                ids.append(int(b, 16))
        self._ids = sorted(ids)

    def NrStoredHistories(self):
        if self._ids is None:
            self.Init()
        return len(self._ids)

    def _run_dir(self, i):
        return os.path.join(self.dir, "%08x" % i)

    def GetStoredHistory(self, i):
        """Returns (SingleTrace, error) like the Go getter."""
        adir = os.path.join(self._run_dir(i), "actions")
        if not os.path.isdir(adir):
            return None, FileNotFoundError(adir)
        idx = sorted(int(m.group(1)) for f in os.listdir(adir)
                     if (m := re.fullmatch(r"(\d+)\.action\.json", f)))
        syms, asyms, ents, evs = [], [], [], []
        for n in idx:
            with open(os.path.join(adir, f"{n}.action.json")) as f:
                asym = action_symbol(json.load(f))
            asyms.append(asym)
            ep = os.path.join(adir, f"{n}.event.json")
            if os.path.exists(ep):  # recordAction writes it iff act.Event() != nil (naive.go:72-79)
                with open(ep) as f:
                    ev = Event.from_json(f.read())
                syms.append(ev.evhash())
                ents.append(ev.EntityID())
                evs.append(ev)
            else:
                syms.append(asym)
                ents.append(None)
                evs.append(None)
        return SingleTrace(syms, evs, action_symbols=asyms, entities=ents), None

    def IsSuccessful(self, i):
        try:
            return bool(json.load(open(os.path.join(self._run_dir(i), "result.json")))["successful"]), None
        except Exception as e:  # getters return errors (naive.go:199-213)
            return False, e

    def GetRequiredTime(self, i):
        try:
            return int(json.load(open(os.path.join(self._run_dir(i), "result.json")))["required_time"]), None
        except Exception as e:
            return 0, e

    def traces(self):
        out = []
        for i in range(self.NrStoredHistories()):
            t, err = self.GetStoredHistory(i)
            if err is not None:
                raise RuntimeError(f"failed to get history {i}: {err}")  # naive.go:241 panics
            out.append(t)
        return out

    def load_all(self):
        """Event-symbol TraceSet of every stored trace (the SimilaritySearcher's input)."""
        return TraceSet([t.symbols for t in self.traces()])

    # ---- search surface (GPU) ------------------------------------------------
    def SearchWithConverter(self, prefix, converter):
        """naive.go:235-252: ids i < NrStoredHistories-1 (the latest trace is excluded, :238) with
        len(trace) >= len(prefix) whose converted trace equals `prefix` under AreActionsSliceEqual
        (equal length, element-wise Action.Equals: action symbols). `prefix`: a SingleTrace, a list of
        actions (signal.Action or JSON maps), or action symbols; `converter`: SingleTrace -> SingleTrace
        (the reference's func([]Action) []Action)."""
        n = self.NrStoredHistories() - 1
        if n <= 0:
            return []
        if isinstance(prefix, SingleTrace):
            p = prefix.action_symbols
        elif len(prefix) and (hasattr(prefix[0], "JSONMap") or isinstance(prefix[0], dict)):
            p = action_symbols(prefix)
        else:
            p = np.asarray(prefix, np.uint64)
        cands = []
        for i in range(n):
            t, err = self.GetStoredHistory(i)
            if err is not None:
                raise RuntimeError(f"failed to get history {i}: {err}")
            if len(t) < len(p):
                continue
            cands.append((i, converter(t)))
        if not cands:
            return []
        ts = TraceSet([p] + [c.action_symbols for _, c in cands])
        pairs = np.array([[0, j + 1] for j in range(len(cands))], np.uint32)
        d = ed_pairs(ts, pairs, band=0)  # band 0: 0 iff equal length and element-wise equal
        return [cands[j][0] for j in range(len(cands)) if d[j] == 0]

    def Search(self, prefix):
        """naive.go:254-257: SearchWithConverter with the identity converter."""
        return self.SearchWithConverter(prefix, lambda t: t)

    def UniqueTraceCurve(self, po_reduction=True):
        """`nmz tools visualize -mode gnuplot` (visualize.go:138-172): nrUniques after each stored trace;
        po_reduction defaults to true as the flag does (:42)."""
        return unique_trace_curve(self.traces(), po_reduction=po_reduction)

    # ---- SimilaritySearcher ----------------------------------------------------
    def SearchSimilar(self, trace, k, band):
        """k nearest stored traces to `trace` by (distance asc, id asc), as [(id, distance)].

        The stored traces are read once and stay on the GPU (SimilarityIndex) until the storage holds a
        different number of traces; each query is one launch against the resident store."""
        t = trace.symbols if isinstance(trace, SingleTrace) else np.asarray(trace, np.uint64)
        n = self.NrStoredHistories()
        key = (band, n)
        if getattr(self, "_index_key", None) != key:
            if getattr(self, "_index", None) is not None:
                self._index.close()
            self._index = SimilarityIndex(self.load_all(), band)
            self._index_key = key
        ids, ds = self._index.query([t], k)
        return [(int(i), int(d)) for i, d in zip(ids[0], ds[0]) if i != _lib.NMZ_NONE]

    def AllPairsKNN(self, k, band):
        return allpairs_knn(self.load_all(), k, band)


def New(name, dir_path):
    """historystorage.go:54-62. Returns (storage, error)."""
    if name == "naive":
        return Naive(dir_path), None
    if name == "mongodb":
        return None, NotImplementedError("mongodb storage is out of scope (SURVEY 2 #8)")
    return None, ValueError(f"unknown history storage: {name}")


def LoadStorage(dir_path):
    """historystorage.go:64-83."""
    try:
        cfg = Config.from_file(os.path.join(dir_path, STORAGE_TOML))
    except Exception as e:
        print(f"error: {e}")
        return None
    if cfg.get("storageType") == "naive":
        return Naive(dir_path)
    print(f"unknown history storage: {cfg.get('storageType')}")
    return None


# ---- GPU entry points ----------------------------------------------------------
def ed_pairs(ts, pairs, band, ctx=None):
    ctx = ctx or _lib.default_context()
    pairs = np.ascontiguousarray(pairs, np.uint32).reshape(-1, 2)
    dist = np.zeros(len(pairs), np.uint32)
    _lib.check(_lib.load().nmz_ed_pairs(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), len(ts),
                                        _lib.ptr(pairs), len(pairs), int(band), _lib.ptr(dist)))
    return dist


class SimilarityIndex:
    """A stored TraceSet resident on the GPU for single-query similarity search (SearchSimilar).

    Every band and plan kind answers through one nmz_ed_plan_query_knn call over the resident store: the
    bit-parallel query kernel (band <= 64), the wide-band query kernel (64 < band <= 8,192: each query's match
    table built once per call, one wave per (query, stored trace)), or the resident generic kernel (other plans,
    queries whose symbols overflow the compact tables, and queries longer than every stored trace)."""

    def __init__(self, ts, band, ctx=None):
        import ctypes
        self.ctx = ctx or _lib.default_context()
        self.ts = ts
        self.band = int(band)
        self.plan = ctypes.c_void_p()
        L = _lib.load()
        _lib.check(L.nmz_ed_plan_create(self.ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), len(ts), self.band,
                                        ctypes.byref(self.plan)))
        self.kind = {3: "wide", 2: "bitparallel", 1: "tile", 0: "generic"}[L.nmz_ed_plan_is_fast(self.plan)]
        self.bitparallel = self.kind == "bitparallel"

    def query(self, queries, k):
        """queries: event-symbol arrays -> (ids [n, k], dists [n, k]) by (ED_band asc, id asc), NMZ_NONE padded."""
        n, N = len(queries), len(self.ts)
        ids = np.full((n, k), _lib.NMZ_NONE, np.uint32)
        ds = np.full((n, k), _lib.NMZ_NONE, np.uint32)
        if n == 0 or N == 0 or k == 0:
            return ids, ds
        if k > 64:
            return self._query_pairs(queries, k)
        qset = TraceSet([np.asarray(q, np.uint64) for q in queries])
        _lib.check(_lib.load().nmz_ed_plan_query_knn(self.plan, _lib.ptr(qset.off), _lib.ptr(qset.sym), n, k,
                                                      _lib.ptr(ids), _lib.ptr(ds)))
        return ids, ds

    def _query_pairs(self, queries, k):
        """k > 64 (the resident kernels keep at most 64 per query; the reference's search has no cap,
        naive.go:235): every (query, stored trace) distance through nmz_ed_pairs on the GPU, one call per query,
        ordered by (distance, id) on the host."""
        n, N = len(queries), len(self.ts)
        kk = min(k, N)
        ids = np.full((n, k), _lib.NMZ_NONE, np.uint32)
        ds = np.full((n, k), _lib.NMZ_NONE, np.uint32)
        stored = [self.ts.trace(i) for i in range(N)]
        pairs = np.stack([np.zeros(N, np.uint32), np.arange(1, N + 1, dtype=np.uint32)], 1)
        for r, q in enumerate(queries):
            both = TraceSet([np.asarray(q, np.uint64)] + stored)
            d = ed_pairs(both, pairs, self.band, ctx=self.ctx)
            order = np.lexsort((np.arange(N), d))[:kk]
            ids[r, :kk] = order
            ds[r, :kk] = d[order]
        return ids, ds

    def close(self):
        if self.plan:
            _lib.load().nmz_ed_plan_destroy(self.plan)
            self.plan = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def allpairs_knn(ts, k, band, ctx=None):
    ctx = ctx or _lib.default_context()
    n = len(ts)
    ids = np.zeros((n, k), np.uint32)
    ds = np.zeros((n, k), np.uint32)
    _lib.check(_lib.load().nmz_ed_allpairs_knn(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), n, int(band),
                                               int(k), _lib.ptr(ids), _lib.ptr(ds)))
    return ids, ds


def po_inputs(traces):
    """Partial-order projection inputs of SingleTraces: CSR of event symbols and per-element entity ids,
    dense per trace in order of first appearance (the kernel needs per-trace counters only: an event
    symbol already determines its entity), NMZ_NONE for actions without an event."""
    ts = TraceSet([t.symbols for t in traces])
    ent = np.full(max(int(ts.off[-1]), 1), _lib.NMZ_NONE, np.uint32)
    pos = 0
    for t in traces:
        ids = {}
        for e in t.entities:
            if e is not None:
                ent[pos] = ids.setdefault(e, len(ids))
            pos += 1
    return ts, ent


def first_equal(traces, po_reduction=True, ctx=None):
    """first_equal[i] = the smallest j with trace j equal to trace i (exact: Equals on action symbols;
    PO: tracesEqualInPO on per-entity event sequences), computed by nmz_unique_traces."""
    ctx = ctx or _lib.default_context()
    if isinstance(traces, TraceSet):
        ts, ent = traces, None
    elif po_reduction:
        ts, ent = po_inputs(traces)
    else:
        ts, ent = TraceSet([t.action_symbols for t in traces]), None
    n = len(ts)
    out = np.zeros(max(n, 1), np.uint32)
    _lib.check(_lib.load().nmz_unique_traces(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), _lib.ptr(ent), n,
                                             _lib.ptr(out)))
    return out[:n]


def unique_trace_curve(traces, po_reduction=True, ctx=None):
    """visualize.go gnuplot mode (:138-172): after trace i, how many distinct traces have been seen.
    traces: SingleTraces (exact or PO mode), or a TraceSet (exact mode over its symbols)."""
    fe = first_equal(traces, po_reduction, ctx)
    return list(np.cumsum(fe == np.arange(len(fe))).astype(int))
