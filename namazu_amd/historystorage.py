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
unique-trace count (cli/tools/visualize.go:51-60,138-172) as distance-0
detection. The gob-encoded `history`/`SearchModeInfo` files are not read;
the per-action JSON files carry the same events.

Trace symbols (build-defined): the FNV-1a 64 of the canonical
JSON of each action's event without "uuid" (Event.Equals semantics); actions
without an event file use their own JSON without "uuid"/"event_uuid".
Every distance is computed by libnmz_gpu.so.
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
    """util/trace.SingleTrace: the stored action sequence (events of each action)."""

    def __init__(self, symbols, events=None):
        self.symbols = np.asarray(symbols, np.uint64)
        self.events = events or []

    def __len__(self):
        return len(self.symbols)

    def Equals(self, other):
        return len(self) == len(other) and bool(np.array_equal(self.symbols, other.symbols))


def _action_symbol(action_json):
    m = {k: v for k, v in action_json.items() if k != "uuid"}
    if isinstance(m.get("option"), dict):
        m["option"] = {k: v for k, v in m["option"].items() if k != "event_uuid"}
    return fnv1a64(go_json(m).encode())


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
        syms, evs = [], []
        for n in idx:
            ep = os.path.join(adir, f"{n}.event.json")
            if os.path.exists(ep):
                ev = Event.from_json(open(ep).read())
                syms.append(ev.evhash())
                evs.append(ev)
            else:
                syms.append(_action_symbol(json.load(open(os.path.join(adir, f"{n}.action.json")))))
                evs.append(None)
        return SingleTrace(syms, evs), None

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

    def load_all(self):
        traces = []
        for i in range(self.NrStoredHistories()):
            t, err = self.GetStoredHistory(i)
            if err is not None:
                raise RuntimeError(f"failed to get history {i}: {err}")  # naive.go:241 panics
            traces.append(t.symbols)
        return TraceSet(traces)

    # ---- search surface (GPU) ------------------------------------------------
    def SearchWithConverter(self, prefix, converter):
        """naive.go:235-252: ids i < NrStoredHistories-1 whose converted trace equals prefix."""
        n = self.NrStoredHistories() - 1
        if n <= 0:
            return []
        cands = []
        for i in range(n):
            t, err = self.GetStoredHistory(i)
            if err is not None:
                raise RuntimeError(f"failed to get history {i}: {err}")
            if len(t) < len(prefix):
                continue
            cands.append((i, converter(t)))
        if not cands:
            return []
        p = prefix.symbols if isinstance(prefix, SingleTrace) else np.asarray(prefix, np.uint64)
        ts = TraceSet([p] + [c.symbols for _, c in cands])
        pairs = np.array([[0, j + 1] for j in range(len(cands))], np.uint32)
        d = ed_pairs(ts, pairs, band=0)
        return [cands[j][0] for j in range(len(cands)) if d[j] == 0]

    def Search(self, prefix):
        return self.SearchWithConverter(prefix, lambda t: t)

    # ---- SimilaritySearcher ----------------------------------------------------
    def SearchSimilar(self, trace, k, band):
        """k nearest stored traces to `trace` by (distance asc, id asc)."""
        ts_all = self.load_all()
        t = trace.symbols if isinstance(trace, SingleTrace) else np.asarray(trace, np.uint64)
        ts = TraceSet([t] + [ts_all.trace(i) for i in range(len(ts_all))])
        pairs = np.array([[0, j + 1] for j in range(len(ts_all))], np.uint32)
        d = ed_pairs(ts, pairs, band)
        order = np.lexsort((np.arange(len(d)), d))[:k]
        return [(int(i), int(d[i])) for i in order]

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


def allpairs_knn(ts, k, band, ctx=None):
    ctx = ctx or _lib.default_context()
    n = len(ts)
    ids = np.zeros((n, k), np.uint32)
    ds = np.zeros((n, k), np.uint32)
    _lib.check(_lib.load().nmz_ed_allpairs_knn(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), n, int(band),
                                               int(k), _lib.ptr(ids), _lib.ptr(ds)))
    return ids, ds


def unique_trace_curve(ts, ctx=None):
    """visualize.go gnuplot mode: after i+1 traces, how many distinct traces
    (SingleTrace.Equals) have been seen. A trace is a repeat iff its nearest
    neighbour is at distance 0 with a smaller id (kNN ties break by id)."""
    n = len(ts)
    if n == 0:
        return []
    ids, ds = allpairs_knn(ts, 1, 0, ctx=ctx) if n > 1 else (np.full((1, 1), _lib.NMZ_NONE),
                                                              np.full((1, 1), _lib.NMZ_NONE))
    seen_before = (ds[:, 0] == 0) & (ids[:, 0] < np.arange(n))
    return list(np.cumsum(~seen_before).astype(int))
