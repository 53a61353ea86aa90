"""`nmz tools visualize` unique-trace counts (exact and partial-order reduced, cli/tools/visualize.go:42,51-172)
and the action-level Search rule (naive.go:235-257 + AreActionsSliceEqual, util/signal/misc.go:22-35).

CPU: the oracle's literal restatements (oracle.unique_curve_exact / unique_curve_po) on hand-built cases, the
symbol rules against plain map equality (BasicSignal.EqualsSignal: reflect.DeepEqual without uuid,
signal.go:174-186) on the reference's 4 stored ZooKeeper traces (tests/golden/zk_store.json).
GPU: nmz_unique_traces / Search through the naive-storage reader vs those rules."""
import copy
import json
import os
import uuid

import numpy as np
import pytest

from namazu_amd import historystorage as hs
from namazu_amd.signal import Event
from oracle import oracle as O


def _without_uuid(m):
    return {k: v for k, v in m.items() if k != "uuid"}


def equals_signal(a, b):
    """EqualsSignal (signal.go:174-186): maps equal once uuid is ignored (arrival time is not in the map)."""
    return _without_uuid(a) == _without_uuid(b)


def zk_store_traces(golden):
    """The 4 stored traces plus two derived runs: 4 = trace 0 re-recorded (new action uuids, same event uuids:
    Action-equal to 0), 5 = trace 0 replayed (new event uuids: Event-equal to 0, not Action-equal)."""
    tr = golden("zk_store.json")["traces"]
    out = [(t["actions"], t["events"]) for t in tr]
    a0, e0 = copy.deepcopy(out[0])
    for a in a0:
        a["uuid"] = str(uuid.UUID(int=hash(a["uuid"]) & ((1 << 128) - 1)))
    out.append((a0, e0))
    a1, e1 = copy.deepcopy(out[0])
    for a, e in zip(a1, e1):
        new = str(uuid.UUID(int=(hash(e["uuid"]) * 31) & ((1 << 128) - 1)))
        e["uuid"] = new
        if "event_uuid" in a:
            a["event_uuid"] = new
        if isinstance(a.get("option"), dict) and "event_uuid" in a["option"]:
            a["option"]["event_uuid"] = new
    out.append((a1, e1))
    return out


def write_store(root, traces):
    os.makedirs(root, exist_ok=True)
    with open(os.path.join(root, "config.toml"), "w") as f:
        f.write('storageType = "naive"\n')
    for i, (acts, evs) in enumerate(traces):
        adir = os.path.join(root, "%08x" % i, "actions")
        os.makedirs(adir)
        for n, (a, e) in enumerate(zip(acts, evs)):
            with open(os.path.join(adir, f"{n}.action.json"), "w") as f:
                json.dump(a, f)
            if e is not None:
                with open(os.path.join(adir, f"{n}.event.json"), "w") as f:
                    json.dump(e, f)


def rule_search(traces, prefix_actions):
    """naive.go:235-252 with the identity converter, on maps."""
    out = []
    for i in range(len(traces) - 1):
        acts = traces[i][0]
        if len(acts) < len(prefix_actions):
            continue
        if len(acts) == len(prefix_actions) and all(equals_signal(a, b) for a, b in zip(prefix_actions, acts)):
            out.append(i)
    return out


def rule_curves(traces):
    """Both visualize modes on maps: exact (action map equality) and PO (per-entity event map equality)."""
    exact_keys = [[json.dumps(_without_uuid(a), sort_keys=True) for a in acts] for acts, _ in traces]
    po = [[(e["entity"], json.dumps(_without_uuid(e), sort_keys=True)) if e is not None else (None, None)
           for e in evs] for _, evs in traces]
    return O.unique_curve_exact(
        [[hash(k) & ((1 << 64) - 1) for k in t] for t in exact_keys]), O.unique_curve_po(
        [[(ent, hash(k) & ((1 << 64) - 1) if k else 0) for ent, k in t] for t in po])


# ------------------------------------------------------------------ CPU
def test_oracle_po_and_exact_modes():
    # entity a: x1 x2, entity b: y1 -- interleavings differ, projections agree
    t0 = [("a", 1), ("b", 9), ("a", 2)]
    t1 = [("b", 9), ("a", 1), ("a", 2)]
    t2 = [("a", 2), ("b", 9), ("a", 1)]      # a's order differs
    t3 = [("a", 1), ("a", 2)]                # b missing
    t4 = [("a", 1), (None, 77), ("b", 9), ("a", 2)]  # an action without an event is skipped
    assert O.unique_curve_po([t0, t1, t2, t3, t4]) == [1, 1, 2, 3, 3]
    assert O.unique_curve_exact([[e for _, e in t] for t in [t0, t1, t2, t3, t0]]) == [1, 2, 3, 4, 4]
    assert O.unique_curve_po([]) == [] and O.unique_curve_po([[], []]) == [1, 1]


def test_action_symbols_follow_equals_signal():
    a = {"class": "EventAcceptanceAction", "entity": "e", "type": "action", "option": {}, "uuid": "u1",
         "event_uuid": "ev1"}
    b = dict(a, uuid="u2")
    c = dict(a, event_uuid="ev2")
    old = {"class": "AcceptEventAction", "entity": "e", "type": "action", "uuid": "u3",
           "option": {"event_uuid": "ev1"}}
    old2 = dict(old, uuid="u4", option={"event_uuid": "ev9"})
    assert hs.action_symbol(a) == hs.action_symbol(b)          # uuid ignored
    assert hs.action_symbol(a) != hs.action_symbol(c)          # top-level event_uuid counts
    assert hs.action_symbol(old) != hs.action_symbol(old2)     # so does the 2015 option.event_uuid
    ev = Event.packet("e", "a", "b")
    acc = ev.DefaultAction()
    assert acc.JSONMap()["event_uuid"] == ev.ID() and "event_uuid" not in acc.JSONMap()["option"]
    nop = Event({"class": "LogEvent", "entity": "e", "uuid": "x"}).DefaultAction()
    assert nop.Class() == "NopAction" and "event_uuid" not in nop.JSONMap()


def test_zk_store_symbols_reproduce_map_equality(golden, tmp_path):
    """Host side only: the reader's action / event symbols induce the same equality relations as the
    reference's map comparisons on the ZooKeeper store (+ derived runs)."""
    traces = zk_store_traces(golden)
    write_store(str(tmp_path), traces)
    st = hs.LoadStorage(str(tmp_path))
    got = st.traces()
    assert [len(t) for t in got] == [48, 41, 26, 36, 48, 48]
    flat_a = [(a, s) for (acts, _), t in zip(traces, got) for a, s in zip(acts, t.action_symbols)]
    flat_e = [(e, s) for (_, evs), t in zip(traces, got) for e, s in zip(evs, t.symbols) if e is not None]
    rng = np.random.default_rng(1)
    for items in (flat_a, flat_e):
        for _ in range(3000):
            (x, sx), (y, sy) = items[rng.integers(len(items))], items[rng.integers(len(items))]
            assert (sx == sy) == equals_signal(x, y)
    assert got[0].Equals(got[4]) and not got[0].Equals(got[5])
    assert np.array_equal(got[0].symbols, got[5].symbols)
    assert set(e for t in got for e in t.entities) == {"_earthquake_ether_inspector"}


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_zk_store_search_and_unique_curves(golden, tmp_path):
    traces = zk_store_traces(golden)
    write_store(str(tmp_path), traces)
    st = hs.LoadStorage(str(tmp_path))
    exact, po = rule_curves(traces)
    assert exact == [1, 2, 3, 4, 4, 5] and po == [1, 2, 3, 4, 4, 4]
    assert st.UniqueTraceCurve(po_reduction=False) == exact
    assert st.UniqueTraceCurve() == po  # the default, -po-reduction=true
    for q in range(6):
        prefix = traces[q][0]
        assert st.Search(prefix) == rule_search(traces, prefix)
        t, _ = st.GetStoredHistory(q)
        assert st.Search(t) == rule_search(traces, prefix)
    assert st.Search(traces[0][0]) == [0, 4]
    # a converter that keeps the first 10 actions: ids whose 10-action prefix equals trace 1's
    t1, _ = st.GetStoredHistory(1)
    pre = hs.SingleTrace(t1.symbols[:10], action_symbols=t1.action_symbols[:10])
    got = st.SearchWithConverter(pre, lambda t: hs.SingleTrace(t.symbols[:10], action_symbols=t.action_symbols[:10]))
    exp = [i for i in range(5) if len(traces[i][0]) >= 10 and
           all(equals_signal(a, b) for a, b in zip(traces[i][0][:10], traces[1][0][:10]))]
    assert got == exp and 1 in got


def _random_po_traces(rng, n, n_ent, lmin, lmax, n_events, p_none=0.0, dup=0.3, shuffle=0.5):
    """Traces over events e (entity e % n_ent); repeats of earlier traces, some with their cross-entity
    interleaving shuffled (PO-equal, not exact-equal), some with one entity's order changed."""
    out = []
    for i in range(n):
        if out and rng.random() < dup:
            t = list(out[int(rng.integers(len(out)))])
            r = rng.random()
            if r < shuffle:  # re-interleave entities, keeping each entity's order
                by = {}
                for x in t:
                    by.setdefault(x[0], []).append(x)
                keys = [k for k, v in by.items() for _ in v]
                rng.shuffle(keys)
                it = {k: iter(v) for k, v in by.items()}
                t = [next(it[k]) for k in keys]
            elif r < shuffle + 0.2 and len(t) > 1:  # swap two events: usually breaks PO equality
                a, b = rng.integers(len(t), size=2)
                t[a], t[b] = t[b], t[a]
        else:
            L = int(rng.integers(lmin, lmax + 1))
            evs = rng.integers(0, n_events, L)
            t = [((None, int(rng.integers(1, 2**63))) if rng.random() < p_none else
                  (f"ent-{e % n_ent}", int(e) * 0x9E3779B97F4A7C15 % (1 << 64) + 1)) for e in evs]
        out.append(t)
    return out


def _to_single(t):
    return hs.SingleTrace([s for _, s in t], entities=[e for e, _ in t],
                          action_symbols=[s for _, s in t])


@pytest.mark.gpu
@pytest.mark.parametrize("n,n_ent,lmin,lmax,n_events,p_none", [
    (200, 4, 0, 30, 40, 0.0),          # short traces, empty ones
    (150, 16, 50, 300, 400, 0.05),     # several 64-element steps, actions without events
    (120, 200, 100, 400, 5000, 0.0),   # > 64 distinct entities per step (entity masks in LDS)
    (60, 2000, 1, 3000, 8000, 0.0),    # > 1,024 entities: the per-bit ballots, four waves per workgroup
    (40, 5000, 1, 6000, 20000, 0.0),   # > 4096 entities: one wave per workgroup
    (6, 1, 66000, 70000, 50, 0.0),     # ranks past the 65,536-entry key table (inline keys)
])
def test_unique_curves_vs_oracle(ctx, n, n_ent, lmin, lmax, n_events, p_none):
    rng = np.random.default_rng(n + n_ent)
    raw = _random_po_traces(rng, n, n_ent, lmin, lmax, n_events, p_none)
    traces = [_to_single(t) for t in raw]
    po = hs.unique_trace_curve(traces, po_reduction=True, ctx=ctx)
    exact = hs.unique_trace_curve(traces, po_reduction=False, ctx=ctx)
    assert po == O.unique_curve_po(raw)
    assert exact == O.unique_curve_exact([[s for _, s in t] for t in raw])
    if n_ent > 1:
        assert po[-1] < exact[-1]  # the shuffled repeats are PO-equal only


@pytest.mark.gpu
def test_unique_first_equal_and_signatures(ctx):
    """first_equal is the smallest equal index; signatures equal exactly on equal traces; empty input."""
    import ctypes
    from namazu_amd import _lib
    rng = np.random.default_rng(9)
    raw = _random_po_traces(rng, 300, 6, 0, 200, 100, 0.02, dup=0.5)
    traces = [_to_single(t) for t in raw]
    fe = hs.first_equal(traces, po_reduction=True, ctx=ctx)
    canon = [tuple(sorted(((e, r), s) for (e, s), r in zip(
        [x for x in t if x[0] is not None],
        [sum(1 for y in [x for x in t if x[0] is not None][:k] if y[0] == x[0])
         for k, x in enumerate([x for x in t if x[0] is not None])]))) for t in raw]
    for i in range(len(raw)):
        j = next(j for j in range(i + 1) if canon[j] == canon[i])
        assert fe[i] == j
    ts, ent = hs.po_inputs(traces)
    sig = np.zeros(2 * len(ts), np.uint64)
    _lib.check(_lib.load().nmz_trace_signatures(ctx.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), _lib.ptr(ent),
                                                len(ts), _lib.ptr(sig)))
    sig = sig.reshape(-1, 2)
    for i in range(len(raw)):
        assert (sig[i] == sig[fe[i]]).all()
    assert len({tuple(s) for s in sig}) == len(set(canon))
    assert hs.unique_trace_curve([], ctx=ctx) == []
    assert _lib.load().nmz_unique_traces(ctx.handle, None, None, None, 0, None) == 0
    assert _lib.load().nmz_unique_traces(None, None, None, None, 1, None) == _lib.NMZ_EINVAL
    del ctypes


@pytest.mark.gpu
def test_unique_traces_dev_entity_bound_and_errors(ctx):
    """nmz_unique_traces_dev with the caller's entity bound: the same classes as the host entry point; more than
    16,384 entities is an error, not an LDS overrun."""
    import ctypes
    import torch
    from namazu_amd import _lib
    rng = np.random.default_rng(3)
    raw = _random_po_traces(rng, 120, 7, 0, 150, 60, 0.05, dup=0.5)
    traces = [_to_single(t) for t in raw]
    ts, ent = hs.po_inputs(traces)
    fe = hs.first_equal(traces, po_reduction=True, ctx=ctx)
    d_off = torch.from_numpy(ts.off.view(np.int64)).cuda()
    d_sym = torch.from_numpy(ts.sym.view(np.int64)).cuda()
    d_ent = torch.from_numpy(ent.view(np.int32)).cuda()
    d_sig = torch.empty(2 * len(ts), dtype=torch.int64, device="cuda")
    d_fe = torch.empty(len(ts), dtype=torch.int32, device="cuda")
    L = _lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    _lib.check(L.nmz_unique_traces_dev(ctx.handle, P(d_off), P(d_sym), P(d_ent), len(ts), 7, P(d_sig), P(d_fe), st))
    torch.cuda.synchronize()
    assert d_fe.cpu().numpy().view(np.uint32).tolist() == fe.tolist()
    assert L.nmz_unique_traces_dev(ctx.handle, P(d_off), P(d_sym), P(d_ent), len(ts), 20000, P(d_sig), P(d_fe),
                                   st) == _lib.NMZ_EINVAL
    big = np.arange(20000, dtype=np.uint32)
    off = np.array([0, 20000], np.uint64)
    sym = np.arange(20000, dtype=np.uint64)
    out = np.zeros(1, np.uint32)
    assert L.nmz_unique_traces(ctx.handle, _lib.ptr(off), _lib.ptr(sym), _lib.ptr(big), 1, _lib.ptr(out)) == \
        _lib.NMZ_EINVAL
