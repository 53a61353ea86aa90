"""The time-bounded queue behind ActionChan (csrc/tbqueue.hip, the restatement of util/queue/impl.go:64-128;
host code only, so these run without a GPU): release order, and closing while consumers are blocked (the queue
must not be freed under a consumer that is still waking up)."""
import queue
import threading
import time

import numpy as np
import pytest

from namazu_amd import _lib
from namazu_amd.explorepolicy import ActionChannel, ChannelClosed


def test_release_order_and_equal_due_times():
    """Items come out by due time; equal due times keep their enqueue order (impl_test.go:50-63)."""
    ch = ActionChannel()
    try:
        now = ch.L.nmz_monotonic_ns()
        due = [now + d for d in (3_000_000, 1_000_000, 2_000_000, 2_000_000, 2_000_000, 0)]
        for k, t in enumerate(due):
            ch.put_at(t, k)
        got = [ch.get(timeout=5) for _ in due]
        assert got == [5, 1, 2, 3, 4, 0]
        assert ch.stats() == (6, 6, 6)
        assert all(e >= 0 for e in ch.delivery_err_ns)
        with pytest.raises(queue.Empty):
            ch.get(timeout=0.01)
    finally:
        ch.close()


@pytest.mark.parametrize("consumers", [1, 4])
def test_close_wakes_blocked_consumers(consumers):
    """close() while consumers block in get() (no timeout): every consumer returns with ChannelClosed (a
    queue.Empty, distinct from a timeout), close()
    returns after they have left the native queue, and later calls fail cleanly. Repeated, so a consumer still
    inside nmz_tbqueue_dequeue when the queue is freed would show up as a crash or a hang."""
    for _ in range(25):
        ch = ActionChannel()
        out = []
        started = threading.Barrier(consumers + 1)

        def consume():
            started.wait()
            try:
                out.append(ch.get())
            except ChannelClosed:
                out.append("closed")
            except queue.Empty:
                out.append("timeout")

        ts = [threading.Thread(target=consume) for _ in range(consumers)]
        for t in ts:
            t.start()
        started.wait()
        time.sleep(0.002)  # let them block in the native dequeue
        ch.close()
        for t in ts:
            t.join(timeout=10)
            assert not t.is_alive()
        assert out == ["closed"] * consumers
        with pytest.raises(ChannelClosed):
            ch.get(timeout=0)
        with pytest.raises(ValueError):
            ch.put(1)
        ch.close()  # idempotent


def test_native_close_then_destroy():
    """nmz_tbqueue_close: enqueue is refused and dequeue returns NMZ_EAGAIN; destroy then frees the queue."""
    import ctypes
    L = _lib.load()
    q = ctypes.c_void_p()
    _lib.check(L.nmz_tbqueue_create(ctypes.byref(q)))
    _lib.check(L.nmz_tbqueue_enqueue(q, 7, L.nmz_monotonic_ns() + 10**9))
    _lib.check(L.nmz_tbqueue_close(q))
    i, d, r = ctypes.c_uint64(), ctypes.c_int64(), ctypes.c_int64()
    assert L.nmz_tbqueue_dequeue(q, -1, ctypes.byref(i), ctypes.byref(d), ctypes.byref(r)) == _lib.NMZ_EAGAIN
    assert L.nmz_tbqueue_enqueue(q, 8, 0) != 0
    _lib.check(L.nmz_tbqueue_destroy(q))


def test_timeout_is_not_closed():
    """A timed-out get() on an open channel raises plain queue.Empty (not ChannelClosed), so a consumer loop
    `except ChannelClosed: break / except queue.Empty: continue` neither exits early nor spins after close."""
    ch = ActionChannel()
    try:
        with pytest.raises(queue.Empty) as e:
            ch.get(timeout=0.001)
        assert not isinstance(e.value, ChannelClosed)
    finally:
        ch.close()
    with pytest.raises(ChannelClosed):
        ch.get(timeout=0.001)


# ------------------------------------------------------------------ the fixed-duration lane (impl.go:77-89)
def _native_queue():
    import ctypes
    L = _lib.load()
    q = ctypes.c_void_p()
    _lib.check(L.nmz_tbqueue_create(ctypes.byref(q)))
    return L, q


def _drain(L, q, n):
    """n releases as (id, due_ns, released_ns), in release order."""
    import ctypes
    out = []
    i, d, r = ctypes.c_uint64(), ctypes.c_int64(), ctypes.c_int64()
    for _ in range(n):
        _lib.check(L.nmz_tbqueue_dequeue(q, 5 * 10**9, ctypes.byref(i), ctypes.byref(d), ctypes.byref(r)))
        out.append((i.value, d.value, r.value))
    return out


def test_fixed_duration_burst_is_serial():
    """BasicTBQueue's fixed-duration goroutine (util/queue/impl.go:77-89): it takes an item, waits time.After(d) from
    that moment, hands the item over, and only then takes the next. A 50-item burst of fixed 2 ms items enqueued at
    one instant is released at ~2, 4, ..., 100 ms, in enqueue order; each item's timer starts at the previous
    item's release, so consecutive releases are at least d apart and the whole burst takes at least 50 d."""
    L, q = _native_queue()
    try:
        d, n = 2_000_000, 50
        t0 = L.nmz_monotonic_ns()
        for k in range(n):
            _lib.check(L.nmz_tbqueue_enqueue_fixed(q, k, t0, d))
        got = _drain(L, q, n)
        assert [g[0] for g in got] == list(range(n))  # FIFO
        prev = t0
        for k, (_, due, rel) in enumerate(got):
            assert due == prev + d, k  # the timer started at the previous release (or the enqueue, first)
            assert rel >= due
            prev = rel
        rel = np.array([g[2] for g in got], np.int64) - t0
        # release k at ~(k+1) d: at least that, and late only by the timer's own error, summed over the burst
        assert np.all(rel >= d * np.arange(1, n + 1))
        err = np.array([g[2] - g[1] for g in got]) / 1e6
        assert np.percentile(err, 50) < 0.5, err
        assert rel[-1] < n * d + 25_000_000, rel[-1]
    finally:
        _lib.check(L.nmz_tbqueue_destroy(q))


def test_fixed_lane_timer_starts_at_enqueue_when_idle():
    """An item enqueued after the lane went idle starts its timer at its own enqueue (the goroutine was waiting in
    `<-fixedDurationQueue.Out()`), not at the previous release; a zero duration releases at once, in order."""
    L, q = _native_queue()
    try:
        t0 = L.nmz_monotonic_ns()
        _lib.check(L.nmz_tbqueue_enqueue_fixed(q, 1, t0, 1_000_000))
        (_, due1, rel1), = _drain(L, q, 1)
        assert due1 == t0 + 1_000_000
        time.sleep(0.005)
        t1 = L.nmz_monotonic_ns()
        _lib.check(L.nmz_tbqueue_enqueue_fixed(q, 2, t1, 1_000_000))
        for k in range(3, 8):
            _lib.check(L.nmz_tbqueue_enqueue_fixed(q, k, t1, 0))
        got = _drain(L, q, 6)
        assert [g[0] for g in got] == [2, 3, 4, 5, 6, 7]
        assert got[0][1] == t1 + 1_000_000  # max(enqueue, last release) = the enqueue
        for (_, _, prev_rel), (_, due, rel) in zip(got, got[1:]):
            assert due == prev_rel and rel >= due  # zero duration: due at the previous release
        assert L.nmz_tbqueue_enqueue_fixed(q, 9, t1, -1) != 0  # a negative duration is refused
    finally:
        _lib.check(L.nmz_tbqueue_destroy(q))


def test_mixed_burst_interleaves_like_the_two_reference_queues():
    """Ranged items (a goroutine each, released at enqueue + their duration, impl.go:120-126) and fixed items (the
    serial lane) enqueued in one burst interleave by due time: ranged at 1, 5, 11, 30 ms between fixed releases at
    ~2, 4, ..., 20 ms (each ranged due time sits >= 1 ms from any fixed release)."""
    L, q = _native_queue()
    try:
        t0 = L.nmz_monotonic_ns()
        ranged = {100: 1.0, 101: 5.0, 102: 11.0, 103: 30.0}
        for k in range(10):
            _lib.check(L.nmz_tbqueue_enqueue_fixed(q, k, t0, 2_000_000))
            if k in (0, 3, 6, 9):
                rid = 100 + (0, 3, 6, 9).index(k)
                _lib.check(L.nmz_tbqueue_enqueue(q, rid, t0 + int(ranged[rid] * 1e6)))
        got = _drain(L, q, 14)
        order = [g[0] for g in got]
        assert order == [100, 0, 1, 101, 2, 3, 4, 102, 5, 6, 7, 8, 9, 103], order
        for i, due, rel in got:
            if i in ranged:
                assert due == t0 + int(ranged[i] * 1e6)  # ranged items keep their own due time
    finally:
        _lib.check(L.nmz_tbqueue_destroy(q))


def test_random_policy_fixed_interval_is_serial():
    """The random policy's default (maxInterval unset -> = minInterval, randompolicy.go:171-178): every QueueEvent item
    goes through the fixed-duration lane, prioritized ones (x0.8, still min == max) too, so a 50-event burst at 2 ms
    comes out in QueueEvent order at ~2, 4, ..., 100 ms (1.6 ms steps for prioritized events); a ranged policy's
    items do not queue behind each other."""
    from namazu_amd import explorepolicy as ep
    from namazu_amd.config import Config
    from namazu_amd.signal import Event
    p = ep.Random()
    assert p.LoadConfig(Config({"explorePolicy": "random", "explorePolicyParam": {
        "minInterval": "2ms", "faultActionProbability": 0.0, "seed": 5,
        "prioritizedEntities": ["entity-0"]}})) is None
    assert p.MaxInterval == p.MinInterval == 2_000_000
    events = [Event.packet(f"entity-{i % 4}", f"entity-{i % 4}", f"entity-{(i + 1) % 4}", {"n": i}) for i in range(50)]
    assert all(p.is_fixed(e) for e in events)
    try:
        t0 = p.ActionChan().L.nmz_monotonic_ns()
        for ev in events:
            p.QueueEvent(ev)
        rel = []
        got = []
        for _ in events:
            got.append(p.ActionChan().get(timeout=5))
            rel.append(p.ActionChan().last_release_ns - t0)
        assert [a.Event().m["option"]["n"] for a in got] == list(range(50))  # FIFO across both durations
        step = np.array([1_600_000 if e.EntityID() == "entity-0" else 2_000_000 for e in events])
        assert np.all(np.array(rel) >= np.cumsum(step))
        assert rel[-1] < step.sum() + 25_000_000
    finally:
        p.ActionChan().close()
    r = ep.Random()
    assert r.LoadConfig(Config({"explorePolicy": "random", "explorePolicyParam": {
        "minInterval": "1ms", "maxInterval": "3ms", "seed": 5}})) is None
    assert not any(r.is_fixed(e) for e in events)
    try:
        t0 = r.ActionChan().L.nmz_monotonic_ns()
        for ev in events:
            r.QueueEvent(ev)
        for _ in events:
            r.ActionChan().get(timeout=5)
        assert r.ActionChan().last_release_ns - t0 < 40_000_000  # all within ~3 ms, not 50 x 2 ms
    finally:
        r.ActionChan().close()


def test_python_delivery_runs_the_same_two_rules():
    """OnlineDecider without an ActionChannel (a caller-supplied deliver): (delay, action, True) decisions go through
    a serial fixed lane, (delay, action) ones at enqueue + delay."""
    from namazu_amd import explorepolicy as ep
    out = []
    d = ep.OnlineDecider(None, lambda a: out.append((a, time.monotonic_ns())),
                         decide_one=lambda ev: (2_000_000, ev, True) if ev < 100 else (5_500_000, ev))
    d.mode = "host"
    t0 = time.monotonic_ns()
    for ev in list(range(10)) + [100]:
        d.submit(ev)
    assert d.wait_delivered(5)
    assert [a for a, _ in out] == [0, 1, 100, 2, 3, 4, 5, 6, 7, 8, 9]
    fixed = [t - t0 for a, t in out if a < 100]
    assert all(t >= 2_000_000 * (k + 1) for k, t in enumerate(fixed))
