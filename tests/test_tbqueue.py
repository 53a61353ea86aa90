"""The time-bounded queue behind ActionChan (csrc/tbqueue.hip, the restatement of util/queue/impl.go:64-128;
host code only, so these run without a GPU): release order, and closing while consumers are blocked (the queue
must not be freed under a consumer that is still waking up)."""
import queue
import threading
import time

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
