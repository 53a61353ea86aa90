"""Explore-policy plugin API with the MI355X decision engine behind it.

Mirrors nmz/explorepolicy:
  * ExplorePolicy interface          explorepolicy/interface.go:24-40
  * RegisterPolicy / CreatePolicy    explorepolicy/explorepolicy.go:24-38
  * RegisterKnownExplorePolicies     explorepolicy/register.go:24-28
  * Replayable (LoadConfig, determineInterval, QueueEvent)
                                     explorepolicy/replayable/replayablepolicy.go:41-126
  * Random (LoadConfig, QueueEvent, makeActionForEvent)
                                     explorepolicy/random/randompolicy.go:93-346

Error behaviour follows the Go code: LoadConfig *returns* an error value
(None on success) instead of raising; runtime failures raise (Go panics).

Every delay / fault decision is computed by libnmz_gpu.so: batch sweeps on the
GPU; the online QueueEvent path by the library's host decision functions, which
run the kernels' own closed forms (shared code) on the calling thread, because
the reference decides at enqueue and a GPU launch per event would cost more than
the decision. NMZ_ONLINE=gpu decides queued events in GPU launches
instead. Without the library nothing runs (namazu_amd._lib raises).

QueueEvent never blocks on the consumer (randompolicy_test.go:112-118 asserts it):
it decides the event and returns; the time-bounded queue puts each action on
ActionChan by the reference's release rules: a ranged or replayable action at its
enqueue time + its delay (the per-event goroutine + time.After of
replayablepolicy.go:121-125 and util/queue/impl.go:120-126), a fixed-duration one
(min == max) through one FIFO lane whose head's timer starts when the previous
fixed action was released (util/queue/impl.go:77-89,117-119).
"""
import collections
import ctypes
import heapq
import itertools
import os
import queue
import threading
import time

import numpy as np

from . import _lib
from .config import Config
from .signal import Event

# ----------------------------------------------------------------- registry
_policy_factories = {}


def RegisterPolicy(name, factory):
    _policy_factories[name] = factory


def CreatePolicy(name):
    """Returns (policy, error) like the Go API."""
    f = _policy_factories.get(name)
    if f is None:
        return None, ValueError(f"unknown explore policy: {name}")
    return f(), None


def RegisterKnownExplorePolicies():
    RegisterPolicy(Replayable.NAME, Replayable)
    RegisterPolicy(Random.NAME, Random)


def to_csr(items):
    """List of str/bytes -> (uint32 offsets[n+1], uint8 bytes)."""
    bs = [x.encode() if isinstance(x, str) else bytes(x) for x in items]
    off = np.zeros(len(bs) + 1, np.uint32)
    if bs:
        np.cumsum([len(b) for b in bs], out=off[1:])
    data = np.frombuffer(b"".join(bs), np.uint8).copy() if off[-1] else np.zeros(1, np.uint8)
    return off, data


class SweepResult:
    """Per-seed statistics (+ optional per-decision dump and top-k)."""

    def __init__(self, stats, delays=None, faults=None, topk=None):
        self.stats = stats
        self.delays = delays
        self.faults = faults
        self.topk = topk


class ChannelClosed(queue.Empty):
    """ActionChannel.get() on a closed channel (a subclass of queue.Empty, so `except queue.Empty` still catches it;
    a consumer loop that must stop once the channel is closed catches this one first)."""


class ActionChannel:
    """ExplorePolicy.ActionChan() over the library's time-bounded queue (nmz_tbqueue_*, the reference's
    BasicTBQueue, util/queue/impl.go:64-128): put_at(due_ns, action) hands a ranged action to the native timer
    thread, which releases it at its due time (CLOCK_MONOTONIC ns); put_fixed(enqueued_ns, duration_ns, action) puts a
    fixed-duration action on the serial lane (released at max(enqueue, previous fixed release) + duration,
    impl.go:77-89); get() blocks (with the GIL released) until an action is released, like a receive on the Go
    channel. Equal due times keep their enqueue order. Each get() records the action's delivered-delay error
    (release time - due time, both taken natively) and last_release_ns the release time of the last action got."""

    def __init__(self, history=100_000):
        self.L = _lib.load()
        self.q = ctypes.c_void_p()
        _lib.check(self.L.nmz_tbqueue_create(ctypes.byref(self.q)))
        self._items = {}
        self._ids = itertools.count()
        self._lock = threading.Lock()
        self._idle = threading.Condition(self._lock)
        self._calls = 0  # native calls in flight: close() frees the queue only after they have returned
        self._closed = False
        self.delivery_err_ns = collections.deque(maxlen=history)
        self.last_release_ns = None

    def _enter(self):
        with self._lock:
            if self._closed:
                raise ValueError("ActionChannel is closed")
            self._calls += 1
            return self.q

    def _leave(self):
        with self._lock:
            self._calls -= 1
            if self._calls == 0:
                self._idle.notify_all()

    def put_at(self, due_ns, action):
        q = self._enter()
        try:
            with self._lock:
                i = next(self._ids)
                self._items[i] = action
            _lib.check(self.L.nmz_tbqueue_enqueue(q, i, int(due_ns)))
        finally:
            self._leave()

    def put_fixed(self, enqueued_ns, duration_ns, action):
        q = self._enter()
        try:
            with self._lock:
                i = next(self._ids)
                self._items[i] = action
            _lib.check(self.L.nmz_tbqueue_enqueue_fixed(q, i, int(enqueued_ns), int(duration_ns)))
        finally:
            self._leave()

    def put(self, action):
        self.put_at(self.L.nmz_monotonic_ns(), action)

    def get(self, block=True, timeout=None):
        """Blocks until an action is released; queue.Empty on timeout, ChannelClosed (a queue.Empty) once the
        channel is closed (a consumer blocked in get() when close() runs returns with ChannelClosed)."""
        i, due, rel = ctypes.c_uint64(), ctypes.c_int64(), ctypes.c_int64()
        t = -1 if (block and timeout is None) else int((timeout if block else 0) * 1e9)
        try:
            q = self._enter()
        except ValueError:
            raise ChannelClosed("ActionChannel is closed")
        try:
            rc = self.L.nmz_tbqueue_dequeue(q, t, ctypes.byref(i), ctypes.byref(due), ctypes.byref(rel))
        finally:
            self._leave()
        if rc == _lib.NMZ_EAGAIN:
            with self._lock:
                closed = self._closed
            if closed:
                raise ChannelClosed("ActionChannel is closed")
            raise queue.Empty
        _lib.check(rc)
        self.delivery_err_ns.append(rel.value - due.value)
        self.last_release_ns = rel.value
        with self._lock:
            return self._items.pop(i.value)

    def get_nowait(self):
        return self.get(block=False)

    def stats(self):
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        q = self._enter()
        try:
            _lib.check(self.L.nmz_tbqueue_stats(q, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        finally:
            self._leave()
        return a.value, b.value, c.value  # enqueued, released, dequeued

    def close(self):
        """Closes the channel: blocked get() calls return (ChannelClosed), then the native queue is freed once no
        call is inside it (nmz_tbqueue_close, then nmz_tbqueue_destroy)."""
        with self._lock:
            if self._closed or not self.q:
                return
            self._closed = True
            q = self.q
        self.L.nmz_tbqueue_close(q)
        with self._lock:
            while self._calls:
                self._idle.wait()
            self.q = None
        self.L.nmz_tbqueue_destroy(q)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class OnlineDecider:
    """The QueueEvent engine: each event's decision, then its delivery by the reference queue's release rules.

    The reference decides at enqueue, on the caller's goroutine (util/queue/impl.go:35-46,110-128;
    replayablepolicy.go:116-126), and delivers after time.After(delay). Two ways to decide:
      * "host" (the default): submit() decides the event on the calling thread through the library's host
        decision path (nmz_random_decide_host / nmz_replayable_decide_host: the kernels' own closed forms,
        shared code, no launch), so a decision never waits for a GPU launch or for other events;
      * "gpu" (NMZ_ONLINE=gpu): a decision thread decides the queued events in GPU launches of at most
        `max_batch` events (nmz_random_decide / nmz_replayable_decide).
    A decision is (delay, action) or (delay, action, fixed). A ranged action (fixed false) goes to ActionChan at its
    enqueue time + its delay; a fixed-duration one (the random policy's min == max) goes through one FIFO lane,
    released at max(its enqueue, the previous fixed release) + delay (util/queue/impl.go:77-89). The library's
    time-bounded queue releases both from a native timer thread (ActionChannel; without one, a Python delivery
    thread runs the same two rules). latencies_ns holds the enqueue-to-decided time of recent events,
    delivery_err_ns the delivered-delay error (actual delivery - the rule's due time); bench.py reports their
    percentiles. A GPU decision failure is kept and raised by
    the next submit(), where a Go policy would panic (randompolicy.go:343, replayablepolicy.go:120)."""

    def __init__(self, decide_batch, deliver, decide_one=None, history=100_000, max_batch=64, chan=None):
        self._decide_batch = decide_batch
        self._decide_one = decide_one
        self._deliver = deliver
        self._chan = chan  # an ActionChannel: the native queue times the deliveries (no Python delivery thread)
        self.mode = os.environ.get("NMZ_ONLINE", "host") if decide_one is not None else "gpu"
        self.max_batch = max_batch
        self._pending = []
        self._cv = threading.Condition()
        self._heap = []
        self._fixed = collections.deque()  # Python delivery's fixed lane: (enqueue_ns, duration_ns, action)
        self._fixed_last = None
        self._hcv = threading.Condition()
        self._seq = itertools.count()
        self.latencies_ns = collections.deque(maxlen=history)
        self.delivery_err_ns = chan.delivery_err_ns if chan is not None else collections.deque(maxlen=history)
        self.batch_sizes = collections.deque(maxlen=history)
        self.error = None
        self._started = False
        self._n_in = 0
        self._n_decided = 0
        self._n_delivered = 0

    def _start(self):
        loops = [] if self._chan is not None else [self._deliver_loop]
        if self.mode != "host":
            loops.append(self._decide_loop)
        for fn in loops:
            threading.Thread(target=fn, daemon=True).start()
        self._started = True

    def _now(self):
        return _lib.load().nmz_monotonic_ns() if self._chan is not None else time.monotonic_ns()

    def _schedule(self, t0, decision):
        delay, action = max(int(decision[0]), 0), decision[1]
        fixed = len(decision) > 2 and bool(decision[2])
        if self._chan is not None:
            if fixed:
                self._chan.put_fixed(t0, delay, action)
            else:
                self._chan.put_at(t0 + delay, action)
            return
        with self._hcv:
            if fixed:
                self._fixed.append((t0, delay, next(self._seq), action))
            else:
                heapq.heappush(self._heap, (t0 + delay, next(self._seq), action))
            self._hcv.notify()

    def submit(self, event):
        if self.error is not None:
            raise RuntimeError(f"explore policy decision failed: {self.error}") from self.error
        if not self._started:
            with self._cv:
                if not self._started:
                    self._start()
        t0 = self._now()
        if self.mode == "host":
            decision = self._decide_one(event)  # raises like the reference's panic
            self.latencies_ns.append(self._now() - t0)
            self._schedule(t0, decision)
            with self._cv:
                self._n_in += 1
                self._n_decided += 1
            return
        with self._cv:
            self._pending.append((t0, event))
            self._n_in += 1
            self._cv.notify()

    def wait_decided(self, timeout=10.0):
        """Block until every submitted event has been decided (tests and bench only)."""
        end = time.monotonic() + timeout
        with self._cv:
            while self._n_decided < self._n_in and self.error is None:
                if not self._cv.wait(max(end - time.monotonic(), 0)) and time.monotonic() >= end:
                    return False
        return self.error is None

    def wait_delivered(self, timeout=10.0):
        """Block until every submitted event's action has been released to ActionChan (tests and bench only)."""
        end = time.monotonic() + timeout
        while time.monotonic() < end:
            with self._cv:
                n_in = self._n_in
                done = self._n_delivered if self._chan is None else None
            if done is None:
                done = self._chan.stats()[1]
            if done >= n_in:
                return True
            time.sleep(0.001)
        return False

    def _decide_loop(self):
        while True:
            with self._cv:
                while not self._pending:
                    self._cv.wait()
                batch, self._pending = self._pending[:self.max_batch], self._pending[self.max_batch:]
            try:
                out = self._decide_batch([e for _, e in batch])
            except Exception as e:  # noqa: BLE001 -- surfaced by the next submit()
                self.error = e
                with self._cv:
                    self._cv.notify_all()
                return
            now = self._now()
            self.batch_sizes.append(len(batch))
            for (t0, _), decision in zip(batch, out):
                self.latencies_ns.append(now - t0)
                self._schedule(t0, decision)
            with self._cv:
                self._n_decided += len(batch)
                self._cv.notify_all()

    def _next_due(self):
        """(due, seq, lane) of the next action to deliver, or None: the heap's top or the fixed lane's head, whose
        timer starts at max(its enqueue, the previous fixed delivery) (util/queue/impl.go:77-89)."""
        cands = []
        if self._heap:
            cands.append((self._heap[0][0], self._heap[0][1], 0))
        if self._fixed:
            t0, d, seq, _ = self._fixed[0]
            start = t0 if self._fixed_last is None else max(t0, self._fixed_last)
            cands.append((start + d, seq, 1))
        return min(cands) if cands else None

    def _deliver_loop(self):
        """Python delivery for a caller-supplied deliver() (no ActionChannel): the same two release rules as the
        native queue, one action at a time in due order."""
        while True:
            with self._hcv:
                while True:
                    nxt = self._next_due()
                    if nxt is not None:
                        wait_ns = nxt[0] - time.monotonic_ns()
                        if wait_ns <= 0:
                            break
                        self._hcv.wait(wait_ns / 1e9)
                    else:
                        self._hcv.wait()
                due, _, lane = nxt
                action = heapq.heappop(self._heap)[2] if lane == 0 else self._fixed.popleft()[3]
            self._deliver(action)
            now = time.monotonic_ns()
            self.delivery_err_ns.append(now - due)
            with self._hcv:
                if lane == 1:
                    self._fixed_last = now
            with self._cv:
                self._n_delivered += 1


class ExplorePolicy:
    """explorepolicy.ExplorePolicy."""

    NAME = ""

    def __init__(self, device=0):
        self._device = device
        self._action_ch = ActionChannel()  # the Go channel the reference's TBQueue feeds
        self.online = OnlineDecider(self._decide_batch, self._action_ch.put, decide_one=self._decide_one,
                                    chan=self._action_ch)

    def Name(self):
        return self.NAME

    def LoadConfig(self, cfg):  # -> error or None
        raise NotImplementedError

    def SetHistoryStorage(self, storage):
        return None

    def ActionChan(self):
        return self._action_ch

    def QueueEvent(self, event):
        """Non-blocking (never waits for the action's consumer): the event is decided at enqueue, as the reference
        does, and its action is released by the time-bounded queue (at enqueue + delay, or through the serial
        fixed-duration lane for the random policy's min == max items)."""
        self.online.submit(event)

    def _decide_batch(self, events):
        raise NotImplementedError

    def _decide_one(self, event):
        raise NotImplementedError

    def _ctx(self):
        return _lib.default_context(self._device)


# ----------------------------------------------------------------- replayable
class Replayable(ExplorePolicy):
    """replayable: delay = FNV1a64(seed || hint) % maxInterval (replayablepolicy.go:100-114)."""

    NAME = "replayable"

    def __init__(self, device=0):
        super().__init__(device)
        self.MaxInterval = 0  # ns
        self.Seed = ""

    def LoadConfig(self, cfg: Config):
        """replayablepolicy.go:63-90."""
        try:
            key = "explorepolicyparam.maxInterval"
            if cfg.is_set(key):
                self.MaxInterval = cfg.get_duration(key)
            else:
                self.MaxInterval = 10 * 1000_000  # 10 ms default (:70)
            key = "explorepolicyparam.seed"
            self.Seed = cfg.get_string(key) if cfg.is_set(key) else ""
            env = os.environ.get("NMZ_REPLAY_SEED", "")
            if env != "":
                self.Seed = env
        except ValueError as e:
            return e
        return None

    def Sweep(self, seeds, hints, n_dump=0, k=0, ctx=None):
        """Evaluate every (seed, hint) decision on the GPU.

        seeds: list of seed strings; hints: list of ReplayHint() strings (one per
        event, in trace order). Returns SweepResult with stats[len(seeds)],
        delays[n_dump, len(hints)] (int64 ns) and topk[k] (seed = index).
        """
        ctx = ctx or self._ctx()
        soff, sb = to_csr(seeds)
        hoff, hb = to_csr(hints)
        n, e = len(seeds), len(hints)
        stats = np.zeros(n, _lib.SCHED_STATS_DTYPE)
        delays = np.zeros((n_dump, e), np.int64) if n_dump else None
        topk = np.zeros(k, _lib.TOPK_DTYPE) if k else None
        _lib.check(_lib.load().nmz_replayable_sweep(
            ctx.handle, _lib.ptr(soff), _lib.ptr(sb), n, _lib.ptr(hoff), _lib.ptr(hb), e,
            int(self.MaxInterval), _lib.ptr(stats), _lib.ptr(delays), n_dump, k, _lib.ptr(topk)))
        return SweepResult(stats, delays=delays, topk=topk)

    def decide_intervals(self, events, ctx=None):
        """determineInterval for a batch of events under self.Seed (nmz_replayable_decide)."""
        ctx = ctx or self._ctx()
        hoff, hb = to_csr([e.ReplayHint() for e in events])
        seed = self.Seed.encode() if isinstance(self.Seed, str) else bytes(self.Seed)
        sb = np.frombuffer(seed, np.uint8).copy() if seed else np.zeros(1, np.uint8)
        out = np.zeros(max(len(events), 1), np.int64)
        _lib.check(_lib.load().nmz_replayable_decide(ctx.handle, _lib.ptr(sb), len(seed), _lib.ptr(hoff),
                                                     _lib.ptr(hb), len(events), int(self.MaxInterval),
                                                     _lib.ptr(out)))
        return out[:len(events)]

    def determineInterval(self, event):
        """replayablepolicy.go:100-114, one decision on the GPU."""
        return int(self.decide_intervals([event])[0])

    def _decide_batch(self, events):
        return list(zip(self.decide_intervals(events).tolist(), [e.DefaultAction() for e in events]))

    def _decide_one(self, event):
        """determineInterval on this thread (nmz_replayable_decide_host): FNV-1a 64 over seed || hint % maxInterval."""
        hint = event.ReplayHint().encode()
        seed = self.Seed.encode() if isinstance(self.Seed, str) else bytes(self.Seed)
        off = (ctypes.c_uint32 * 2)(0, len(hint))
        out = ctypes.c_int64()
        _lib.check(_lib.load().nmz_replayable_decide_host(seed or None, len(seed), off, hint or None, 1,
                                                          int(self.MaxInterval), ctypes.byref(out)))
        return out.value, event.DefaultAction()


# ----------------------------------------------------------------- random
class Random(ExplorePolicy):
    """random: Int63n delay in [min, max) and Intn(999) fault draw per event.

    Determinism contract (the reference re-seeds the global math/rand from the
    wall clock per event, util/queue/impl.go:39, so it is not reproducible):
    each decision uses a fresh rand.New(rand.NewSource(FNV1a64(le64(seed) ||
    le64(evhash)))) and draws delay first, then fault. The optional "seed"
    parameter fixes the seed; without it one is drawn from os.urandom.
    """

    NAME = "random"

    def __init__(self, device=0):
        super().__init__(device)
        self.MinInterval = 0
        self.MaxInterval = 0
        self.PrioritizedEntities = {}
        self.ShellActionInterval = 0
        self.ShellActionCommand = ""
        self.FaultActionProbability = 0.0
        self.ProcPolicy = "mild"
        self.Seed = int.from_bytes(os.urandom(8), "little")

    def LoadConfig(self, cfg: Config):
        """randompolicy.go:156-228 (ProcSet sub-policies are out of scope)."""
        try:
            epp = "explorepolicyparam."
            if cfg.is_set(epp + "minInterval"):
                self.MinInterval = cfg.get_duration(epp + "minInterval")
            if cfg.is_set(epp + "maxInterval"):
                self.MaxInterval = cfg.get_duration(epp + "maxInterval")
            else:
                self.MaxInterval = self.MinInterval
            if cfg.is_set(epp + "prioritizedEntities"):
                for s in cfg.get_string_slice(epp + "prioritizedEntities") or []:
                    self.PrioritizedEntities[s] = True
            if cfg.is_set(epp + "shellActionInterval"):
                self.ShellActionInterval = cfg.get_duration(epp + "shellActionInterval")
            if cfg.is_set(epp + "shellActionCommand"):
                self.ShellActionCommand = cfg.get_string(epp + "shellActionCommand")
            if self.ShellActionInterval < 0:
                return ValueError(f"shellActionInterval(={self.ShellActionInterval}) must be non-negative value")
            if cfg.is_set(epp + "faultActionProbability"):
                self.FaultActionProbability = cfg.get_float64(epp + "faultActionProbability")
            if self.FaultActionProbability < 0.0 or self.FaultActionProbability > 1.0:
                return ValueError(f"bad faultActionProbability {self.FaultActionProbability:f}")
            if cfg.is_set(epp + "seed"):
                self.Seed = cfg.get_int(epp + "seed") & ((1 << 64) - 1)
            pp = cfg.get_string(epp + "procPolicy")
            if pp:
                self.ProcPolicy = pp
            if self.ProcPolicy not in ("mild", "extreme", "dirichlet"):
                return ValueError(f"bad procPolicy {self.ProcPolicy}")
            if self.ProcPolicy == "dirichlet":
                rp = cfg.get_float64(epp + "procPolicyParam.resetProbability") \
                    if cfg.is_set(epp + "procPolicyParam.resetProbability") else 0.1
                if rp < 0.0 or rp > 1.0:
                    return ValueError(f"bad procPolicyParam.resetProbability {rp:f}")
        except ValueError as e:
            return e
        return None

    def params(self):
        """Resolved integer parameters (x0.8 prioritized intervals, fault threshold)."""
        return _lib.resolve_random_params(self.MinInterval, self.MaxInterval,
                                          self.FaultActionProbability)

    def event_inputs(self, events, ctx=None):
        """events -> (evhash uint64[E], evclass uint8[E]) as the kernel consumes them. The event hashes of a
        batch are computed on the GPU (nmz_fnv1a64_batch over the events' canonical JSON)."""
        evhash = np.zeros(len(events), np.uint64)
        evclass = np.zeros(len(events), np.uint8)
        if events:
            off, data = to_csr([ev.canonical_json() for ev in events])
            off64 = off.astype(np.uint64)
            _lib.check(_lib.load().nmz_fnv1a64_batch((ctx or self._ctx()).handle, _lib.ptr(off64), _lib.ptr(data),
                                                     len(events), _lib.ptr(evhash)))
        for i, ev in enumerate(events):
            if ev.Class() == "ProcSetEvent":
                raise ValueError("ProcSetEvent decisions belong to procPolicy (out of scope)")
            c = 0
            if ev.EntityID() in self.PrioritizedEntities:
                c |= _lib.NMZ_EV_PRIORITIZED
            if ev.faultable():
                c |= _lib.NMZ_EV_FAULTABLE
            evclass[i] = c
        return evhash, evclass

    def Sweep(self, seed0, n_seeds, evhash, evclass, n_dump=0, k=0, ctx=None):
        """All decisions for seeds seed0..seed0+n_seeds-1 over one trace, on the GPU."""
        ctx = ctx or self._ctx()
        evhash = np.ascontiguousarray(evhash, np.uint64)
        evclass = np.ascontiguousarray(evclass, np.uint8)
        p = self.params()
        e = len(evhash)
        stats = np.zeros(n_seeds, _lib.SCHED_STATS_DTYPE)
        delays = np.zeros((n_dump, e), np.int64) if n_dump else None
        faults = np.zeros((n_dump, e), np.uint8) if n_dump else None
        topk = np.zeros(k, _lib.TOPK_DTYPE) if k else None
        _lib.check(_lib.load().nmz_random_sweep(
            ctx.handle, int(seed0), int(n_seeds), _lib.ptr(evhash), _lib.ptr(evclass), e,
            ctypes.byref(p), _lib.ptr(stats), _lib.ptr(delays), _lib.ptr(faults), n_dump, k,
            _lib.ptr(topk)))
        return SweepResult(stats, delays=delays, faults=faults, topk=topk)

    def decide_events(self, events, ctx=None):
        """(delays int64[n], faults bool[n]) of a batch of events under self.Seed (nmz_random_decide)."""
        ctx = ctx or self._ctx()
        h, c = self.event_inputs(events)
        n = len(events)
        delays = np.zeros(max(n, 1), np.int64)
        faults = np.zeros(max(n, 1), np.uint8)
        p = self.params()
        _lib.check(_lib.load().nmz_random_decide(ctx.handle, int(self.Seed), _lib.ptr(h), _lib.ptr(c), n,
                                                 ctypes.byref(p), _lib.ptr(delays), _lib.ptr(faults)))
        return delays[:n], faults[:n].astype(bool)

    def decide(self, event):
        """(delay_ns, fault) for one event under self.Seed, on the GPU."""
        d, f = self.decide_events([event])
        return int(d[0]), bool(f[0])

    def is_fixed(self, event):
        """QueueEvent's queue kind (randompolicy.go:332-346 + util/queue/impl.go:117-119): the event's interval
        bounds after the prioritized x0.8 are equal, so its item goes through BasicTBQueue's fixed-duration lane."""
        p = self._cached_params()
        pr = 1 if event.EntityID() in self.PrioritizedEntities else 0
        return p.min_ns[pr] == p.max_ns[pr]

    def _cached_params(self):
        key = (self.MinInterval, self.MaxInterval, self.FaultActionProbability)
        if getattr(self, "_params_key", None) != key:
            self._params, self._params_key = self.params(), key
        return self._params

    def _decide_batch(self, events):
        d, f = self.decide_events(events)
        return [(int(dl), e.DefaultFaultAction() if fl else e.DefaultAction(), self.is_fixed(e))
                for dl, fl, e in zip(d.tolist(), f.tolist(), events)]

    def event_class(self, ev):
        if ev.Class() == "ProcSetEvent":
            raise ValueError("ProcSetEvent decisions belong to procPolicy (out of scope)")
        c = _lib.NMZ_EV_PRIORITIZED if ev.EntityID() in self.PrioritizedEntities else 0
        return c | (_lib.NMZ_EV_FAULTABLE if ev.faultable() else 0)

    def _decide_one(self, event):
        """makeActionForEvent + the queue's delay draw on this thread (nmz_random_decide_host): the event's hash
        (FNV-1a 64 of its canonical JSON, nmz_fnv1a64_batch_host), its class, and the kernels' closed forms."""
        L = _lib.load()
        js = event.canonical_json()
        js = js.encode() if isinstance(js, str) else bytes(js)
        off = (ctypes.c_uint64 * 2)(0, len(js))
        h = ctypes.c_uint64()
        _lib.check(L.nmz_fnv1a64_batch_host(off, js or None, 1, ctypes.byref(h)))
        cls = ctypes.c_uint8(self.event_class(event))
        p = self._cached_params()
        d, f = ctypes.c_int64(), ctypes.c_uint8()
        _lib.check(L.nmz_random_decide_host(int(self.Seed), ctypes.byref(h), ctypes.byref(cls), 1,
                                            ctypes.byref(p), ctypes.byref(d), ctypes.byref(f)))
        pr = 1 if cls.value & _lib.NMZ_EV_PRIORITIZED else 0
        return (d.value, (event.DefaultFaultAction() if f.value else event.DefaultAction()),
                p.min_ns[pr] == p.max_ns[pr])


RegisterKnownExplorePolicies()
