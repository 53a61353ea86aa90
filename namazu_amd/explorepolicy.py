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

Every delay / fault decision -- batch sweeps and the online QueueEvent path --
is computed by libnmz_gpu.so on the GPU. There is no CPU decision path.
"""
import os
import queue
import threading

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


class ExplorePolicy:
    """explorepolicy.ExplorePolicy."""

    NAME = ""

    def __init__(self, device=0):
        self._device = device
        self._action_ch = queue.Queue()  # unbuffered Go channel -> thread-safe queue

    def Name(self):
        return self.NAME

    def LoadConfig(self, cfg):  # -> error or None
        raise NotImplementedError

    def SetHistoryStorage(self, storage):
        return None

    def ActionChan(self):
        return self._action_ch

    def QueueEvent(self, event):
        raise NotImplementedError

    def _ctx(self):
        return _lib.default_context(self._device)

    def _deliver_after(self, delay_ns, action):
        # goroutine + time.After(interval); QueueEvent never blocks
        t = threading.Timer(max(delay_ns, 0) / 1e9, self._action_ch.put, args=(action,))
        t.daemon = True
        t.start()


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

    def determineInterval(self, event):
        """Single decision, computed on the GPU."""
        r = self.Sweep([self.Seed], [event.ReplayHint()], n_dump=1)
        return int(r.delays[0, 0])

    def QueueEvent(self, event):
        interval = self.determineInterval(event)
        self._deliver_after(interval, event.DefaultAction())


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

    def event_inputs(self, events):
        """events -> (evhash uint64[E], evclass uint8[E]) as the kernel consumes them."""
        evhash = np.zeros(len(events), np.uint64)
        evclass = np.zeros(len(events), np.uint8)
        for i, ev in enumerate(events):
            if ev.Class() == "ProcSetEvent":
                raise ValueError("ProcSetEvent decisions belong to procPolicy (out of scope)")
            evhash[i] = ev.evhash()
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
        import ctypes
        _lib.check(_lib.load().nmz_random_sweep(
            ctx.handle, int(seed0), int(n_seeds), _lib.ptr(evhash), _lib.ptr(evclass), e,
            ctypes.byref(p), _lib.ptr(stats), _lib.ptr(delays), _lib.ptr(faults), n_dump, k,
            _lib.ptr(topk)))
        return SweepResult(stats, delays=delays, faults=faults, topk=topk)

    def decide(self, event):
        """(delay_ns, fault) for one event under self.Seed, on the GPU."""
        h, c = self.event_inputs([event])
        r = self.Sweep(self.Seed, 1, h, c, n_dump=1)
        return int(r.delays[0, 0]), bool(r.faults[0, 0])

    def QueueEvent(self, event):
        delay, fault = self.decide(event)
        action = event.DefaultFaultAction() if fault else event.DefaultAction()
        self._deliver_after(delay, action)


RegisterKnownExplorePolicies()
