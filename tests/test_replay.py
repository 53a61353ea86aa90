"""Feedback loop top-k seeds -> replay (namazu_amd/replay.py).

CPU: the helpers and the reference's config/env route (replayablepolicy.go:74-87).
GPU: a sweep's best schedule, replayed through Replayable.LoadConfig +
determineInterval event by event, reproduces the sweep's statistics; BASELINE configs[0] (the random
policy over one 10k-event trace, single seed) through LoadConfig / decide / QueueEvent vs the oracle."""
import numpy as np
import pytest

from namazu_amd import _lib
from namazu_amd import explorepolicy as ep
from namazu_amd import replay
from namazu_amd.config import Config
from namazu_amd.signal import Event


def _topk(seeds):
    t = np.zeros(len(seeds), _lib.TOPK_DTYPE)
    t["seed"] = seeds
    return t


def test_replayable_seeds_map_indices_and_stop_at_sentinel():
    seeds = ["s0", "s1", b"s2"]
    assert replay.replayable_seeds(_topk([2, 0, 2**64 - 1]), seeds) == ["s2", "s0"]


def test_random_seeds_wrap_and_sentinel():
    seed0 = 2**64 - 2
    tk = _topk([2**64 - 1, 1, 2**64 - 1])
    tk["seed"][2] = 2**64 - 1
    assert replay.random_seeds(tk, seed0, 4) == [2**64 - 1, 1, 2**64 - 1]
    assert replay.random_seeds(_topk([5]), 0, 4) == []


def test_replay_env_overrides_config_seed(monkeypatch):
    monkeypatch.delenv(replay.REPLAY_SEED_ENV, raising=False)
    cfg = Config({"explorePolicy": "replayable", "explorePolicyParam": {"seed": "old", "maxInterval": "1s"}})
    for k, v in replay.replay_env("12345").items():
        monkeypatch.setenv(k, v)
    p = ep.Replayable()
    assert p.LoadConfig(cfg) is None and p.Seed == "12345"


def test_replay_config_roundtrip_through_toml(monkeypatch):
    monkeypatch.delenv(replay.REPLAY_SEED_ENV, raising=False)
    base = Config({"explorePolicy": "replayable", "run": "run.sh",
                   "explorePolicyParam": {"maxInterval": "100ms", "seed": ""}})
    text = replay.to_toml(replay.replay_config(base, "834593"))
    p = ep.Replayable()
    assert p.LoadConfig(Config.from_toml(text)) is None
    assert (p.Seed, p.MaxInterval) == ("834593", 100_000_000)
    rnd = Config({"explorePolicy": "random", "explorePolicyParam": {"minInterval": "30ms", "maxInterval": "100ms"}})
    q = ep.Random()
    assert q.LoadConfig(Config.from_toml(replay.to_toml(replay.replay_config(rnd, 2**63 + 5)))) is None
    assert q.Seed == 2**63 + 5
    with pytest.raises(ValueError):
        replay.replay_config(Config({"explorePolicy": "dumb"}), 1)


@pytest.mark.gpu
def test_best_replayable_schedule_replays_event_by_event(monkeypatch):
    ctx = _lib.Context(0)
    p = ep.Replayable()
    p.MaxInterval = 100_000_000
    seeds = [str(i) for i in range(3000)]
    hints = [f"hint-entity-{i % 5}-{i}" for i in range(96)]
    r = p.Sweep(seeds, hints, k=4, ctx=ctx)
    best = replay.replayable_seeds(r.topk, seeds)
    assert len(best) == 4
    for k, v in replay.replay_env(best[0]).items():
        monkeypatch.setenv(k, v)
    q = ep.Replayable()
    cfg = Config({"explorePolicy": "replayable", "explorePolicyParam": {"maxInterval": "100ms"}})
    assert q.LoadConfig(cfg) is None and q.Seed == best[0]
    # the online path: one determineInterval (replayablepolicy.go:100-114) per event
    delays = [q.determineInterval(Event.packet(f"entity-{i % 5}", "a", "b", replay_hint=h))
              for i, h in enumerate(hints)]
    st = r.stats[int(r.topk["seed"][0])]
    assert sum(delays) == int(st["sum_delay_ns"])
    assert max(delays) == int(st["max_delay_ns"]) and delays.index(max(delays)) == int(st["argmax_event"])
    ctx.close()


@pytest.mark.gpu
def test_random_config0_online_path():
    """BASELINE configs[0]: the random policy over one 10k-event trace under a single seed, through the
    reference's own surface (LoadConfig -> QueueEvent / decide, randompolicy.go:156-228,300-346), against
    the oracle. 16 entities entity-0..15 (explorepolicytester.go:36), entity-0..3 prioritized,
    30 ms / 100 ms (randompolicy_test.go:53-54), fault probability 0.1, seed 1."""
    from oracle import oracle as O

    cfg = Config({"explorePolicy": "random", "explorePolicyParam": {
        "minInterval": "30ms", "maxInterval": "100ms", "faultActionProbability": 0.1, "seed": 1,
        "prioritizedEntities": [f"entity-{i}" for i in range(4)]}})
    p = ep.Random()
    assert p.LoadConfig(cfg) is None and p.Seed == 1
    rng = np.random.default_rng(0x5EED)
    events = [Event.packet(f"entity-{i % 16}", f"entity-{i % 16}", f"entity-{(i + 1) % 16}",
                           replay_hint=str(int(rng.integers(-2**63, 2**63 - 1))))
              for i in range(10_000)]
    evhash, evclass = p.event_inputs(events)
    assert int((evclass & _lib.NMZ_EV_PRIORITIZED).astype(bool).sum()) == 2500
    st, dl, fl = O.random_sweep(1, 1, evhash, evclass, O.random_params(30_000_000, 100_000_000, 0.1), n_dump=1)
    # batched: the whole trace for the policy's seed in one call
    r = p.Sweep(p.Seed, 1, evhash, evclass, n_dump=1)
    assert np.array_equal(r.delays, dl) and np.array_equal(r.faults, fl) and np.array_equal(r.stats, st)
    # online: one decision per QueueEvent-sized call, on a sample of the trace
    for i in range(0, 10_000, 97):
        assert p.decide(events[i]) == (int(dl[0, i]), bool(fl[0, i]))
    # QueueEvent delivers the decided action after the decided delay (non-blocking)
    for i in range(8):
        p.QueueEvent(events[i])
    got = {}
    for _ in range(8):
        a = p.ActionChan().get(timeout=5)
        got[a.Event().ID()] = a.Class()
    for i in range(8):
        assert got[events[i].ID()] == ("PacketFaultAction" if fl[0, i] else "EventAcceptanceAction")
    # delays lie in [0.8 min, max) and prioritized entities in [0.8 min, 0.8 max)
    pr = (evclass & _lib.NMZ_EV_PRIORITIZED).astype(bool)
    assert dl[0][pr].min() >= 24_000_000 and dl[0][pr].max() < 80_000_000
    assert dl[0][~pr].min() >= 30_000_000 and dl[0][~pr].max() < 100_000_000
