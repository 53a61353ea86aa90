"""Feedback loop top-k seeds -> replay (namazu_amd/replay.py).

CPU: the helpers and the reference's config/env route (replayablepolicy.go:74-87).
GPU: a sweep's best schedule, replayed through Replayable.LoadConfig +
determineInterval event by event, reproduces the sweep's statistics; BASELINE configs[0] (the random
policy over one 10k-event trace, single seed) through LoadConfig / decide / QueueEvent vs the oracle."""
import re

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


def test_random_seeds_real_uint64_max_vs_padding():
    """A range wrapping past 2^64 holds UINT64_MAX as a real seed; padding entries (fewer seeds than k)
    carry the sentinel signature and stop the list (csrc/topk_dev.h topk_sentinel)."""
    tk = _topk([2**64 - 1, 2**64 - 2, 2**64 - 1, 2**64 - 1])
    tk["sum_delay_ns"][:2] = [7, 5]
    tk["sum_delay_ns"][2:] = -2**63
    tk["n_fault"][:2] = 1
    assert replay.random_seeds(tk, 2**64 - 3, 3) == [2**64 - 1, 2**64 - 2]
    # n_seeds bounds the list even without a sentinel
    tk2 = _topk([1, 0, 2**64 - 1])
    tk2["sum_delay_ns"] = [3, 2, 1]
    assert replay.random_seeds(tk2, 2**64 - 2, 4) == [1, 0, 2**64 - 1]
    assert replay.random_seeds(tk2, 2**64 - 2, 2) == []
    assert replay.random_seeds(_topk([2**64 - 1, 2**64 - 2, 0]), 2**64 - 2, 2) == [2**64 - 1, 2**64 - 2]


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
    # the emitted TOML integer fits in int64 (Go TOML decoders reject anything larger)
    text = replay.to_toml(replay.replay_config(rnd, 2**63 + 5))
    v = int(re.search(r"^seed = (-?\d+)$", text, re.M).group(1))
    assert -2**63 <= v < 2**63 and v == 2**63 + 5 - 2**64
    for s in (0, 1, 2**63 - 1, 2**63, 2**64 - 1):
        assert -2**63 <= replay.as_int64(s) < 2**63 and replay.as_int64(s) % 2**64 == s
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
