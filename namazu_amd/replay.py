"""Feedback loop: GPU schedule search -> `nmz run` replay.

A seed sweep ranks schedules by the failure-candidate score (n_fault desc,
sum_delay desc, seed asc; nmz_topk_entry). This module turns the top-k
entries into what the reference's run path consumes to replay one schedule:

* replayable policy: the seed *string* goes to `explorepolicyparam.seed`
  (replayablepolicy.go:74-81) or, overriding it, the environment variable
  NMZ_REPLAY_SEED (replayablepolicy.go:83-87). `nmz run <storage>` reads the
  storage's config.toml (cli/run.go:65-73) and calls policy.LoadConfig
  (cli/run.go:123-136), so either route reaches determineInterval.
* random policy: the u64 seed goes to `explorepolicyparam.seed`, the
  determinism-contract parameter of this engine.

The top-k `seed` field of a replayable sweep is the index into the seed list
that was swept (nmz_replayable_sweep: seed = index); of a random sweep it is
the seed itself (seed0 + i).
"""
from .config import Config

REPLAY_SEED_ENV = "NMZ_REPLAY_SEED"  # replayablepolicy.go:83
UINT64_MAX = (1 << 64) - 1
INT64_MIN = -(1 << 63)


def as_int64(seed):
    """u64 seed -> the int64 with the same bits. TOML integers (and Go's TOML/viper decoders) are
    int64, so seeds >= 2^63 are written as negative numbers; Random.LoadConfig masks them back
    with & (2^64-1)."""
    seed = int(seed) & UINT64_MAX
    return seed - (1 << 64) if seed >= (1 << 63) else seed


def _is_sentinel(e):
    """A padding entry of a top-k list shorter than k (topk_sentinel(), csrc/topk_dev.h)."""
    return int(e["seed"]) == UINT64_MAX and int(e["sum_delay_ns"]) == INT64_MIN and int(e["n_fault"]) == 0


def replayable_seeds(topk, seeds):
    """Top-k entries of a replayable sweep over `seeds` -> seed strings, best first."""
    out = []
    for e in topk[:len(seeds)]:
        idx = int(e["seed"])
        if _is_sentinel(e) or idx >= len(seeds):  # fewer seeds than k
            break
        s = seeds[idx]
        out.append(s.decode() if isinstance(s, bytes) else str(s))
    return out


def random_seeds(topk, seed0, n_seeds):
    """Top-k entries of a random sweep over seed0..seed0+n_seeds-1 -> u64 seeds, best first."""
    out = []
    # at most n_seeds real entries; padding is recognised by its full signature, not by its seed
    # value (a range that wraps past 2^64 can hold UINT64_MAX as a real seed)
    for e in topk[:n_seeds]:
        s = int(e["seed"])
        if _is_sentinel(e) or (s - seed0) % (1 << 64) >= n_seeds:
            break
        out.append(s)
    return out


def replay_env(seed, environ=None):
    """Environment for `nmz run` that replays a replayable-policy schedule."""
    env = dict(environ or {})
    env[REPLAY_SEED_ENV] = str(seed)
    return env


def replay_config(cfg: Config, seed):
    """A copy of `cfg` whose explore-policy parameter `seed` replays the schedule.

    replayable: seed string; random: int seed (the engine's restatement parameter).
    """
    out = Config(cfg.all_settings())
    policy = out.get_string("explorePolicy").lower()
    if policy == "replayable":
        out.set("explorePolicyParam.seed", str(seed))
    elif policy == "random":
        out.set("explorePolicyParam.seed", as_int64(seed))
    else:
        raise ValueError(f"policy {policy!r} has no replay seed")
    return out


def to_toml(cfg: Config):
    """Serialise a Config to TOML text (the storage's config.toml, historystorage.go:30)."""
    def val(v):
        if isinstance(v, bool):
            return "true" if v else "false"
        if isinstance(v, (int, float)):
            return repr(v)
        if isinstance(v, (list, tuple)):
            return "[" + ", ".join(val(x) for x in v) + "]"
        return '"' + str(v).replace("\\", "\\\\").replace('"', '\\"') + '"'

    def emit(d, prefix, lines):
        tables = []
        for k, v in d.items():
            if isinstance(v, dict):
                tables.append((k, v))
            else:
                lines.append(f"{k} = {val(v)}")
        for k, v in tables:
            name = f"{prefix}.{k}" if prefix else k
            lines.append("")
            lines.append(f"[{name}]")
            emit(v, name, lines)
        return lines

    return "\n".join(emit(cfg.all_settings(), "", [])) + "\n"
