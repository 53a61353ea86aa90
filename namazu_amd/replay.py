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


def replayable_seeds(topk, seeds):
    """Top-k entries of a replayable sweep over `seeds` -> seed strings, best first."""
    out = []
    for idx in topk["seed"].tolist():
        if idx >= len(seeds):  # sentinel (fewer seeds than k)
            break
        s = seeds[idx]
        out.append(s.decode() if isinstance(s, bytes) else str(s))
    return out


def random_seeds(topk, seed0, n_seeds):
    """Top-k entries of a random sweep over seed0..seed0+n_seeds-1 -> u64 seeds, best first."""
    out = []
    for s in topk["seed"].tolist():
        if (s - seed0) % (1 << 64) >= n_seeds:  # sentinel
            break
        out.append(int(s))
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
        out.set("explorePolicyParam.seed", int(seed))
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
