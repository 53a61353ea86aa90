#!/usr/bin/env python3
"""Generates the golden fixtures in tests/golden/ (run in the dev container).

Provenance of each fixture:
  fnv_kat.json        published FNV-1a 64 test vectors (not generated)
  go_rand_kat.json    published Go math/rand seed-1 outputs (not generated)
  replayable_foobar.json
                      inputs of the reference's own test
                      (nmz/explorepolicy/replayable/replayablepolicy_test.go:41-110:
                      seed "foobar", maxInterval 1s, hint "hint-entity-%d-%d"),
                      expected delays from the CPU oracle (the reference test
                      asserts no values, so these are oracle-pinned)
  random_decisions.json
                      per-decision outputs of the oracle's random-policy
                      restatement (inputs of randompolicy_test.go:46-56:
                      minInterval 30ms, maxInterval 100ms)
  zk_traces.json      the 4 stored ZooKeeper traces shipped with the reference
                      (example/zk-found-2212.ryu/example-result.20150805/0000000{0..3}/
                      actions/*.event.json), reduced to event-hash sequences
                      (namazu_amd.signal canonical JSON + FNV-1a 64), with the
                      oracle's all-pairs distances. Only the hashes are kept,
                      not the event files.
  ed_kat.json         textbook Levenshtein pairs
  zk_store.json       the same 4 stored traces as data: every action map
                      (N.action.json) and event map (N.event.json) in order,
                      so tests can rebuild the naive store and check Search /
                      visualize against the reference's map-equality rule
"""
import glob
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from namazu_amd.signal import Event  # noqa: E402
from oracle import oracle as O  # noqa: E402

REF = "/root/reference"


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", name)


def main():
    dump("fnv_kat.json", {
        "source": "FNV-1a 64-bit published test vectors (offset basis cbf29ce484222325, prime 100000001b3)",
        "vectors": [["", "cbf29ce484222325"], ["a", "af63dc4c8601ec8c"], ["foobar", "85944171f73967e8"]]})
    dump("go_rand_kat.json", {
        "source": "published outputs of Go math/rand with seed 1 (rand.Seed(1) / rand.New(rand.NewSource(1)))",
        "seed": 1,
        "int63": [5577006791947779410, 8674665223082153551, 6129484611666145821, 4037200794235010051,
                  3916589616287113937, 6334824724549167320],
        "intn100": [81, 87, 47, 59, 81, 18, 25, 40, 56, 0],
        "intn10": [1, 7, 7, 9, 1, 8, 5, 0, 6, 0],
        "rng_cooked_head": [-4181792142133755926, -4576982950128230565, 1395769623340756751]})

    cases = []
    for n, entities in [(10, 2), (10, 10)]:
        hints = [f"hint-entity-{i % entities}-{i}" for i in range(n)]
        delays = [O.replayable_interval("foobar", h, 1_000_000_000) for h in hints]
        cases.append({"seed": "foobar", "max_interval_ns": 1_000_000_000, "hints": hints, "delays_ns": delays})
    extra_seeds = ["", "0", "1048575", "foobar", "-1"]
    extra_hints = ["", "-9223372036854775808", "1234567890123456789", "x" * 40]
    for m in [10_000_000, 100_000_000, 1, 2**30 + 7, 2**63 + 3]:
        mi = m if m < 2**63 else m - 2**64  # uint64(negative Duration)
        cases.append({"seed_list": extra_seeds, "max_interval_ns": mi, "hints": extra_hints,
                      "delays_ns": [[O.replayable_interval(s, h, mi) for h in extra_hints] for s in extra_seeds]})
    dump("replayable_foobar.json", {"source": "oracle (replayablepolicy.go:100-114); inputs from "
                                    "replayablepolicy_test.go:41-110 and edge cases", "cases": cases})

    rng = np.random.default_rng(20150805)
    params = [(30_000_000, 100_000_000, 0.1), (0, 0, 0.5), (5_000_000, 5_000_000, 1.0),
              (80_000_000, 3_000_000_000, 0.999), (0, 1 << 20, 0.0), (-5_000_000, 5_000_000, 0.3)]
    recs = []
    for (mn, mx, p) in params:
        pr = O.random_params(mn, mx, p)
        for _ in range(24):
            seed = int(rng.integers(0, 2**63)) * 2 + int(rng.integers(0, 2))
            eh = int(rng.integers(0, 2**63)) * 2 + int(rng.integers(0, 2))
            cls = int(rng.integers(0, 4))
            d, f, nout = O.random_decide(seed, eh, cls, pr)
            recs.append({"min_ns": mn, "max_ns": mx, "p": p, "seed": seed, "evhash": eh, "evclass": cls,
                         "event_seed": O.random_event_seed(seed, eh), "delay_ns": d, "fault": f,
                         "rng_outputs": nout})
    dump("random_decisions.json", {"source": "oracle (randompolicy.go:300-346, util/queue/impl.go:94-128, "
                                   "deterministic per-event seeding contract)", "decisions": recs})

    traces = []
    base = os.path.join(REF, "example/zk-found-2212.ryu/example-result.20150805")
    for d in sorted(glob.glob(os.path.join(base, "0000000?"))):
        files = glob.glob(os.path.join(d, "actions", "*.event.json"))
        files.sort(key=lambda p: int(re.match(r"(\d+)\.event\.json", os.path.basename(p)).group(1)))
        evs = [Event.from_json(open(p).read()) for p in files]
        traces.append({"dir": os.path.relpath(d, REF), "evhash": ["%016x" % e.evhash() for e in evs]})
    seqs = [np.array([int(h, 16) for h in t["evhash"]], np.uint64) for t in traces]
    n = len(seqs)
    full = [[int(O.levenshtein(seqs[i], seqs[j])) for j in range(n)] for i in range(n)]
    band = {str(w): [[int(O.levenshtein_banded(seqs[i], seqs[j], w)) for j in range(n)] for i in range(n)]
            for w in (4, 8, 32)}
    distinct = len(set(h for t in traces for h in t["evhash"]))
    dump("zk_traces.json", {"source": "reference example traces reduced to evhash sequences; distances from the "
                            "oracle", "traces": traces, "levenshtein": full, "banded": band,
                            "distinct_events": distinct})

    store = []
    for d in sorted(glob.glob(os.path.join(base, "0000000?"))):
        files = glob.glob(os.path.join(d, "actions", "*.action.json"))
        idx = sorted(int(re.match(r"(\d+)\.action\.json", os.path.basename(p)).group(1)) for p in files)
        acts, evs = [], []
        for i in idx:
            with open(os.path.join(d, "actions", f"{i}.action.json")) as f:
                acts.append(json.load(f))
            ep = os.path.join(d, "actions", f"{i}.event.json")
            evs.append(json.load(open(ep)) if os.path.exists(ep) else None)
        store.append({"dir": os.path.relpath(d, REF), "actions": acts, "events": evs})
    dump("zk_store.json", {"source": "reference example traces (data), action and event maps in order",
                           "traces": store})

    kat = [("kitten", "sitting", 3), ("flaw", "lawn", 2), ("", "abc", 3), ("abc", "", 3), ("", "", 0),
           ("intention", "execution", 5), ("namazu", "namazu", 0), ("gumbo", "gambol", 2)]
    dump("ed_kat.json", {"source": "textbook Levenshtein distances (bytes as symbols)",
                         "pairs": [{"a": a, "b": b, "d": d} for a, b, d in kat]})


if __name__ == "__main__":
    main()
