"""CPU: host-side mirror of the reference interfaces (config, policies'
LoadConfig, signal model, storage reader) -- no device calls."""
import json
import os

import numpy as np
import pytest

from namazu_amd import explorepolicy as ep
from namazu_amd import historystorage as hs
from namazu_amd.config import Config, DurationError, parse_duration, to_duration
from namazu_amd.signal import Event, fnv1a64, go_json


# ---- Go time.ParseDuration / cast.ToDuration ----------------------------------
@pytest.mark.parametrize("s,ns", [("30ms", 30_000_000), ("100ms", 100_000_000), ("1s", 10**9), ("10s", 10**10),
                                  ("1.5s", 1_500_000_000), ("1h2m3.5s", 3_723_500_000_000), ("-5ms", -5_000_000),
                                  ("0", 0), (".5us", 500), ("1µs", 1000), ("1μs", 1000), ("2h", 7_200_000_000_000),
                                  ("1.000000001s", 1_000_000_001), ("+3ns", 3)])
def test_parse_duration(s, ns):
    assert parse_duration(s) == ns


@pytest.mark.parametrize("s", ["", "ms", "1", "1x", ".s", "1.2.3s", "9223372036854775808ns", "-"])
def test_parse_duration_errors(s):
    with pytest.raises(DurationError):
        parse_duration(s)


def test_cast_to_duration():
    assert to_duration("100") == 100  # no unit letter -> ns appended
    assert to_duration(1_000_000) == 1_000_000
    assert to_duration(2.9) == 2
    assert to_duration("3ms") == 3_000_000


# ---- replayable LoadConfig (replayablepolicy.go:63-90) --------------------------
def test_replayable_defaults(monkeypatch):
    monkeypatch.delenv("NMZ_REPLAY_SEED", raising=False)
    p = ep.Replayable()
    assert p.LoadConfig(Config({"explorePolicy": "replayable"})) is None
    assert p.MaxInterval == 10_000_000 and p.Seed == ""
    assert p.Name() == "replayable"


def test_replayable_params_and_env(monkeypatch):
    monkeypatch.delenv("NMZ_REPLAY_SEED", raising=False)
    cfg = Config()
    cfg.set("explorePolicy", "replayable")
    cfg.set("explorePolicyParam", {"maxInterval": 1_000_000_000, "seed": "foobar"})  # replayablepolicy_test.go:54-61
    p = ep.Replayable()
    assert p.LoadConfig(cfg) is None
    assert (p.MaxInterval, p.Seed) == (1_000_000_000, "foobar")
    monkeypatch.setenv("NMZ_REPLAY_SEED", "fromenv")
    assert p.LoadConfig(cfg) is None and p.Seed == "fromenv"


# ---- random LoadConfig (randompolicy_test.go:61-102) -----------------------------
def test_random_policy_parameters():
    p = ep.Random()
    assert p.LoadConfig(Config.from_toml('explorePolicy = "random"\n[explorePolicyParam]\n')) is None
    assert p.MinInterval == 0 and p.MaxInterval == 0
    assert p.PrioritizedEntities == {}
    assert p.ShellActionInterval == 0 and p.ShellActionCommand == ""
    assert p.FaultActionProbability < 0.01

    toml = '''
explorePolicy = "randomBADBAD"
[explorePolicyParam]
  minInterval = "30ms"
  maxInterval = "100ms"
  prioritizedEntities = ["foo", "bar", "baz"]
  shellActionInterval = "10s"
  shellActionCommand = "echo hello world"
  faultActionProbability = 0.1
  thisParameterDoesNotExistButShouldNotMatter = 42
  procPolicy = "dirichlet"

[explorePolicyParam.procPolicyParam]
  resetProbability = 0.0
'''
    p = ep.Random()
    assert p.LoadConfig(Config.from_toml(toml)) is None
    assert p.MinInterval == 30_000_000 and p.MaxInterval == 100_000_000
    assert p.PrioritizedEntities == {"foo": True, "bar": True, "baz": True}
    assert p.ShellActionInterval == 10_000_000_000
    assert p.ShellActionCommand == "echo hello world"
    assert p.FaultActionProbability > 0.09
    assert p.ProcPolicy == "dirichlet"


def test_random_max_defaults_to_min():
    p = ep.Random()
    assert p.LoadConfig(Config.from_toml('[explorePolicyParam]\n minInterval = "5ms"\n')) is None
    assert p.MaxInterval == 5_000_000


@pytest.mark.parametrize("toml,msg", [
    ('[explorePolicyParam]\n faultActionProbability = 1.5\n', "bad faultActionProbability"),
    ('[explorePolicyParam]\n shellActionInterval = "-1s"\n', "must be non-negative"),
    ('[explorePolicyParam]\n procPolicy = "nope"\n', "bad procPolicy"),
    ('[explorePolicyParam]\n procPolicy = "dirichlet"\n[explorePolicyParam.procPolicyParam]\n'
     ' resetProbability = 2.0\n', "resetProbability")])
def test_random_config_errors(toml, msg):
    err = ep.Random().LoadConfig(Config.from_toml(toml))
    assert err is not None and msg in str(err)


def test_registry():
    p, err = ep.CreatePolicy("replayable")
    assert err is None and p.Name() == "replayable"
    p, err = ep.CreatePolicy("random")
    assert err is None and p.Name() == "random"
    p, err = ep.CreatePolicy("nonexistent")
    assert p is None and err is not None


# ---- signal model ------------------------------------------------------------------
def test_event_semantics():
    e = Event.packet("entity-0", "zk1", "zk2", {"x": 1}, replay_hint="h1")
    assert e.ReplayHint() == "h1" and e.Deferred() and e.faultable()
    assert e.DefaultAction().Class() == "EventAcceptanceAction"
    assert e.DefaultFaultAction().Class() == "PacketFaultAction"
    nd = Event.packet("entity-0", "zk1", "zk2", deferred=False)
    assert nd.DefaultFaultAction() is None and nd.DefaultAction().Class() == "NopAction"
    assert Event({"class": "LogEvent", "entity": "e"}).DefaultFaultAction() is None
    assert Event({"class": "NopEvent"}).ReplayHint() == ""


def test_evhash_equals_semantics():
    a = Event.packet("entity-0", "zk1", "zk2", {"message": {"zxid": 1.0}})
    b = Event.packet("entity-0", "zk1", "zk2", {"message": {"zxid": 1}})  # new uuid, int vs float
    c = Event.packet("entity-1", "zk1", "zk2", {"message": {"zxid": 1}})
    assert a.ID() != b.ID()
    assert a.Equals(b) and a.evhash() == b.evhash()
    assert not a.Equals(c) and a.evhash() != c.evhash()


def test_go_json_canonical_form():
    assert go_json({"b": [1, "<&>"], "a": None, "c": -9.223372036854776e+18, "d": 1e-7, "e": True}) == \
        '{"a":null,"b":[1,"\\u003c\\u0026\\u003e"],"c":-9223372036854776000,"d":1e-7,"e":true}'
    assert fnv1a64(b"foobar") == 0x85944171F73967E8


# ---- storage reader ----------------------------------------------------------------
def _make_storage(root, traces, results=None):
    os.makedirs(root, exist_ok=True)
    with open(os.path.join(root, "config.toml"), "w") as f:
        f.write('storageType = "naive"\n')
    for i, tr in enumerate(traces):
        adir = os.path.join(root, "%08x" % i, "actions")
        os.makedirs(adir)
        for n, ev in enumerate(tr):
            json.dump(ev.DefaultAction().JSONMap(), open(os.path.join(adir, f"{n}.action.json"), "w"))
            json.dump(ev.JSONMap(), open(os.path.join(adir, f"{n}.event.json"), "w"))
        res = {"successful": bool((results or [True] * len(traces))[i]), "required_time": 1000 + i, "metadata": {}}
        json.dump(res, open(os.path.join(root, "%08x" % i, "result.json"), "w"))


def test_naive_reader(tmp_path):
    evs = [Event.packet(f"entity-{i % 3}", "a", "b", {"n": i}) for i in range(6)]
    _make_storage(str(tmp_path), [evs[:4], evs[1:6], evs[:4]], results=[True, False, True])
    st = hs.LoadStorage(str(tmp_path))
    assert st is not None and st.Name() == "naive"
    assert st.NrStoredHistories() == 3
    t0, err = st.GetStoredHistory(0)
    assert err is None and len(t0) == 4
    t2, _ = st.GetStoredHistory(2)
    assert t0.Equals(t2)  # re-recorded events have new uuids, still Equal
    t1, _ = st.GetStoredHistory(1)
    assert not t0.Equals(t1)
    assert list(t0.symbols) == [e.evhash() for e in evs[:4]]
    assert st.IsSuccessful(1) == (False, None)
    assert st.GetRequiredTime(2) == (1002, None)
    assert st.GetStoredHistory(7)[1] is not None
    ts = st.load_all()
    assert len(ts) == 3 and list(ts.trace(1)) == list(t1.symbols)


def test_storage_factory():
    s, err = hs.New("naive", "/tmp/x")
    assert err is None and s.Name() == "naive"
    assert hs.New("bogus", "/tmp/x")[1] is not None


def test_to_csr():
    off, data = ep.to_csr(["", "ab", "c"])
    assert list(off) == [0, 0, 2, 3] and bytes(data[:3]) == b"abc"
    off, data = ep.to_csr([])
    assert list(off) == [0]
    assert isinstance(np.asarray(off)[0], np.uint32)
