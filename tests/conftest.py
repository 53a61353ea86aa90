import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libnmz_gpu.so on the device)")


@pytest.fixture(autouse=True)
def _production_env(monkeypatch):
    """Every test starts from a production environment: no NMZ_* variable from the caller's shell reaches the
    library (the A/B and test knobs, csrc ab_env, are read only under NMZ_AB=1, and NMZ_REPLAY_SEED changes
    Replayable.LoadConfig)."""
    for k in [k for k in os.environ if k.startswith("NMZ_")]:
        monkeypatch.delenv(k)


@pytest.fixture
def ab_knobs(monkeypatch):
    """NMZ_AB=1 for a test that sets an A/B or test knob (the library ignores the knobs without it;
    tests/test_ed_gpu.py::test_knobs_need_nmz_ab checks that)."""
    monkeypatch.setenv("NMZ_AB", "1")


@pytest.fixture(scope="session")
def ctx():
    """Device context; a GPU test must fail loudly if the HIP library is missing."""
    from namazu_amd import _lib
    c = _lib.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="session")
def golden():
    import json

    def load(name):
        with open(os.path.join(ROOT, "tests", "golden", name)) as f:
            return json.load(f)
    return load
