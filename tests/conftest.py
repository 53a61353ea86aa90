import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libnmz_gpu.so on the device)")


@pytest.fixture(autouse=True)
def _ab_knobs(monkeypatch):
    """The library reads its NMZ_* A/B and test knobs only under NMZ_AB=1 (csrc ab_env); the tests that set a knob
    need it. tests/test_ed_gpu.py::test_knobs_need_nmz_ab checks that without it a knob changes nothing."""
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
