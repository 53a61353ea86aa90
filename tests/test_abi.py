"""CPU: the C-ABI library builds, loads, exports every declared symbol, and its
host-only entry points follow the reference semantics (no device needed)."""
import ctypes
import os
import re

import pytest

from namazu_amd import _lib
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "nmz_gpu.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(nmz_[a-z0-9_]+)\s*\(", hdr)))


def test_library_loads_and_exports_all_declared_symbols():
    L = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), f"{s} declared in include/nmz_gpu.h but not exported"
    # and the ctypes binding covers every declared entry point
    assert set(syms) <= set(_lib.SIGNATURES)


def test_abi_version():
    assert _lib.load().nmz_abi_version() == 1


def test_gfx950_code_object_present():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_params_resolve_matches_reference_semantics():
    for (mn, mx, p) in [(30_000_000, 100_000_000, 0.1), (0, 0, 0.0), (80_000_000, 3_000_000_000, 0.5),
                        (7, 9, 0.999), (-5_000_000, 5_000_000, 1.0), (123456789, 987654321, 0.3)]:
        got = _lib.resolve_random_params(mn, mx, p)
        exp = O.random_params(mn, mx, p)
        assert list(got.min_ns) == list(exp.min_ns)
        assert list(got.max_ns) == list(exp.max_ns)
        assert got.fault_threshold == exp.fault_threshold


@pytest.mark.parametrize("p", [-0.1, 1.0000001, float("nan")])
def test_params_resolve_rejects_bad_probability(p):
    with pytest.raises(_lib.NmzInvalidArgument, match="bad faultActionProbability"):
        _lib.resolve_random_params(0, 0, p)


def test_params_resolve_rejects_min_gt_max():
    with pytest.raises(_lib.NmzInvalidArgument, match="minDuration"):
        _lib.resolve_random_params(100, 10, 0.1)


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.NmzLibraryError):
        _lib.load()


def test_null_ctx_is_an_error_not_a_crash():
    L = _lib.load()
    assert L.nmz_close(None) == 0
    rc = L.nmz_replayable_sweep(None, None, None, 0, None, None, 0, 0, None, None, 0, 0, None)
    assert rc == _lib.NMZ_EINVAL
    assert "ctx is NULL" in _lib.last_error()
    assert L.nmz_timing_enable(None, 1) == _lib.NMZ_EINVAL
    out = ctypes.c_void_p()
    assert L.nmz_open(-1, ctypes.byref(out)) != 0
