"""Host-side sanitizer runs (SURVEY 4 / .travis.yml:23's `go test -race` counterpart), CPU only:
  * tools/sanitize/build/host_abi_asan  -- libnmz_gpu's host code (every .hip file; device code unchanged)
    under ASan + UBSan: argument validation of every entry point, parameter resolution, clean failure of
    nmz_open without a device, thread-local errors;
  * tools/sanitize/build/host_abi_tsan  -- the same host code under ThreadSanitizer, 8 threads calling into
    the library concurrently (thread-local error messages, argument checks);
  * tools/sanitize/build/oracle_asan    -- the C oracle under ASan + UBSan on edge inputs.
(GPU-side ASan / xnack runs are not available on the MI355X pool.)"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tools", "sanitize")


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-j8", "-C", SAN], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


@pytest.mark.parametrize("binary,env", [
    ("host_abi_asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "UBSAN_OPTIONS": "halt_on_error=1"}),
    ("host_abi_tsan", {"TSAN_OPTIONS": "halt_on_error=1"}),
    ("oracle_asan", {"ASAN_OPTIONS": "detect_leaks=1", "UBSAN_OPTIONS": "halt_on_error=1"}),
])
def test_sanitized_driver(built, binary, env):
    r = subprocess.run([os.path.join(SAN, "build", binary)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **env))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "WARNING: ThreadSanitizer" not in out
    assert "runtime error:" not in out  # UBSan
    assert "checks ok" in r.stdout
