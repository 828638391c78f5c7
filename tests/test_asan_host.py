"""Host sanitizer run of the C-ABI (SURVEY §5 "ASan host tests"): `make asan` builds api.hip — plan
derivation, argument validation, graph bookkeeping — with AddressSanitizer + UBSan on the host side
(GPU code is never sanitised) and links tests/native/capi_asan.cpp against it.  The driver derives
~200 plans over BASELINE configs 1-5 and edge shapes (checking their layout invariants) and calls
every entry point with invalid arguments; it needs no GPU, since each call returns before any HIP
runtime call.  A sanitizer report aborts the driver (-fno-sanitize-recover=all)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dgp-rf-mcmc_amd", "csrc")


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_capi_host_asan_ubsan():
    jobs = str(min(8, os.cpu_count() or 1))
    b = subprocess.run(["make", "-C", CSRC, f"-j{jobs}", "asan"], capture_output=True, text=True,
                       timeout=1500)
    assert b.returncode == 0, b.stdout[-2000:] + b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(CSRC, "build_asan", "capi_asan")], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "every check passed" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
