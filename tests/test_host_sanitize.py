"""Host code of the library under AddressSanitizer + UndefinedBehaviorSanitizer
(`make sanitize`: the host objects rebuilt instrumented, linked with the
regular device objects; tools/host_api_check.cc drives the planner exports,
selection parsing, op encoding and argument checks on random inputs — no
GPU call).  The reference's ASAN=1 / UBSAN=1 build knobs
(makefiles/common.mk:98-109).  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs hipcc")
def test_host_api_under_asan_ubsan():
    p = subprocess.run(["make", "-s", "sanitize"], cwd=ROOT, capture_output=True, text=True, timeout=900)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-3000:]
    assert "0 failures" in out, out[-2000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-3000:]
