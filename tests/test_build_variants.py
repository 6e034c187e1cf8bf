"""The ring's opt-in build switches (device/ring.hpp) still compile: scalar
credit polls (VCCL_RING_SPOLL=1) and the non-draining last step
(VCCL_RING_LAST_DRAINS=0) of the per-wave hand-off are not in the default
library, so nothing else would notice them rotting.  Front end only
(-fsyntax-only: parse + template instantiation of the kernels for gfx950),
for the per-wave SIMPLE ring (PART 4, where the switches act) and, with the
switches on, the workgroup SIMPLE and LL128 ring families.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="needs hipcc")
@pytest.mark.parametrize("defs", [
    ["-DVCCL_RING_SPOLL=1"],
    ["-DVCCL_RING_LAST_DRAINS=0"],
    ["-DVCCL_RING_SPOLL=1", "-DVCCL_RING_LAST_DRAINS=0"],
])
@pytest.mark.parametrize("part", [0, 3, 4])
def test_ring_switch_compiles(defs, part):
    cmd = [HIPCC, "-std=c++20", "-O3", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
           "--offload-arch=gfx950", "-I", "include", "-DVCCL_KT=4", f"-DVCCL_PART={part}", *defs,
           "-fsyntax-only", "vccl_amd/csrc/device/ring_kernels.hip"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    assert "error" not in p.stderr, p.stderr[-3000:]
