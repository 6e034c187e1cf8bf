"""The C API as a compiled caller sees it: tools/coll_perf.hip (an
nccl-tests-style driver built against include/nccl.h and linked to
libvccl.so, no Python in the data path) runs all-reduce, reduce-scatter,
all-gather, broadcast and reduce size sweeps with 2 and 3 ranks (processes sharing the box's GPU)
and checks every output element against its closed form."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PERF = os.path.join(ROOT, "vccl_amd", "lib", "coll_perf")


@pytest.mark.parametrize("coll,ranks,dtype,op", [
    ("allreduce", 2, "float", "sum"), ("allreduce", 3, "bfloat16", "sum"),
    ("allreduce", 2, "half", "max"), ("reducescatter", 2, "float", "sum"),
    ("reducescatter", 3, "int32", "min"), ("allgather", 2, "bfloat16", "sum"),
    ("allgather", 3, "float", "sum"), ("broadcast", 3, "half", "sum"),
    ("reduce", 3, "float", "sum"), ("reduce", 2, "int32", "max")])
def test_coll_perf(coll, ranks, dtype, op):
    assert os.path.exists(PERF), "build first: make (vccl_amd/lib/coll_perf)"
    env = dict(os.environ, VCCL_ALLOW_SHARED_DEVICE="1", VCCL_SPIN_TIMEOUT_S="20",
               VCCL_NTHREADS="512", VCCL_LL_MAX_BLOCKS="32", VCCL_DIRECT_MAX_BLOCKS="16",
               VCCL_CHANNELS_PER_RING="8")
    out = subprocess.run([PERF, "-C", coll, "-r", str(ranks), "-b", "8", "-e", str(16 << 20),
                          "-f", "4", "-n", "5", "-w", "2", "-d", dtype, "-o", op, "-R", str(ranks - 1)],
                         env=env, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "# Out of bounds values : 0 OK" in out.stdout, out.stdout[-3000:]
