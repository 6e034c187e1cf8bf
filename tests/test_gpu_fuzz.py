"""Randomised soak of every collective path (tools/fuzz_coll.py) inside the
GPU suite: ranks sharing the GPU draw the same seeded sequence of
all-reduce / reduce-scatter / all-gather / broadcast / reduce calls over
every element type and reduction, ragged counts up to 4 MiB, in place or
not, the path automatic or forced (ring, direct, LL, LL128), in runs of up to
4 calls per group — and every output is compared bit for bit with the
reduction folded on the device.  The long runs (3 / 8 ranks, net transport,
4000 groups each) are in profiles/r06fz."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,seed,net", [(2, 11, False), (3, 12, False), (2, 13, True)])
def test_fuzz_collectives_bit_exact(world, seed, net):
    env = dict(os.environ, FUZZ_SEED=str(seed), FUZZ_ITERS="300", FUZZ_MAX_BYTES=str(4 << 20),
               FUZZ_SECONDS="60", FUZZ_REPORT="100")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "VCCL_NET_FORCE"):
        env.pop(k, None)
    if net:
        env["VCCL_NET_FORCE"] = "1"
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), os.path.join(ROOT, "tools", "fuzz_coll.py")],
                       env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    bad = [ln for ln in p.stdout.splitlines() if ln.startswith('{"mismatch_at"')]
    assert p.returncode == 0 and not bad, (bad, p.stderr[-3000:])
    summary = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith('{"summary"')][-1])
    assert summary["all_exact"] and summary["world"] == world and summary["iters"] > 0
    assert len(summary["by_type"]) >= 8 and {"sum", "max", "min"} <= set(summary["by_op"])
    sent = summary["net_stats"][0]
    assert (sent > 0) if net else (sent == 0), summary["net_stats"]
