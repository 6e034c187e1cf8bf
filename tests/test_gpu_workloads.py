"""BASELINE configs 3 and 4 at their stated sizes, on the GPU.

Ranks share the one GPU of the box (separate processes, IPC-mapped FIFOs):
  * config 4 — reduce-scatter then all-gather of a 4 GiB bf16 bucket per rank,
    on the default path and with the direct path forced;
  * config 3 — all-reduce of 1 GiB fp32 per rank, ring and direct forced and
    the library's choice.
Every output is checked over the whole buffer with the integer pattern
(exact in any fold order), and — with hashed fp inputs of varied exponent —
bit-exactly at sampled windows straddling every channel-part boundary, a
sample of the chunk boundaries and random positions, against the CPU
oracle's fold in VCCL's ring order (tests/_workload.py).  At 2 ranks a sum of
two values does not depend on the order; the 4-rank case (arc-balanced ring
set, 6 rings on 14 channels) and the 8-rank case (library defaults, the 7-ring
set on the channels eight ranks sharing one GPU get) do.
"""
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch

from tests import _mp
from tests import _ring
from tests import _workload as W
from tests._util import assert_bitexact

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from tests.test_gpu_collectives import TEST_GEOM  # noqa: E402
from vccl_amd import nccl  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = ["c4", "c4_direct", "c3_ring", "c3_direct", "c3_default"]


def _run(n, geom):
    env = dict(os.environ)
    env.setdefault("VCCL_SPIN_TIMEOUT_S", "30")
    if geom == "test":
        env.update(TEST_GEOM)
        nch, slot, nt = int(TEST_GEOM["VCCL_NCHANNELS"]), int(TEST_GEOM["VCCL_SLOT_BYTES"]), 512
    else:
        # geom "xgmi" / "xgmi_fences": one rank per GPU, the
        # latter with system-scope fences around every FIFO slot
        if geom == "xgmi_fences":
            env["VCCL_FENCES"] = "1"
        # library defaults: nothing overridden — no channel, LL-grid or
        # direct-grid knob — so the co-residency caps that ranks sharing one
        # GPU get (host/init.cc: 7/8 of the CUs / sharing ranks, for ring
        # channels and the LL / direct grids alike; the fix of the 8-rank
        # capture abort, 10b3277) are what runs
        for k in TEST_GEOM:
            env.pop(k, None)
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        nch, slot, nt = _mp.shared_channel_cap(n, _ring.n_channels(n), cus), 512 << 10, 512
    uid = nccl.get_unique_id()
    hexid = nccl.unique_id_to_bytes(uid).hex()
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "mp_workload_worker.py"),
                                   str(r), str(n), hexid, d, str(nch), str(slot), str(nt), ",".join(CASES)],
                                  env=_mp.worker_env(env), stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(n)]
        logs = []
        for p in procs:
            try:
                out, _ = p.communicate(timeout=500)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            logs.append(out.decode(errors="replace")[-3000:])
        codes = [p.returncode for p in procs]
        assert codes == [0] * n, f"worker exit codes {codes}\n" + "\n".join(logs)
        res = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(n)]
    return res, (nch, slot, nt)


_NDEV = torch.cuda.device_count()
_MULTI = [(min(_NDEV, 8), g) for g in ("xgmi", "xgmi_fences")] if _NDEV >= 2 else [(2, "xgmi")]


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("n,geom", [(2, "default"), (4, "test"), (8, "default")] + _MULTI)
def test_baseline_workloads_full_size(n, geom):
    if geom.startswith("xgmi") and _NDEV < n:
        pytest.skip(f"one rank per GPU needs {n} GPUs; this box has {_NDEV}")
    res, geo = _run(n, geom)
    # config 4: pattern over the whole outputs
    for case in ("c4", "c4_direct"):
        for r in range(n):
            assert bool(res[r][f"{case}_pattern_rs"]), f"{case} RS pattern, rank {r}"
            assert bool(res[r][f"{case}_pattern_ag"]), f"{case} AG pattern, rank {r}"
        assert str(res[0]["c4_direct_algo_rs"]) == "direct"
    rc = (4 << 30) // 2 // n
    win, work = W.rs_windows(rc, 2, n, *geo)
    exp = [W.expected_rs_windows(9, win, n, r, rc, work) for r in range(n)]
    for case in ("c4", "c4_direct"):
        for r in range(n):
            assert_bitexact(9, res[r][f"{case}_rs_win"], exp[r], what=f"{case} RS windows n={n} rank {r}")
            assert_bitexact(9, res[r][f"{case}_ag_win"], np.concatenate(exp),
                            what=f"{case} AG windows n={n} rank {r}")
    # config 3
    count = (1 << 30) // 4
    win3, work3 = W.ar_windows(count, 4, n, *geo)
    exp3 = W.expected_ar_windows(7, win3, n, work3)
    for case in ("c3_ring", "c3_direct", "c3_default"):
        for r in range(n):
            assert bool(res[r][f"{case}_pattern"]), f"{case} pattern, rank {r}"
            assert_bitexact(7, res[r][f"{case}_win"], exp3, what=f"{case} windows n={n} rank {r}")
    assert str(res[0]["c3_ring_algo"]) == "ring" and str(res[0]["c3_direct_algo"]) == "direct"
