"""The N > 1 bench line end to end on the GPU: `bench.py
--gpus 2` starts its own two rank processes (one per GPU where the box has
two, sharing the one GPU otherwise) and prints rank 0's line.  The line must
carry the roofline of the topology it ran on — the device's HBM when the
ranks share a GPU, the ring set's xGMI ceiling when each has its own — with
frac <= 1 on a shared device, a checked host-core baseline for configs 3, 4
and 5, and a correct verdict for every timed path."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_line_roofline_and_cpu_baseline():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("VCCL_ALLOW_SHARED_DEVICE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                        "--warmup", "1", "--bytes", str(64 << 20), "--no-extras", "--no-initall"],
                       env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["unit"] == "GB/s" and line["value"] > 0
    assert line["correct"]["all"] is True, line["correct"]
    rpd = line["config"]["devices"]["ranks_per_device"]
    roof = line["roofline"]
    if rpd > 1:
        assert roof["bound"] == "hbm" and 0 < roof["frac"] <= 1, roof
    else:
        assert roof["bound"] == "xgmi" and roof["links"] == 1, roof
    cpu = line["cpu_baseline"]
    assert cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["kind"] == "port", cpu
    assert "checked bit-exactly" in cpu["sample"]
    for name in ("config4_rs_ag_bf16", "config5_ll_f16"):
        assert cpu["other_configs"][name]["value"] > 0, cpu["other_configs"]


def test_broken_path_line_fails_fast():
    """A path that fails during the headline timing (here every net slot
    check trips: VCCL_NET_FORCE + VCCL_DEBUG_NET_SHORT_SLOT, ring.hpp
    recv_size_ok) still yields a line, at once: correct false, the async
    error recorded, the extras skipped rather than each fresh comm waiting
    out its own spin timeout."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update({"VCCL_NET_FORCE": "1", "VCCL_DEBUG_NET_SHORT_SLOT": str(64 << 10),
                "VCCL_SPIN_TIMEOUT_S": "6"})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--bytes", str(64 << 20), "--no-initall", "--no-cpu"],
                       env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    c = line["correct"]
    assert c["all"] is False and c["headline_async_error"] != 0, c
    assert "extras_skipped" in c and "extras" not in line, sorted(line)
    assert line["config"]["async_error"] != 0


def test_error_mid_extras_still_prints_line():
    """The headline passes, then a later row breaks the comm (a 64 KiB
    headline on the forced net path moves no slot of 512 KiB; the first extras
    row that does lands short): the ranks see the error at different calls,
    yet the line prints — the refused calls are recorded (bench._Tolerant),
    the remaining extras rows are skipped at the next error gate, and every
    check reports false instead of raising."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update({"VCCL_NET_FORCE": "1", "VCCL_DEBUG_NET_SHORT_SLOT": str(512 << 10),
                "VCCL_SPIN_TIMEOUT_S": "6"})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--bytes", str(64 << 10), "--no-initall", "--no-cpu",
                        "--rs-ag-bytes", str(8 << 20)],
                       env=env, capture_output=True, text=True, timeout=400, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    c = line["correct"]
    assert c["headline_async_error"] == 0 and c["all"] is False, c
    assert "stopped" in line["extras"], sorted(line["extras"])
    assert line["config"]["async_error"] != 0


def test_staging_row_checked():
    """SURVEY §8(d)'s staging row (D2H, H2D, D2H -> host sum -> H2D) as the
    N = 1 line's cpu_baseline carries it, on a 16 MiB bucket: rates positive
    and the staged sum bitwise equal to the device's a + b."""
    sys.path.insert(0, ROOT)
    import bench
    g = torch.Generator(device="cuda").manual_seed(5)
    a = torch.rand(4 << 20, device="cuda", generator=g) * 2 - 1
    b = torch.rand(4 << 20, device="cuda", generator=g) * 2 - 1
    r = bench.staging_rates(a, b, reps=2)
    assert r["correct"] is True and r["bucket_bytes"] == 16 << 20, r
    assert min(r["d2h_GBs"], r["h2d_GBs"], r["staged_reduce_GBs"]) > 0, r
