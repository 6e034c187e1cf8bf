"""The hot path's failure handling on MI355X.

VCCL polls an abort word in every spin (src/device/primitives.h:142-152) and
ncclCommAbort raises it and reclaims the comm waiting only on its own work
(src/init.cc:2079-2111).  Here every spin of the ring, LL and direct kernels
checks the abort word and a no-progress timeout (VCCL_SPIN_TIMEOUT_S), and
comm_destroy waits on the comm's own launches (host/init.cc
wait_own_launches), never the whole device.  With one rank that never
enqueues (tests/mp_fail_worker.py):
  * the other ranks' ring, LL and direct all-reduce kernels end within the
    spin timeout, ncclCommGetAsyncError reports ncclRemoteError, and
    ncclCommAbort / ncclCommDestroy return;
  * ncclCommAbort from a second host thread ends a kernel spinning on the
    lost peer long before its timeout;
and the process stays usable (a torch kernel and vcclReduceCopy, exact).
"""
import json
import os
import subprocess
import sys
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, mode, ncomms, spin_timeout, wave=0):
    uids = ",".join(nccl.unique_id_to_bytes(nccl.get_unique_id()).hex() for _ in range(ncomms))
    env = _mp.worker_env(os.environ)
    env["VCCL_SPIN_TIMEOUT_S"] = str(spin_timeout)
    # the SIMPLE ring's workgroup (0) or per-wave (1) slot hand-off: each has
    # its own spins (ring.hpp prim_wg / prim_ws), each must end on a lost peer.
    # "mixed" (ADVICE r5): the per-wave kernels at the default
    # VCCL_RING_WAVE_MIN with a ragged ring bucket, so one launch mixes
    # per-wave slots and workgroup slots (prim_ws -> prim_wg) while it aborts
    env["VCCL_RING_WAVE"] = "0" if wave == 0 else "1"
    if wave == "mixed":
        env.pop("VCCL_RING_WAVE_MIN", None)
        env["FAIL_RING_BYTES"] = str((8 << 20) + (96 << 10) + 20)
    else:
        env["VCCL_RING_WAVE_MIN"] = "0"
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "mp_fail_worker.py"),
                                   str(r), str(n), d, mode, uids], env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(n)]
        logs = []
        for p in procs:
            try:
                logs.append(p.communicate(timeout=300)[0].decode(errors="replace")[-3000:])
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
        assert [p.returncode for p in procs] == [0] * n, "\n".join(logs)
        res = []
        for r in range(n):
            with open(os.path.join(d, f"rank{r}.json")) as f:
                res.append(json.load(f))
    return res, "\n".join(logs)


@pytest.mark.parametrize("wave", [0, 1, "mixed"])
def test_lost_peer_ends_ring_ll_direct_kernels(wave):
    n, timeout_s = 3, 3
    res, logs = _run(n, "peer_loss", 3, timeout_s, wave)
    for r in res[:-1]:
        for path in ("ring", "ll", "direct"):
            v = r[path]
            assert v["ok"], (r["rank"], path, v, logs)
            assert v["async_error"] == nccl.ncclRemoteError
        assert r["usable_after"], (r, logs)
    assert res[-1]["ok"] and res[-1]["lost_peer"]


@pytest.mark.parametrize("wave", [0, 1])
def test_abort_from_second_thread_ends_spinning_kernel(wave):
    res, logs = _run(2, "abort", 1, 60, wave)  # the spin timeout alone would take 60 s
    v = res[0]["abort_thread"]
    assert v["ok"], (v, logs)
    assert v["kernel_end_s"] < 20 and v["abort_s"] < 15
    assert res[0]["usable_after"], (res[0], logs)


@pytest.mark.parametrize("no_mark,launch_event", [("0", "1"), ("1", "1"), ("1", "0")])
def test_destroy_right_after_launch(no_mark, launch_event):
    """ncclCommDestroy straight after a launch waits for it in
    every ordering mode — also under VCCL_DEBUG_NO_MARK=1, where no marker is
    recorded (the kernel's bound stop event, or with VCCL_LAUNCH_EVENT=0 the
    stream itself, tracks the launch) — so the FIFOs are never freed under a
    running kernel and the output is exact."""
    n = 2
    env = _mp.worker_env(os.environ)
    env.update(VCCL_DEBUG_NO_MARK=no_mark, VCCL_LAUNCH_EVENT=launch_event)
    uid = nccl.unique_id_to_bytes(nccl.get_unique_id()).hex()
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "mp_destroy_worker.py"),
                                   str(r), str(n), d, uid], env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(n)]
        logs = []
        for p in procs:
            try:
                logs.append(p.communicate(timeout=180)[0].decode(errors="replace")[-3000:])
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
        assert [p.returncode for p in procs] == [0] * n, "\n".join(logs)
        for r in range(n):
            with open(os.path.join(d, f"rank{r}.json")) as f:
                v = json.load(f)
            assert v["idle_after_destroy"] and v["exact"], (v, logs)


@pytest.mark.parametrize("wave", [0, 1])
def test_net_short_slot_is_an_error(wave):
    """a net slot whose landed byte count is not its step's
    slice (VCCL_DEBUG_NET_SHORT_SLOT makes rank 0's proxy ship its first
    slot of >= 64 KiB 16 bytes short, as the stale size of round 5 did) ends
    the call with an error from ncclCommGetAsyncError on every rank —
    ncclInternalError where the short slot landed (ring.hpp recv_size_ok),
    ncclRemoteError where a rank then waits on it — never a silent result;
    the small call before it (slots below the hook's size) is exact.  Both
    hand-offs check (prim_wg, and prim_ws with every slot per wave)."""
    n = 2
    env = _mp.worker_env(os.environ)
    env.update(VCCL_NET_FORCE="1", VCCL_NET_NCHANNELS="2", VCCL_SPIN_TIMEOUT_S="3",
               VCCL_RING_WAVE=str(wave), VCCL_RING_WAVE_MIN="0")
    uid = nccl.unique_id_to_bytes(nccl.get_unique_id()).hex()
    with tempfile.TemporaryDirectory() as d:
        procs = []
        for r in range(n):
            e = dict(env)
            if r == 0:
                e["VCCL_DEBUG_NET_SHORT_SLOT"] = str(64 << 10)
            procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "mp_net_guard_worker.py"),
                                           str(r), str(n), d, uid], env=e,
                                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        logs = []
        for p in procs:
            try:
                logs.append(p.communicate(timeout=180)[0].decode(errors="replace")[-3000:])
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
        assert [p.returncode for p in procs] == [0] * n, "\n".join(logs)
        res = []
        for r in range(n):
            with open(os.path.join(d, f"rank{r}.json")) as f:
                res.append(json.load(f))
    for v in res:
        assert v["first_exact"], (v, logs)
        assert int(v["net_stats"][2]) == 2 * 2, v  # every ring connection through the proxy
        assert v["async_error"] in (nccl.ncclInternalError, nccl.ncclRemoteError), (v, logs)
        assert v["kernel_end_s"] < 30, v
    # rank 1 receives rank 0's short slot and refuses it
    assert res[1]["async_error"] == nccl.ncclInternalError, (res, logs)
    assert (min(v["wave_launches"] for v in res) > 0) == (wave == 1), res  # the hand-off asked for ran
    assert "slice length" in res[1]["last_error"], res[1]
