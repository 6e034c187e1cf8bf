"""Non-blocking communicators (VERDICT r5 missing #4): with
ncclConfig_t.blocking = 0 or NCCL_COMM_BLOCKING=0, ncclCommInitRank* returns
ncclInProgress at once, the initialisation runs on a thread of its own, and
ncclCommGetAsyncError reports ncclInProgress until it has ended, then its
result (the reference's group.cc:553-576 helper thread and init.cc:1836-1860
async state); the comm then runs collectives exactly (tests/
mp_nonblocking_worker.py, two ranks)."""
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


def test_nonblocking_init_reports_in_progress_then_success():
    n = 2
    env = _mp.worker_env(os.environ)
    env.pop("NCCL_COMM_BLOCKING", None)
    uids = [nccl.unique_id_to_bytes(nccl.get_unique_id()).hex() for _ in range(2)]
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "mp_nonblocking_worker.py"),
                                   str(r), str(n), d, *uids], env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(n)]
        logs = []
        for p in procs:
            try:
                logs.append(p.communicate(timeout=240)[0].decode(errors="replace")[-3000:])
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
        assert [p.returncode for p in procs] == [0] * n, "\n".join(logs)
        for r in range(n):
            with open(os.path.join(d, f"rank{r}.json")) as f:
                v = json.load(f)
            assert v["config_rc"] == nccl.ncclInProgress and v["config_state"] == nccl.ncclSuccess, v
            assert v["config_polls"] >= 1 and v["config_exact"], v
            assert v["env_rc"] == nccl.ncclInProgress and v["env_state"] == nccl.ncclSuccess and v["env_exact"], v


_ABORT_PENDING = r"""
import ctypes, json, sys, time
sys.path.insert(0, %r)
import torch
from vccl_amd import nccl
torch.cuda.set_device(0)
uid = nccl.get_unique_id()  # the root lives here; rank 1 never comes
cfg = nccl.ncclConfig_t.initializer(blocking=0)
h = ctypes.c_void_p()
rc = nccl.lib().ncclCommInitRankConfig(ctypes.byref(h), 2, uid, 0, ctypes.byref(cfg))
time.sleep(1.0)
st = ctypes.c_int(-1)
nccl.lib().ncclCommGetAsyncError(h, ctypes.byref(st))
# ncclCommEnsureReady: a comm still initialising is not usable, not waited for
cnt = ctypes.c_int(-1)
rc_count = nccl.lib().ncclCommCount(h, ctypes.byref(cnt))
x = torch.zeros(4, device="cuda")
rc_ar = nccl.lib().ncclAllReduce(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(x.data_ptr()), ctypes.c_size_t(4),
                                 nccl.ncclFloat32, nccl.ncclSum, h, ctypes.c_void_p(0))
rc_destroy = nccl.lib().ncclCommDestroy(h)
t0 = time.monotonic()
rc_abort = nccl.lib().ncclCommAbort(h)
print(json.dumps({"rc": rc, "state_before": st.value, "rc_count": rc_count, "rc_ar": rc_ar,
                  "rc_destroy": rc_destroy, "rc_abort": rc_abort, "abort_s": round(time.monotonic() - t0, 2)}))
"""


def test_abort_ends_a_pending_nonblocking_init():
    """ncclCommAbort on a non-blocking comm whose initialisation waits for a
    peer that never comes (a 2-rank comm, rank 1 absent): the bootstrap
    socket is shut, the init thread ends, abort returns within seconds — not
    after the 600 s bootstrap timeout.  Before that, every other use of the
    comm fails at once with ncclInvalidArgument, as the reference's
    ncclCommEnsureReady makes it (init.cc:300-317; destroy too, :2066)."""
    p = subprocess.run([sys.executable, "-c", _ABORT_PENDING % ROOT], capture_output=True, text=True,
                       timeout=120, env=_mp.worker_env(os.environ))
    assert p.returncode == 0, p.stderr[-3000:]
    v = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert v["rc"] == nccl.ncclInProgress and v["state_before"] == nccl.ncclInProgress, v
    assert v["rc_count"] == v["rc_ar"] == v["rc_destroy"] == nccl.ncclInvalidArgument, v
    assert v["rc_abort"] == nccl.ncclSuccess and v["abort_s"] < 10, v
