"""CPU checks of the C-ABI library: it loads, exports every symbol declared in
include/*.h (plus the pnccl* aliases), and its host-only entry points behave.
No GPU call is made."""
import ctypes
import os
import re

from oracle import oracle as O
from vccl_amd import nccl

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if not h.endswith(".h"):
            continue
        text = open(os.path.join(ROOT, "include", h)).read()
        names |= set(re.findall(r"^\s*(?:ncclResult_t|const char\*|int|void)\s+(p?(?:nccl|vccl)[A-Z]\w*)\s*\(",
                                text, flags=re.M))
    return names


def test_every_declared_symbol_exported():
    L = nccl.lib()
    declared = _declared()
    assert "ncclAllReduce" in declared and "pncclReduceScatter" in declared
    assert "vcclReduceCopy" in declared
    missing = [n for n in declared if not hasattr(L, n)]
    assert not missing, missing
    for n in nccl.EXPORTED:
        assert n in declared, n


def test_version_and_errors():
    assert nccl.get_version() == 22662  # NCCL_VERSION(2,26,62)
    L = nccl.lib()
    for code in range(8):
        assert L.ncclGetErrorString(code)
    L.pncclGetErrorString.restype = ctypes.c_char_p
    assert L.pncclGetErrorString(4) == L.ncclGetErrorString(4)


def test_host_to_dev_redop_matches_oracle():
    for op in range(5):
        for t in range(12):
            for n in (1, 2, 3, 8):
                assert nccl.host_to_dev_redop(op, t, n) == O.host_to_dev_redop(op, t, n), (op, t, n)
    # fp8 avg scalar fp8(float(1/n)) (enqueue.cc:2265-2272) over every rank
    # count up to 4096 (RN-even ties, subnormal scalars, the E4M3 zero)
    for t in (10, 11):
        for n in range(1, 4097):
            assert nccl.host_to_dev_redop(4, t, n) == O.host_to_dev_redop(4, t, n), (t, n)
    assert nccl.lib().vcclHostToDevRedOp(0, 12, 1, ctypes.byref(ctypes.c_int()),
                                         ctypes.byref(ctypes.c_uint64())) == nccl.ncclInvalidArgument


def test_unique_id_is_fresh():
    a = nccl.unique_id_to_bytes(nccl.get_unique_id())
    b = nccl.unique_id_to_bytes(nccl.get_unique_id())
    assert len(a) == 128 and a != b
    assert nccl.unique_id_to_bytes(nccl.unique_id_from_bytes(a)) == a


def test_null_comm_queries():
    L = nccl.lib()
    v = ctypes.c_int()
    assert L.ncclCommCount(None, ctypes.byref(v)) == nccl.ncclInvalidArgument
    assert L.ncclCommDestroy(None) == nccl.ncclSuccess
    assert L.ncclAllReduce(None, None, 1, 7, 0, None, None) == nccl.ncclInvalidArgument
    n = ctypes.c_ulonglong(7)
    assert L.vcclCommSetRingWave(None, 1, ctypes.byref(n)) == nccl.ncclInvalidArgument and n.value == 7
    assert L.vcclCommSetFences(None, 1) == nccl.ncclInvalidArgument


def test_out_of_scope_calls_are_invalid_usage():
    """Send / Recv / AllToAll(v) are exported (include/nccl.h) so a
    libnccl-linked binary loads, and refuse loudly."""
    L = nccl.lib()
    vp = ctypes.c_void_p
    # reduce and broadcast are implemented: a NULL comm is an invalid argument
    assert L.ncclReduce(vp(0x10), vp(0x10), ctypes.c_size_t(4), 7, 0, 0, None, None) == nccl.ncclInvalidArgument
    assert L.ncclBcast(vp(0x10), ctypes.c_size_t(4), 7, 0, None, None) == nccl.ncclInvalidArgument
    assert L.ncclBroadcast(vp(0x10), vp(0x10), ctypes.c_size_t(4), 7, 0, None, None) == nccl.ncclInvalidArgument
    assert L.ncclSend(vp(0x10), ctypes.c_size_t(4), 7, 1, None, None) == nccl.ncclInvalidUsage
    assert L.ncclRecv(vp(0x10), ctypes.c_size_t(4), 7, 1, None, None) == nccl.ncclInvalidUsage
    out = vp(0x1234)  # ncclCommSplit is implemented: a NULL parent is an invalid argument
    assert L.ncclCommSplit(None, 0, 0, ctypes.byref(out), None) == nccl.ncclInvalidArgument
    assert out.value is None
    assert L.pncclSend(vp(0x10), ctypes.c_size_t(4), 7, 1, None, None) == nccl.ncclInvalidUsage
    # RCCL's all-to-all extensions (imported by PyTorch's ROCm build)
    assert L.ncclAllToAll(vp(0x10), vp(0x10), ctypes.c_size_t(4), 7, None, None) == nccl.ncclInvalidUsage
    assert L.ncclAllToAllv(vp(0x10), None, None, vp(0x10), None, None, 7, None, None) == nccl.ncclInvalidUsage


def test_group_simulate_end_and_registration():
    """ncclGroupSimulateEnd ends the group (nothing launched, no estimate:
    out of scope); the next group is clean.  Registration needs a comm
    (no-op otherwise); ncclCommInitRankScalable refuses an empty id list;
    ncclMemAlloc of 0 bytes is a null pointer (no GPU needed for these)."""
    L = nccl.lib()

    class SimInfo(ctypes.Structure):
        _fields_ = [("size", ctypes.c_size_t), ("magic", ctypes.c_uint), ("version", ctypes.c_uint),
                    ("estimatedTime", ctypes.c_float)]
    info = SimInfo(ctypes.sizeof(SimInfo), 0x74685283, nccl.get_version(), 0.0)
    assert L.ncclGroupSimulateEnd(ctypes.byref(info)) == nccl.ncclInvalidUsage  # not in a group
    nccl.group_start()
    assert L.ncclGroupSimulateEnd(ctypes.byref(info)) == nccl.ncclInvalidUsage
    assert info.estimatedTime == -1.0
    nccl.group_start()
    nccl.group_end()  # the thread is out of the first group
    h = ctypes.c_void_p()
    assert L.ncclCommRegister(None, ctypes.c_void_p(0x10), ctypes.c_size_t(16), ctypes.byref(h)) == \
        nccl.ncclInvalidArgument
    assert L.ncclCommDeregister(None, None) == nccl.ncclInvalidArgument
    out = ctypes.c_void_p(0x1234)
    assert L.ncclCommInitRankScalable(ctypes.byref(out), 2, 0, 0, None, None) == nccl.ncclInvalidArgument
    p = ctypes.c_void_p(0x1234)
    assert L.ncclMemAlloc(ctypes.byref(p), ctypes.c_size_t(0)) == nccl.ncclSuccess and p.value is None
    assert L.ncclMemFree(None) == nccl.ncclSuccess


def test_group_with_failing_call_launches_nothing():
    """ncclGroupErrCheck (enqueue.cc:2516) / group.cc:528,591: one invalid call
    inside a group makes the outermost ncclGroupEnd fail; the next group is clean."""
    L = nccl.lib()
    nccl.group_start()
    assert L.ncclAllReduce(None, None, 1, 7, 0, None, None) == nccl.ncclInvalidArgument
    n = ctypes.c_ulonglong(7)
    assert L.vcclCommSetRingWave(None, 1, ctypes.byref(n)) == nccl.ncclInvalidArgument and n.value == 7
    assert L.vcclCommSetFences(None, 1) == nccl.ncclInvalidArgument
    assert L.ncclGroupEnd() == nccl.ncclInvalidArgument
    nccl.group_start()
    nccl.group_end()
    # nested: the error surfaces only at the outermost end
    nccl.group_start()
    nccl.group_start()
    assert L.ncclReduceScatter(None, None, 1, 99, 0, None, None) == nccl.ncclInvalidArgument
    assert L.ncclGroupEnd() == nccl.ncclSuccess
    assert L.ncclGroupEnd() == nccl.ncclInvalidArgument


def test_reset_debug_init_reloads_level():
    """ncclResetDebugInit (nccl.h.in:191-193): NCCL_DEBUG is re-read, so a
    WARN is silenced under NONE and printed again under WARN (a child process
    owns the C-level stderr)."""
    code = r"""
import ctypes, os, sys
sys.path.insert(0, sys.argv[1])
from vccl_amd import nccl
L = nccl.lib()
def warn():  # a NULL-comm call: WARN + invalid argument, no GPU needed
    L.ncclReduce(ctypes.c_void_p(16), ctypes.c_void_p(16), ctypes.c_size_t(4), 7, 0, 0, None, None)
os.environ["NCCL_DEBUG"] = "NONE"; L.ncclResetDebugInit(); warn()
sys.stderr.flush(); print("--mark--", file=sys.stderr, flush=True)
os.environ["NCCL_DEBUG"] = "WARN"; L.pncclResetDebugInit(); warn()
"""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("NCCL_DEBUG", "VCCL_DEBUG")}
    r = subprocess.run([sys.executable, "-c", code, ROOT], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    before, after = r.stderr.split("--mark--")
    assert "WARN" not in before, before
    assert "WARN" in after, after


def test_get_last_error_returns_the_warn_text():
    """ncclGetLastError (init.cc:2223-2225, debug.cc:29 / :265-272): the text
    of the last WARN, kept whatever NCCL_DEBUG says; comm unused (NULL here).
    A NULL-comm ncclCommCount is ncclInvalidArgument and WARNs (no GPU needed)."""
    code = r"""
import ctypes, os, sys
sys.path.insert(0, sys.argv[1])
from vccl_amd import nccl
L = nccl.lib()
os.environ["NCCL_DEBUG"] = "NONE"; L.ncclResetDebugInit()
assert nccl.last_error() == "", nccl.last_error()
v = ctypes.c_int()
assert L.ncclCommCount(None, ctypes.byref(v)) == nccl.ncclInvalidArgument
print(nccl.last_error())
assert L.ncclAllReduce(None, None, 1, 99, 0, None, None) == nccl.ncclInvalidArgument
print(L.pncclGetLastError(ctypes.c_void_p(0x10)).decode())
"""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("NCCL_DEBUG", "VCCL_DEBUG")}
    r = subprocess.run([sys.executable, "-c", code, ROOT], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    first, second = r.stdout.splitlines()[-2:]
    assert first == "ncclCommCount : comm argument is NULL", first
    assert "NULL" in second or "invalid" in second.lower(), second
    assert "WARN" not in r.stderr  # NCCL_DEBUG=NONE: nothing printed, the text still kept


def test_debug_file(tmp_path):
    """NCCL_DEBUG_FILE (debug.cc:209-255): with an explicit level above
    VERSION the log goes to the named file — %h the host name (up to its
    first '.'), %p the pid, %% a '%', other %-sequences kept — and not to
    stderr; ncclResetDebugInit closes it and a later NCCL_DEBUG_FILE opens
    the next one."""
    code = r"""
import ctypes, os, socket, sys
sys.path.insert(0, sys.argv[1])
from vccl_amd import nccl
L = nccl.lib()
d = sys.argv[2]
def warn():  # a NULL-comm call: WARN + invalid argument, no GPU needed
    v = ctypes.c_int()
    L.ncclCommCount(None, ctypes.byref(v))
os.environ["NCCL_DEBUG"] = "WARN"
os.environ["NCCL_DEBUG_FILE"] = os.path.join(d, "a.%h.%p.%%.%q.log")
L.ncclResetDebugInit(); warn()
os.environ["NCCL_DEBUG_FILE"] = os.path.join(d, "b.%p.log")
L.ncclResetDebugInit(); warn(); warn()
print(os.getpid(), socket.gethostname().split(".")[0])
"""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("NCCL_DEBUG", "VCCL_DEBUG", "NCCL_DEBUG_FILE",
                                                            "VCCL_DEBUG_FILE")}
    r = subprocess.run([sys.executable, "-c", code, ROOT, str(tmp_path)], capture_output=True, text=True,
                       env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    pid, host = r.stdout.split()
    a = tmp_path / f"a.{host}.{pid}.%.%q.log"
    b = tmp_path / f"b.{pid}.log"
    assert sorted(p.name for p in tmp_path.iterdir()) == sorted([a.name, b.name])
    assert a.read_text().count("WARN") == 1 and b.read_text().count("WARN") == 2
    assert "comm argument is NULL" in b.read_text()
    assert "WARN" not in r.stderr, r.stderr
