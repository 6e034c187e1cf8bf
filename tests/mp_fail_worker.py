#!/usr/bin/env python3
"""One rank of the failure-path tests (tests/test_gpu_failure.py).

argv: rank nranks outdir mode uid_hex[,uid_hex...]
The LAST rank plays the lost peer: it joins every communicator (init is
collective) but never enqueues a collective; it stays alive, holding its
FIFOs, until every survivor has written <outdir>/done<r>, then aborts its
comms and exits 0.  The survivors:

  peer_loss  — one comm per path (ring, LL, direct, forced with
               vcclCommSetAlgo): an all-reduce that waits on the lost peer
               must END within VCCL_SPIN_TIMEOUT_S (the bounded spins of
               ring.hpp / ll.hpp / direct.hpp), ncclCommGetAsyncError must
               report ncclRemoteError, and ncclCommAbort (ring, direct) /
               ncclCommDestroy (LL: the error skips the teardown barrier a
               lost peer would never join) must return;
  abort      — a ring all-reduce spins on the lost peer with a long spin
               timeout; a second host thread calls ncclCommAbort after 1 s,
               which must end the kernel (primitives.h:142-152 checkAbort;
               init.cc:2079-2111 ncclCommAbort) long before the timeout.
Afterwards the process must still be usable: a torch kernel and a
vcclReduceCopy on the same device give exact results.  Verdicts go to
<outdir>/rank<r>.json.
"""
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402

PATHS = (("ring", int(os.environ.get("FAIL_RING_BYTES", 8 << 20)) // 4 * 4), ("ll", 4 << 10), ("direct", 2 << 20))


def usable_after(res):
    """A torch kernel and the library's reduce-copy still run, exactly."""
    a = torch.arange(1 << 20, device="cuda", dtype=torch.float32)
    b = torch.full_like(a, 3.0)
    d = torch.empty_like(a)
    s = torch.cuda.current_stream().cuda_stream
    srcs = (ctypes.c_void_p * 2)(a.data_ptr(), b.data_ptr())
    dsts = (ctypes.c_void_p * 1)(d.data_ptr())
    rc = nccl.lib().vcclReduceCopy(0, nccl.ncclFloat32, 0, 0, 0, 2, srcs, 1, dsts, a.numel(), s)
    torch.cuda.synchronize()
    res["usable_after"] = rc == 0 and bool(torch.equal(d, a + 3.0)) and float((a * 2).sum()) == float(
        (1 << 20) * ((1 << 20) - 1))


def survivor_peer_loss(comms, res, timeout_s):
    s = torch.cuda.current_stream().cuda_stream
    for (path, nbytes), comm in zip(PATHS, comms):
        comm.set_algo(path)
        n = nbytes // 4
        x = torch.ones(n, device="cuda")
        y = torch.empty_like(x)
        torch.cuda.synchronize()
        t0 = time.monotonic()
        comm.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum, s)
        torch.cuda.synchronize()  # the kernel must end by itself (spin timeout)
        r = {"kernel_end_s": round(time.monotonic() - t0, 2), "async_error": comm.async_error(),
             "algo": comm.coll_algo(0, n, nccl.ncclFloat32)}
        t1 = time.monotonic()
        if path == "ll":
            comm.destroy()
        else:
            comm.abort()
        r["teardown_s"] = round(time.monotonic() - t1, 2)
        r["ok"] = (r["async_error"] == nccl.ncclRemoteError and r["kernel_end_s"] < timeout_s + 15
                   and r["teardown_s"] < 15 and r["algo"] == path)
        res[path] = r


def survivor_abort(comms, res):
    comm = comms[0]
    comm.set_algo("ring")
    s = torch.cuda.current_stream().cuda_stream
    n = (8 << 20) // 4
    x = torch.ones(n, device="cuda")
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    out = {}

    def aborter():
        time.sleep(1.0)
        t = time.monotonic()
        try:
            comm.abort()
            out["abort_rc"] = 0
        except nccl.VcclError as e:
            out["abort_rc"] = e.code
        out["abort_s"] = round(time.monotonic() - t, 2)

    t0 = time.monotonic()
    comm.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum, s)
    th = threading.Thread(target=aborter)
    th.start()
    torch.cuda.synchronize()  # returns once the abort word ended the kernel
    end = time.monotonic() - t0
    th.join(timeout=120)
    r = {"kernel_end_s": round(end, 2), **out}
    r["ok"] = out.get("abort_rc") == 0 and 0.9 < end < 20 and not th.is_alive()
    res["abort_thread"] = r


def main():
    rank, n, outdir, mode = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    uids = [nccl.unique_id_from_bytes(bytes.fromhex(h)) for h in sys.argv[5].split(",")]
    _mp.bind(rank, n)
    comms = [nccl.Comm.init_rank(n, u, rank) for u in uids]
    lost = rank == n - 1
    res = {"rank": rank, "lost_peer": lost}
    timeout_s = int(os.environ.get("VCCL_SPIN_TIMEOUT_S", "60"))
    if lost:
        deadline = time.monotonic() + 240
        while time.monotonic() < deadline and not all(
                os.path.exists(os.path.join(outdir, f"done{r}")) for r in range(n - 1)):
            time.sleep(0.2)
        for c in comms:
            c.abort()  # no launch of its own: returns at once
        res["ok"] = True
    else:
        try:
            if mode == "peer_loss":
                survivor_peer_loss(comms, res, timeout_s)
            else:
                survivor_abort(comms, res)
            usable_after(res)
        finally:
            open(os.path.join(outdir, f"done{rank}"), "w").close()
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
