#!/usr/bin/env python3
"""One rank of test_gpu_failure.py::test_net_short_slot_is_an_error.

argv: rank nranks outdir uid_hex
Every ring connection goes through the net proxy (VCCL_NET_FORCE=1).  The
caller sets VCCL_DEBUG_NET_SHORT_SLOT=k on rank 0 only: its send proxy ships
its k-th slot 16 bytes short — the stale / short size that produced garbage
in round 5 (gpurun_out/r05c).  The receiving kernel compares the landed byte
count with the slice length it computes itself (ring.hpp recv_size_ok), so
the call must END with an error from ncclCommGetAsyncError — ncclInternalError
at the receiver of the short slot, ncclRemoteError (spin timeout) where a
rank waits on it — never a silent wrong result.  A clean all-reduce runs first
(with the hook's k past it) and must be exact.  Verdict to <outdir>/rank<r>.json."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402


def main():
    rank, n, outdir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    uid = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[4]))
    _mp.bind(rank, n)
    comm = nccl.Comm.init_rank(n, uid, rank)
    s = torch.cuda.current_stream().cuda_stream
    res = {"rank": rank, "net_stats": list(comm.net_stats())}
    # a small exact call first: the first slots of every connection, before
    # the short one
    S0 = 4 << 10
    x0 = torch.empty(S0 // 4, device="cuda")
    y0 = torch.full_like(x0, float("nan"))
    bench.pattern_fill(x0, rank, n)
    comm.all_reduce(x0.data_ptr(), y0.data_ptr(), x0.numel(), nccl.ncclFloat32, nccl.ncclSum, s)
    torch.cuda.synchronize()
    res["first_exact"] = bench.pattern_ok(y0, n) and comm.async_error() == 0
    S = 8 << 20
    x = torch.empty(S // 4, device="cuda")
    y = torch.full_like(x, float("nan"))
    bench.pattern_fill(x, rank, n)
    torch.cuda.synchronize()
    t0 = time.monotonic()
    rc = 0
    try:
        comm.all_reduce(x.data_ptr(), y.data_ptr(), x.numel(), nccl.ncclFloat32, nccl.ncclSum, s)
    except nccl.VcclError as e:
        rc = e.code
    torch.cuda.synchronize()  # the kernel must end by itself (size guard or spin timeout)
    res["kernel_end_s"] = round(time.monotonic() - t0, 2)
    res["enqueue_rc"] = rc
    res["async_error"] = comm.async_error()
    res["exact"] = bench.pattern_ok(y, n)
    res["last_error"] = nccl.last_error()
    res["wave_launches"] = comm.set_ring_wave(None)
    comm.abort()
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
