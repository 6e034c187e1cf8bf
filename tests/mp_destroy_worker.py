#!/usr/bin/env python3
"""One rank of test_gpu_failure.py::test_destroy_right_after_launch.

argv: rank nranks outdir uid_hex
Every rank launches one 1 GiB f32 ring all-reduce with integer-pattern
inputs and calls ncclCommDestroy straight away, without synchronising.
Destroy must wait for the comm's own launch before it frees the FIFOs: the
stream must be idle when it returns, and the output exact.  The test runs it
with the environment the caller sets (VCCL_DEBUG_NO_MARK=1 with and without a
bound stop event, VCCL_LAUNCH_EVENT=0), since the library reads both once per
process.  Verdict to <outdir>/rank<r>.json."""
import json
import os
import sys

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
    comm.set_algo("ring")
    S = 1 << 30
    x = torch.empty(S // 4, device="cuda")
    y = torch.full_like(x, float("nan"))
    bench.pattern_fill(x, rank, n)
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()
    comm.all_reduce(x.data_ptr(), y.data_ptr(), x.numel(), nccl.ncclFloat32, nccl.ncclSum, stream.cuda_stream)
    busy_at_launch = not stream.query()
    comm.destroy()  # no synchronisation before it
    idle_after_destroy = stream.query()
    torch.cuda.synchronize()
    res = {"rank": rank, "busy_at_launch": busy_at_launch, "idle_after_destroy": idle_after_destroy,
           "exact": bench.pattern_ok(y, n), "no_mark": os.environ.get("VCCL_DEBUG_NO_MARK"),
           "launch_event": os.environ.get("VCCL_LAUNCH_EVENT")}
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
