#!/usr/bin/env python3
"""One rank of the ring slot-timeline test (tests/test_gpu_collectives.py
test_ring_trace_and_shared_cap).

argv: rank nranks uid_hex outdir.  Ring all-reduce of 8 MiB fp32 (integer
values, exact in any order) with VCCL_RING_TRACE set; saves the output check,
the comm's channel count and the trace records (vcclCommRingTrace)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402


def main():
    rank, n, outdir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[4]
    uid = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[3]))
    _mp.bind(rank, n)
    comm = nccl.Comm.init_rank(n, uid, rank)
    comm.set_algo("ring")
    count = 2 << 20
    x = torch.full((count,), float(rank + 1), device="cuda")
    y = torch.empty_like(x)
    sp = torch.cuda.current_stream().cuda_stream
    comm.all_reduce(x.data_ptr(), y.data_ptr(), count, nccl.ncclFloat32, nccl.ncclSum, sp)
    torch.cuda.synchronize()
    ok = bool(torch.all(y == float(n * (n + 1) // 2)).item())
    tr = comm.ring_trace()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), ok=ok, nch=tr.shape[0], cus=cus,
             t=np.stack([tr[k].astype(np.int64) for k in ("t0", "t1", "t2", "tc", "t3", "t4")], axis=-1),
             shape=tr["shape"].astype(np.int64), bytes=tr["bytes"].astype(np.int64))
    comm.destroy()


if __name__ == "__main__":
    main()
