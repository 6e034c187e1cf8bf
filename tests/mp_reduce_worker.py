#!/usr/bin/env python3
"""One rank of the reduce test (tests/test_gpu_collectives.py).

argv: rank nranks uid_hex outdir
ncclReduce (reduce.h: the ring into the root) over tests/ring_cases.py
REDUCE_CASES with every root: the root's output is saved to
outdir/rank<r>.npz for the parent's oracle check; a non-root passes a NULL
recvbuff (out of place) or its own buffer (in place), which must stay
untouched.  Then ONE group of reduces to different roots with an all-reduce
(fused ring parts with per-part roots).  Exit 0 when the local checks pass."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from tests import ring_cases as RC  # noqa: E402
from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402

# the group: (case index, root) — one aggregate of f32 sums, a bf16 sum
GROUP = [(0, 1), (4, 0), (2, 1), (0, 0)]


def to_dev(x):
    return torch.from_numpy(x.view(np.uint8).copy()).cuda()


def main():
    rank, n = int(sys.argv[1]), int(sys.argv[2])
    uid = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[3]))
    outdir = sys.argv[4]
    _mp.bind(rank, n)
    comm = nccl.Comm.init_rank(n, uid, rank)
    sp = torch.cuda.current_stream().cuda_stream
    res, bad = {}, []
    for ri, (name, op, dt, count, inplace) in enumerate(RC.REDUCE_CASES):
        x = RC.gen_reduce_input(ri, rank)
        for root in range(n):
            xb = to_dev(x)
            if inplace:
                comm.reduce(xb.data_ptr(), xb.data_ptr(), count, dt, op, root, sp)
                yb = xb
            else:
                yb = torch.full((x.nbytes,), 0xCD, dtype=torch.uint8, device="cuda")
                comm.reduce(xb.data_ptr(), yb.data_ptr() if rank == root else 0, count, dt, op, root, sp)
            torch.cuda.synchronize()
            if rank == root:
                res[f"{name}_r{root}"] = yb.cpu().numpy().view(x.dtype)
            elif inplace and not np.array_equal(yb.cpu().numpy(), x.view(np.uint8)):
                bad.append((name, root, "non-root buffer written"))
            if not inplace and not np.array_equal(xb.cpu().numpy(), x.view(np.uint8)):
                bad.append((name, root, "input written"))
    # one group: reduces to different roots + an all-reduce
    ins = [to_dev(RC.gen_reduce_input(ri, rank)) for ri, _ in GROUP]
    outs = [torch.full_like(b, 0xCD) for b in ins]
    calls = []
    x = torch.empty(1 << 20, device="cuda")
    bench.pattern_fill(x, rank, n, base=5 << 20)
    y = torch.full_like(x, float("nan"))
    torch.cuda.synchronize()
    gcalls = [(4, RC.REDUCE_CASES[ri][3], RC.REDUCE_CASES[ri][2], RC.REDUCE_CASES[ri][1]) for ri, _ in GROUP]
    res["group_algos"] = np.array(comm.group_algos(gcalls + [(0, x.numel(), nccl.ncclFloat32, nccl.ncclSum)]))
    nccl.group_start()
    for k, (ri, root) in enumerate(GROUP):
        name, op, dt, count, _ = RC.REDUCE_CASES[ri]
        root %= n
        comm.reduce(ins[k].data_ptr(), outs[k].data_ptr(), count, dt, op, root, sp)
        calls.append((root, ri))
    comm.all_reduce(x.data_ptr(), y.data_ptr(), x.numel(), nccl.ncclFloat32, nccl.ncclSum, sp)
    nccl.group_end()
    torch.cuda.synchronize()
    for k, (root, ri) in enumerate(calls):
        npdt = RC.gen_reduce_input(ri, rank).dtype
        if rank == root:
            res[f"group{k}"] = outs[k].cpu().numpy().view(npdt)
        elif not bool((outs[k] == 0xCD).all()):
            bad.append(("group", k, "non-root output written"))
    if not bench.pattern_ok(y, n, base=5 << 20):
        bad.append(("group all-reduce",))
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **res)
    err = comm.async_error()
    comm.destroy()
    if bad or err:
        print(f"rank {rank}: {bad} async error {err}", flush=True)
        sys.exit(1)


if __name__ == "__main__":
    main()
