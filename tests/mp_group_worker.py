#!/usr/bin/env python3
"""One rank of the group-aggregation test (tests/test_gpu_collectives.py).

argv: rank nranks uid_hex outdir
Inside ONE ncclGroupStart/End: the ZeRO pattern — 16 reduce-scatters of 8 MiB
bf16 buckets (GROUP_RS) — then 8 mid-size fp32 all-reduces (GROUP_AR).  Each
run of same-type calls must launch once (vcclCommLaunchStats: fused
launches); outputs saved for the bit-exact check against the oracle's ring
fold.  Inputs: seeded per (bucket, rank) (tests/ring_cases.py style).
"""
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from vccl_amd import nccl  # noqa: E402

GROUP_RS = [(f"rs{i}", 9, (8 << 20) // 2) for i in range(16)]        # (name, dtype, bucket elements)
GROUP_AR = [(f"ar{i}", 7, (2 << 20) // 4 + 37 * i) for i in range(8)]


def gen(name, dt, count, rank):
    rng = np.random.default_rng(zlib.crc32(name.encode()) * 16 + rank)
    x = rng.uniform(-1, 1, count).astype(np.float32)
    return O.f32_to_bf16_bits(x) if dt == 9 else x


def main():
    rank, n = int(sys.argv[1]), int(sys.argv[2])
    uid = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[3]))
    outdir = sys.argv[4]
    torch.cuda.set_device(0)
    comm = nccl.Comm.init_rank(n, uid, rank)
    s = torch.cuda.current_stream().cuda_stream
    bufs = {}
    for name, dt, count in GROUP_RS + GROUP_AR:
        x = gen(name, dt, count, rank)
        xb = torch.from_numpy(x.view(np.uint8).copy()).cuda()
        nout = count // n if name.startswith("rs") else count
        yb = torch.empty(nout * x.dtype.itemsize, dtype=torch.uint8, device="cuda")
        bufs[name] = (xb, yb, x.dtype)
    algos = {"rs": comm.coll_algo(1, GROUP_RS[0][2] // n, 9), "ar": comm.coll_algo(0, GROUP_AR[0][2], 7)}
    torch.cuda.synchronize()
    f0 = comm.launch_stats()[1]
    nccl.group_start()
    for name, dt, count in GROUP_RS:
        xb, yb, _ = bufs[name]
        comm.reduce_scatter(xb.data_ptr(), yb.data_ptr(), count // n, dt, nccl.ncclSum, s)
    for name, dt, count in GROUP_AR:
        xb, yb, _ = bufs[name]
        comm.all_reduce(xb.data_ptr(), yb.data_ptr(), count, dt, nccl.ncclSum, s)
    nccl.group_end()
    torch.cuda.synchronize()
    fused = comm.launch_stats()[1] - f0
    res = {name: yb.cpu().numpy().view(npdt) for name, (xb, yb, npdt) in bufs.items()}
    res["fused"] = np.array(fused)
    res["algo_rs"] = np.array(algos["rs"])
    res["algo_ar"] = np.array(algos["ar"])
    err = comm.async_error()
    comm.destroy()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **res)
    sys.exit(0 if err == 0 else 3)


if __name__ == "__main__":
    main()
