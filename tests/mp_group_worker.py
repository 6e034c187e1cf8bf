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
from tests import _ring  # noqa: E402
from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402

GROUP_RS = [(f"rs{i}", 9, (8 << 20) // 2) for i in range(16)]        # (name, dtype, bucket elements)
GROUP_AR = [(f"ar{i}", 7, (2 << 20) // 4 + 37 * i) for i in range(8)]
# ADVICE r3 (direct batches of very different sizes): all-reduces of 1.1 MiB
# and 4 MiB, reduce-scatters of 5 MiB and 48 MiB buckets (f32), interleaved —
# on the direct path under the test geometry at 4 ranks, one fused launch per
# collective whose parts differ ~4-10x in size (one block length for all)
MIXED_RS = [("mrs0", 7, (48 << 20) // 4), ("mrs1", 7, (5 << 20) // 4), ("mrs2", 7, (48 << 20) // 4 + 4096)]
MIXED_AR = [("mar0", 7, (1 << 20) // 4 + 70_000), ("mar1", 7, (4 << 20) // 4), ("mar2", 7, 300_001)]
SETS = {"zero": (GROUP_RS, GROUP_AR, 1), "mixed": (MIXED_RS, MIXED_AR, 3)}


def call_list(group_rs, group_ar, reps, n):
    """The group's calls in call order, as _ring.group_works takes them:
    interleaved RS / AR when reps > 1, else every RS then every AR."""
    rs = [("rs", 0, dt, count // n) for _, dt, count in group_rs]
    ar = [("ar", 0, dt, count) for _, dt, count in group_ar]
    if reps == 1:
        return rs + ar
    out = []
    for i in range(max(len(rs), len(ar))):
        out += ([rs[i]] if i < len(rs) else []) + ([ar[i]] if i < len(ar) else [])
    return out


def gen(name, dt, count, rank):
    rng = np.random.default_rng(zlib.crc32(name.encode()) * 16 + rank)
    x = rng.uniform(-1, 1, count).astype(np.float32)
    return O.f32_to_bf16_bits(x) if dt == 9 else x


def main():
    rank, n = int(sys.argv[1]), int(sys.argv[2])
    uid = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[3]))
    outdir = sys.argv[4]
    group_rs, group_ar, reps = SETS[sys.argv[5] if len(sys.argv) > 5 else "zero"]
    _mp.bind(rank, n)
    comm = nccl.Comm.init_rank(n, uid, rank)
    s = torch.cuda.current_stream().cuda_stream
    bufs = {}
    for name, dt, count in group_rs + group_ar:
        x = gen(name, dt, count, rank)
        xb = torch.from_numpy(x.view(np.uint8).copy()).cuda()
        nout = count // n if (name, dt, count) in group_rs else count
        yb = torch.empty(nout * x.dtype.itemsize, dtype=torch.uint8, device="cuda")
        bufs[name] = (xb, yb, x.dtype)
    # every call's path: its aggregate's (ncclPrepareTasks, _ring.group_algos)
    calls = call_list(group_rs, group_ar, reps, n)
    group_algos = _ring.group_algos(calls, n, comm.coll_algo)
    algos = {"rs": group_algos[[c[0] for c in calls].index("rs")],
             "ar": group_algos[[c[0] for c in calls].index("ar")]}
    torch.cuda.synchronize()
    res, fused = {}, 0
    for rep in range(reps):
        for name, (xb, yb, npdt) in bufs.items():
            yb.fill_(0xFF)  # NaN / all-ones: stale output cannot pass
        torch.cuda.synchronize()
        f0 = comm.launch_stats()[1]
        nccl.group_start()
        # reduce-scatters and all-reduces interleaved in call order (the
        # planner bins them per collective)
        for i in range(max(len(group_rs), len(group_ar))):
            if i < len(group_rs):
                name, dt, count = group_rs[i]
                xb, yb, _ = bufs[name]
                comm.reduce_scatter(xb.data_ptr(), yb.data_ptr(), count // n, dt, nccl.ncclSum, s)
            if i < len(group_ar) and reps > 1:
                name, dt, count = group_ar[i]
                xb, yb, _ = bufs[name]
                comm.all_reduce(xb.data_ptr(), yb.data_ptr(), count, dt, nccl.ncclSum, s)
        if reps == 1:
            for name, dt, count in group_ar:
                xb, yb, _ = bufs[name]
                comm.all_reduce(xb.data_ptr(), yb.data_ptr(), count, dt, nccl.ncclSum, s)
        nccl.group_end()
        torch.cuda.synchronize()
        fused = comm.launch_stats()[1] - f0
        for name, (xb, yb, npdt) in bufs.items():
            out = yb.cpu().numpy().view(npdt)
            if rep == 0:
                res[name] = out
            elif not np.array_equal(out.view(np.uint8), res[name].view(np.uint8)):
                res[name + "_differs"] = np.array(rep)
    res["fused"] = np.array(fused)
    res["algo_rs"] = np.array(algos["rs"])
    res["algo_ar"] = np.array(algos["ar"])
    res["group_algos"] = np.array(group_algos)
    codes = {"ar": 0, "rs": 1, "ag": 2}
    res["lib_group_algos"] = np.array(comm.group_algos([(codes[c], cnt, dt, op) for c, op, dt, cnt in calls]))
    err = comm.async_error()
    comm.destroy()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **res)
    sys.exit(0 if err == 0 else 3)


if __name__ == "__main__":
    main()
