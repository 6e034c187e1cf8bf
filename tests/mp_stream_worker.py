#!/usr/bin/env python3
"""One rank of the cross-stream ordering test (tests/test_gpu_collectives.py).

argv: rank nranks uid_hex
Calls of one comm OUTSIDE any group, issued back to back on three streams in
turn with no host synchronisation: LL, direct / ring all-reduces, reduce-
scatters and all-gathers of several sizes.  Two calls of one comm must never
run at once (they share FIFOs, LL slots and inbox regions): the library
orders each launch after the previous one through the comm's ordering event
(bound to the previous kernel's completion).  Every output checked exactly
(integer-valued patterns, exact in any fold order); exit 0 on success.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402

# (collective, bytes per rank of the input)
PLAN = [("ar", 4096), ("ar", 1 << 20), ("rs", 256 << 10), ("ar", 64), ("ag", 64 << 10),
        ("ar", 6 << 20), ("rs", 8 << 20), ("ar", 32 << 10), ("ag", 4 << 20), ("ar", 12 << 20)]


def main():
    rank, n = int(sys.argv[1]), int(sys.argv[2])
    uid = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[3]))
    _mp.bind(rank, n)
    comm = nccl.Comm.init_rank(n, uid, rank)
    streams = [torch.cuda.Stream() for _ in range(3)]
    calls = []
    for rep in range(4):
        for i, (coll, nbytes) in enumerate(PLAN):
            k = rep * len(PLAN) + i
            cnt = nbytes // 4
            if coll == "rs":
                cnt = cnt // n * n
            x = torch.empty(cnt, device="cuda")
            if coll == "ag":
                x.fill_(float(rank * 1000 + k))
                y = torch.full((cnt * n,), float("nan"), device="cuda")
            else:
                bench.pattern_fill(x, rank, n, base=k << 16)
                y = torch.full((cnt // n if coll == "rs" else cnt,), float("nan"), device="cuda")
            calls.append((coll, cnt, x, y, k))
    torch.cuda.synchronize()
    for j, (coll, cnt, x, y, k) in enumerate(calls):
        sp = streams[j % 3].cuda_stream
        if coll == "ar":
            comm.all_reduce(x.data_ptr(), y.data_ptr(), cnt, nccl.ncclFloat32, nccl.ncclSum, sp)
        elif coll == "rs":
            comm.reduce_scatter(x.data_ptr(), y.data_ptr(), cnt // n, nccl.ncclFloat32, nccl.ncclSum, sp)
        else:
            comm.all_gather(x.data_ptr(), y.data_ptr(), cnt, nccl.ncclFloat32, sp)
    torch.cuda.synchronize()
    bad = []
    for coll, cnt, x, y, k in calls:
        if coll == "ar":
            ok = bench.pattern_ok(y, n, base=k << 16)
        elif coll == "rs":  # this rank's block of the summed pattern
            ok = bench.pattern_ok(y, n, base=(k << 16) + rank * (cnt // n))
        else:
            want = torch.cat([torch.full((cnt,), float(r * 1000 + k), device="cuda") for r in range(n)])
            ok = bool(torch.equal(y, want))
        if not ok:
            bad.append((coll, cnt, k))
    err = comm.async_error()
    comm.destroy()
    if bad or err:
        print(f"rank {rank}: bad {bad} async error {err}", flush=True)
        sys.exit(1)
    sys.exit(0)


if __name__ == "__main__":
    main()
