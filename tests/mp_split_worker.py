#!/usr/bin/env python3
"""One rank of the ncclCommSplit test (tests/test_gpu_collectives.py).

argv: rank nranks uid_hex [uid_hex of the CTA-bounded parent]
Splits the n-rank comm by color = rank % 2 with key = -rank (each half in
reversed parent order), and a second split where rank 0 passes
NCCL_SPLIT_NOCOLOR; checks the sub-comms' sizes and ranks and an exact
all-reduce on each (integer pattern), then the parent still works."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402


def allreduce_ok(comm, world, n=300_001, base=0):
    x = torch.empty(n, device="cuda")
    bench.pattern_fill(x, comm.rank, world, base=base)
    y = torch.full_like(x, float("nan"))
    comm.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum,
                    torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return bench.pattern_ok(y, world, base=base)


def main():
    rank, n = int(sys.argv[1]), int(sys.argv[2])
    uid = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[3]))
    _mp.bind(rank, n)
    comm = nccl.Comm.init_rank(n, uid, rank)
    bad = []
    sub = comm.split(rank % 2, -rank)
    members = [r for r in range(n) if r % 2 == rank % 2][::-1]  # ordered by key = -rank
    if sub is None or sub.count != len(members) or sub.rank != members.index(rank):
        bad.append(("split", None if sub is None else (sub.count, sub.rank)))
    elif not allreduce_ok(sub, len(members), base=1 << 20):
        bad.append(("sub all-reduce", rank % 2))
    sub2 = comm.split(-1 if rank == 0 else 7, rank)  # rank 0: NCCL_SPLIT_NOCOLOR
    if rank == 0:
        if sub2 is not None:
            bad.append(("nocolor", sub2.count))
    elif sub2 is None or sub2.count != n - 1 or sub2.rank != rank - 1 or not allreduce_ok(sub2, n - 1, base=2 << 20):
        bad.append(("split2", None if sub2 is None else (sub2.count, sub2.rank)))
    if not allreduce_ok(comm, n, base=3 << 20):
        bad.append(("parent after split", n))
    for c in (sub, sub2):
        if c is not None:
            c.destroy()
    # a split with config NULL takes the parent's config
    # (copyCommConfig, src/init.cc:2160-2161) — a parent bounded to 3 CTAs
    # gives a child of 3 channels, not the default count
    uid2 = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[4])) if len(sys.argv) > 4 else None
    if uid2 is not None:
        bounded = nccl.Comm.init_rank(n, uid2, rank, config=nccl.ncclConfig_t.initializer(maxCTAs=3))
        child = bounded.split(0, rank)
        if bounded.n_channels() != 3 or child is None or child.n_channels() != 3:
            bad.append(("split of a bounded parent", bounded.n_channels(), child and child.n_channels()))
        elif not allreduce_ok(child, n, base=4 << 20):
            bad.append(("bounded child all-reduce", n))
        if child is not None:
            child.destroy()
        bounded.destroy()
    err = comm.async_error()
    comm.destroy()
    if bad or err:
        print(f"rank {rank}: {bad} async error {err}", flush=True)
        sys.exit(1)


if __name__ == "__main__":
    main()
