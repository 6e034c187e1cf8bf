#!/usr/bin/env python3
"""One rank of a fixed ring all-reduce run, for counter and A/B passes over
the SIMPLE ring kernel (tools/pmc_ring.py).  Rendezvous from the environment
(RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT; gloo ships the unique id only).

    python tools/ring_ar_driver.py [bytes=1 GiB] [calls=6]

The ring is forced (vcclCommSetAlgo); fp32 sum over `bytes` per rank, one
warmup call then `calls` timed calls, each bracketed by a barrier and a
device synchronize; the output of the last call is checked against the
integer pattern (exact in any fold order).  Rank 0 prints one JSON line:
{"bytes", "calls", "us": [per call, max over ranks], "correct"}.
Measurement tool, not product code."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from vccl_amd import nccl  # noqa: E402


def main():
    nbytes = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    if world > torch.cuda.device_count():
        os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"
    dist.init_process_group("gloo")
    obj = [nccl.unique_id_to_bytes(nccl.get_unique_id()) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    comm = nccl.Comm.init_rank(world, nccl.unique_id_from_bytes(obj[0]), rank)
    comm.set_algo("ring")
    n = nbytes // 4
    x = torch.empty(n, device="cuda")
    y = torch.empty(n, device="cuda")
    bench.pattern_fill(x, rank, world)
    sp = torch.cuda.current_stream().cuda_stream
    comm.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum, sp)
    torch.cuda.synchronize()
    us = []
    for _ in range(calls):
        dist.barrier()
        t0 = time.perf_counter()
        comm.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum, sp)
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        us.append(round(float(t.item()) * 1e6, 1))
    ok = bench.pattern_ok(y, world) and comm.async_error() == 0
    ok = bool(bench._all_ok(dist, ok))
    comm.destroy()
    if rank == 0:
        print(json.dumps({"bytes": nbytes, "calls": calls, "world": world, "us": us, "correct": ok}),
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
