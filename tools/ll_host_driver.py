#!/usr/bin/env python3
"""One rank of a small-bucket all-reduce latency run, separating the host's
enqueue cost from the device time (config 5: is an eager LL call bound by
the host?).  Rendezvous from the environment (RANK, WORLD_SIZE, MASTER_*).

    python tools/ll_host_driver.py [bytes=8] [calls=2000] [dtype=f16]

Per rep: barrier, device synchronize, `calls` back-to-back ncclAllReduce on
one stream (host time of the loop = enqueue cost), then synchronize (total).
Rank 0 prints one JSON line: us per call enqueued and completed (best of 5
reps, max over ranks).  Run under `rocprofv3 --hip-runtime-trace --stats`
for the per-API split.  Measurement tool, not product code."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vccl_amd import nccl  # noqa: E402


def main():
    nbytes = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    dt = {"f16": (torch.float16, 6), "f32": (torch.float32, 7)}[sys.argv[3] if len(sys.argv) > 3 else "f16"]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    if world > torch.cuda.device_count():
        os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"
    dist.init_process_group("gloo")
    obj = [nccl.unique_id_to_bytes(nccl.get_unique_id()) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    comm = nccl.Comm.init_rank(world, nccl.unique_id_from_bytes(obj[0]), rank)
    n = max(1, nbytes // torch.tensor([], dtype=dt[0]).element_size())
    x = torch.ones(n, dtype=dt[0], device="cuda")
    y = torch.empty_like(x)
    sp = torch.cuda.current_stream().cuda_stream
    f = nccl.lib().ncclAllReduce
    h, xp, yp = comm.handle, x.data_ptr(), y.data_ptr()
    for _ in range(50):
        f(xp, yp, n, dt[1], 0, h, sp)
    torch.cuda.synchronize()
    enq, tot = [], []
    for _ in range(5):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            f(xp, yp, n, dt[1], 0, h, sp)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        t = torch.tensor([t1 - t0, t2 - t0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        enq.append(float(t[0]) / calls * 1e6)
        tot.append(float(t[1]) / calls * 1e6)
    ok = comm.async_error() == 0
    algo = comm.coll_algo(0, n, dt[1])
    comm.destroy()
    if rank == 0:
        print(json.dumps({"bytes": nbytes, "calls": calls, "world": world, "algo": algo,
                          "us_enqueue": round(min(enq), 2), "us_total": round(min(tot), 2),
                          "reps_enqueue": [round(v, 2) for v in enq], "reps_total": [round(v, 2) for v in tot],
                          "ok": ok}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
