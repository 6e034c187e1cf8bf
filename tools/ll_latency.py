#!/usr/bin/env python3
"""Where the config-5 eager latency goes: fp16 LL
all-reduces of 8 B - 4 KiB on n ranks, each size timed four ways on one comm:
  eager_us  back-to-back calls, one synchronize at the end (bench.py's row);
  host_us   the host time per call of the same loop, before the synchronize
            (capture query + launch with the bound stop event);
  sync_us   call + synchronize, one at a time (launch-to-completion);
  graph_us  50 calls captured in one graph, replayed (bench.py's graph row).
Max over ranks.  Run under torch.distributed.run with the environment to
A/B (e.g. GPU_MAX_HW_QUEUES, ranks per device).  Rank 0 prints one JSON line.
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


def _max(v):
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    if world > torch.cuda.device_count():
        os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"
    dist.init_process_group("gloo")
    obj = [nccl.unique_id_to_bytes(nccl.get_unique_id()) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    comm = nccl.Comm.init_rank(world, nccl.unique_id_from_bytes(obj[0]), rank)
    sp = torch.cuda.current_stream().cuda_stream
    steps = int(os.environ.get("LAT_STEPS", 200))
    sizes = [int(v) for v in os.environ.get("LAT_SIZES", "8,1024,4096").split(",")]
    out = {"world": world, "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
           "visible": torch.cuda.device_count(), "rows": []}
    for S in sizes:
        n = max(1, S // 2)
        x = (torch.rand(n, device="cuda") * 2 - 1).half()
        y = torch.empty_like(x)

        def call():
            comm.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat16, nccl.ncclSum, sp)
        row = {"bytes": S, "algo": comm.coll_algo(0, n, nccl.ncclFloat16)}
        for _ in range(20):
            call()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            call()
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        te = time.perf_counter() - t0
        dist.barrier()
        row["host_us"] = round(_max(th / steps * 1e6), 2)
        row["eager_us"] = round(_max(te / steps * 1e6), 2)
        row["eager_us_time_coll"] = round(bench._time_coll(dist, call, steps, 5) / steps * 1e6, 2)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps // 4):
            call()
            torch.cuda.synchronize()
        row["sync_us"] = round(_max((time.perf_counter() - t0) / (steps // 4) * 1e6), 2)
        g = bench._ar_graph_row(dist, comm, rank, world, S, "f16", calls=50, replays=10)
        row["graph_us"] = g["us"]
        row["graph_matches_eager"] = g["matches_eager"]
        row["ok"] = bench.check_ar(dist, comm, rank, world, S, "f16")
        out["rows"].append(row)
        if rank == 0:
            print(f"# {row}", file=sys.stderr, flush=True)
        del x, y
    out["async_error"] = comm.async_error()
    comm.destroy()
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
