#!/usr/bin/env python3
"""Graph-mode LL all-reduce latency over a fine size sweep (VERDICT r3 #6:
the 1 KiB fp16 row of the N>1 line ran 5x slower than 8 B and 16 KiB).

Run under torch.distributed.run (ranks may share one GPU).  For each size in
PROBE_SIZES (bytes) and dtype in PROBE_DTYPES: bench._ar_graph_row (50 calls
captured in one HIP graph, replayed; us per call, each replay alone too).
Rank 0 prints one JSON line per row.  Measurement tool, not product code."""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from vccl_amd import nccl  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    if world > torch.cuda.device_count():
        os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"
    dist.init_process_group("gloo")
    obj = [nccl.unique_id_to_bytes(nccl.get_unique_id()) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    comm = nccl.Comm.init_rank(world, nccl.unique_id_from_bytes(obj[0]), rank)
    sizes = [int(v) for v in os.environ.get(
        "PROBE_SIZES", "8,64,256,512,768,1024,1536,2048,4096,8192,16384").split(",")]
    # PROBE_STREAM=fresh: a new capture stream per row (as the bench line);
    # shared: one capture stream for every row
    shared = torch.cuda.Stream() if os.environ.get("PROBE_STREAM", "fresh") == "shared" else None
    for dtype in os.environ.get("PROBE_DTYPES", "f16,f32").split(","):
        for i, S in enumerate(sizes):
            row = bench._ar_graph_row(dist, comm, rank, world, S, dtype, stream=shared)
            if rank == 0:
                row["dtype"] = dtype
                row["row"] = i
                row["stream"] = "shared" if shared is not None else "fresh"
                print(json.dumps(row), flush=True)
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
