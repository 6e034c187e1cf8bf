#!/usr/bin/env python3
"""Cost of the system-scope fences (VCCL_FENCES=1 / vcclCommSetFences) on the
paths VERDICT r5 #4 names — the SIMPLE ring at 1 GiB and 1 MiB, the LL
all-reduce at 8 B — fences off and on interleaved FENCE_REPS times on ONE
comm, every row checked once per setting with bench.py's integer pattern.
Run under torch.distributed.run (ranks may share one GPU: a rehearsal).
Rank 0 prints one JSON line.  Measurement tool, not product code."""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from vccl_amd import nccl  # noqa: E402

ROWS = (("ring", 1 << 30, 5), ("ring", 1 << 20, 200), (None, 8, 2000))


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
    reps = int(os.environ.get("FENCE_REPS", 3))
    out = {"world": world, "channels": comm.n_channels(), "rows": []}
    for algo, S, steps in ROWS:
        n = max(1, S // 4)
        x = torch.rand(n, device="cuda")
        y = torch.empty_like(x)
        comm.set_algo(algo)
        used = comm.coll_algo(0, n, nccl.ncclFloat32)
        row = {"bytes": S, "algo": used, "off_us": [], "on_us": [], "ok": {}}
        for fences in (False, True):
            comm.set_fences(fences)
            row["ok"]["on" if fences else "off"] = bench.check_ar(dist, comm, rank, world, S, "f32", algo)
            comm.set_algo(algo)
        for _ in range(reps):
            for fences in (False, True):
                comm.set_fences(fences)
                dt = bench._time_coll(dist, lambda: comm.all_reduce(x.data_ptr(), y.data_ptr(), n,
                                                                    nccl.ncclFloat32, nccl.ncclSum, sp),
                                      steps, 3)
                row["on_us" if fences else "off_us"].append(round(dt / steps * 1e6, 2))
        comm.set_fences(False)
        comm.set_algo(None)
        row["cost"] = round(min(row["on_us"]) / min(row["off_us"]) - 1, 4)
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
