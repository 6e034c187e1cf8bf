#!/usr/bin/env python3
"""Per-algorithm latency of RS / AG / AR at small and mid buckets (run under
torch.distributed.run; ranks may share one GPU for a protocol rehearsal).

For each collective, bucket size and algorithm in LAT_ALGOS (auto = the
library's choice, or forced ll / direct / ring via vcclCommSetAlgo): one
integer-pattern correctness check (bench.py's checker) then LAT_STEPS timed
calls; rank 0 prints one JSON line per row (max over ranks).
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
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    if world > torch.cuda.device_count():
        os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"
    os.environ.setdefault("VCCL_LL128_ALLOC", "1")  # so LAT_ALGOS may force ll128
    dist.init_process_group("gloo")
    obj = [nccl.unique_id_to_bytes(nccl.get_unique_id()) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    comm = nccl.Comm.init_rank(world, nccl.unique_id_from_bytes(obj[0]), rank)
    sp = torch.cuda.current_stream().cuda_stream
    sizes = [int(v) for v in os.environ.get("LAT_SIZES", "8192,65536,262144,1048576,8388608").split(",")]
    algos = os.environ.get("LAT_ALGOS", "auto,ring,direct,ll").split(",")
    colls = os.environ.get("LAT_COLLS", "rs,ag,ar").split(",")
    steps = int(os.environ.get("LAT_STEPS", 50))
    for coll in colls:
        for S in sizes:
            n = S // 4
            rc = n // world
            x = torch.rand(n, device="cuda")
            y = torch.empty(n if coll != "rs" else rc, device="cuda")
            if coll == "ar":
                fn = lambda: comm.all_reduce(x.data_ptr(), y.data_ptr(), n, 7, 0, sp)  # noqa: E731
            elif coll == "rs":
                fn = lambda: comm.reduce_scatter(x.data_ptr(), y.data_ptr(), rc, 7, 0, sp)  # noqa: E731
            else:
                fn = lambda: comm.all_gather(x.data_ptr(), y.data_ptr(), rc, 7, sp)  # noqa: E731
            for algo in algos:
                comm.set_algo(None if algo == "auto" else algo)
                used = comm.coll_algo({"ar": 0, "rs": 1, "ag": 2}[coll], n if coll == "ar" else rc, 7)
                if algo != "auto" and used != algo:
                    continue  # the forced algorithm cannot carry this bucket
                if coll == "ar":
                    ok = bench.check_ar(dist, comm, rank, world, S, "f32",
                                        None if algo == "auto" else algo)
                else:
                    r_ok, a_ok = bench.check_rs_ag(dist, comm, rank, world, S, "f32",
                                                   None if algo == "auto" else algo)
                    ok = r_ok if coll == "rs" else a_ok
                comm.set_algo(None if algo == "auto" else algo)
                dt = bench._time_coll(dist, fn, steps, 5)
                if rank == 0:
                    print(json.dumps({"coll": coll, "bytes": S, "world": world, "algo": algo,
                                      "used": used, "us": round(dt / steps * 1e6, 2), "correct": ok}),
                          flush=True)
            comm.set_algo(None)
            del x, y
    err = comm.async_error()
    comm.destroy()
    if rank == 0:
        print(json.dumps({"async_error": err}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
