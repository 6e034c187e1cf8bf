#!/usr/bin/env python3
"""Rate of the inter-node path with its staging copies included (north_star:
"the rate including the copies to and from the GPU is measured as well").

Two comms over the same ranks: the default one (xGMI peer memory, SIMPLE ring
forced) and one created with VCCL_NET_FORCE=1, whose every ring connection
goes through host-pinned staging slots and the TCP proxy pair (host/proxy.cc,
the reference's net transport without GPUDirect: src/transport/net.cc:
1293-1482, src/proxy.cc:914-971).  fp32 sum all-reduce at NET_SIZES, each
row checked once with bench.py's integer pattern, then timed; busbw =
(S/t) * 2(n-1)/n with the max time over ranks.  Net rows are also run at
VCCL_NET_NCHANNELS 2 and 16 beside the default 8.  Run under
torch.distributed.run (ranks may share one GPU).  Rank 0 prints one JSON
line.  Measurement tool, not product code."""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from vccl_amd import nccl  # noqa: E402

SIZES = [int(s) for s in os.environ.get("NET_SIZES", f"{1 << 20},{16 << 20},{256 << 20}").split(",")]


def new_comm(rank, world, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        obj = [nccl.unique_id_to_bytes(nccl.get_unique_id()) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return nccl.Comm.init_rank(world, nccl.unique_id_from_bytes(obj[0]), rank)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def rows(comm, rank, world, label, algo):
    sp = torch.cuda.current_stream().cuda_stream
    out = []
    for S in SIZES:
        n = S // 4
        ok = bench.check_ar(dist, comm, rank, world, S, "f32", algo)
        x = torch.rand(n, device="cuda")
        y = torch.empty_like(x)
        steps = max(3, min(200, (64 << 20) // S * 4))
        comm.set_algo(algo)
        dt = bench._time_coll(dist, lambda: comm.all_reduce(x.data_ptr(), y.data_ptr(), n,
                                                            nccl.ncclFloat32, nccl.ncclSum, sp),
                              steps, 2)
        comm.set_algo(None)
        t = dt / steps
        row = {"path": label, "bytes": S, "channels": comm.n_channels(), "us_per_call": round(t * 1e6, 1),
               "busbw_GBs": round(S / t / 1e9 * 2 * (world - 1) / world, 2), "correct": bool(ok)}
        out.append(row)
        if rank == 0:
            print(f"# {row}", file=sys.stderr, flush=True)
        del x, y
    return out


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    if world > torch.cuda.device_count():
        os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"
    dist.init_process_group("gloo")
    res = {"world": world, "ranks_per_device": -(-world // torch.cuda.device_count()), "rows": []}
    comm = new_comm(rank, world, {})
    res["rows"] += rows(comm, rank, world, "xgmi_ring", "ring")
    comm.destroy()
    for nch in (8, 2, 16):
        comm = new_comm(rank, world, {"VCCL_NET_FORCE": "1", "VCCL_NET_NCHANNELS": str(nch)})
        res["rows"] += rows(comm, rank, world, f"net_{nch}ch", None)
        res.setdefault("async_error", {})[f"net_{nch}ch"] = comm.async_error()
        comm.destroy()
    res["correct"] = all(r["correct"] for r in res["rows"])
    if rank == 0:
        print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
