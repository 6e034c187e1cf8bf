#!/usr/bin/env python3
"""Slot timeline of the SIMPLE ring (VCCL_RING_TRACE, vcclCommRingTrace):
run under torch.distributed.run (ranks may share the GPU).  For each
collective in TRACE_COLLS on a TRACE_BYTES fp32 bucket (ring forced): two
warm-up calls, one traced call, then per primitive shape the mean time
waiting for credits (t1-t0), for the workgroup release (t2-t1), moving and
draining the payload (t3-t2: thread 0's accesses issued, tc-t2, then the
drain and the wait for the slowest wave, t3-tc), posting (t4-t3), the gap to the channel's next
slot, and the payload rate of the copy phase.  Rank 0 prints one JSON line
per collective.  Measurement tool, not product code."""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("VCCL_RING_TRACE", "2048")
from vccl_amd import nccl  # noqa: E402

def summarize(tr):
    """Per primitive shape: mean credit wait, release, copy (issue + drain),
    post and gap per slot, and the payload rate of the copy phase
    (bench.ring_trace_summary, shared with the N > 1 bench line)."""
    import bench
    return bench.ring_trace_summary(tr)


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    if world > torch.cuda.device_count():
        os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"
    dist.init_process_group("gloo")
    obj = [nccl.unique_id_to_bytes(nccl.get_unique_id()) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    comm = nccl.Comm.init_rank(world, nccl.unique_id_from_bytes(obj[0]), rank)
    comm.set_algo("ring")
    sp = torch.cuda.current_stream().cuda_stream
    S = int(os.environ.get("TRACE_BYTES", 512 << 20))
    n = S // 4
    x = torch.rand(n, device="cuda")
    y = torch.empty(n, device="cuda")
    for coll in os.environ.get("TRACE_COLLS", "rs,ag,ar").split(","):
        if coll == "ar":
            fn = lambda: comm.all_reduce(x.data_ptr(), y.data_ptr(), n, 7, 0, sp)  # noqa: E731
        elif coll == "rs":
            fn = lambda: comm.reduce_scatter(x.data_ptr(), y.data_ptr(), n // world, 7, 0, sp)  # noqa: E731
        else:
            fn = lambda: comm.all_gather(x.data_ptr(), y.data_ptr(), n // world, 7, sp)  # noqa: E731
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        comm.ring_trace()  # clears
        dist.barrier()
        fn()
        torch.cuda.synchronize()
        tr = comm.ring_trace()
        s = summarize(tr)
        t0 = int(tr["t0"][tr["t0"] > 0].min())
        t4 = int(tr["t4"].max())
        res = [None] * world
        dist.all_gather_object(res, {"rank": rank, "span_us": round((t4 - t0) / 100.0, 1), "shapes": s})
        if rank == 0:
            print(json.dumps({"coll": coll, "bytes": S, "world": world, "channels": tr.shape[0], "ranks": res}),
                  flush=True)
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
