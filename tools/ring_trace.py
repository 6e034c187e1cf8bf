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

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("VCCL_RING_TRACE", "2048")
from vccl_amd import nccl  # noqa: E402

SHAPES = {0b0110: "S->F", 0b0111: "S+F->F", 0b1111: "S+F->F+O", 0b1101: "S+F->O", 0b1011: "F->F+O",
          0b1001: "F->O", 0b1110: "S->F+O"}


def summarize(tr):
    rows = {}
    for ch in range(tr.shape[0]):
        rec = tr[ch][tr[ch]["t4"] > 0]
        for i, r in enumerate(rec):
            d = rows.setdefault(SHAPES.get(int(r["shape"]), str(int(r["shape"]))),
                                {"n": 0, "wait": 0.0, "release": 0.0, "copy": 0.0, "post": 0.0, "gap": 0.0,
                                 "issue": 0.0, "drain": 0.0, "bytes": 0})
            d["n"] += 1
            d["wait"] += (int(r["t1"]) - int(r["t0"])) / 100.0  # us (100 MHz)
            d["release"] += (int(r["t2"]) - int(r["t1"])) / 100.0
            d["copy"] += (int(r["t3"]) - int(r["t2"])) / 100.0
            d["post"] += (int(r["t4"]) - int(r["t3"])) / 100.0
            if int(r["tc"]):  # copy = issue (thread 0's accesses issued) + drain (pipeline empty, all waves)
                d["issue"] += (int(r["tc"]) - int(r["t2"])) / 100.0
                d["drain"] += (int(r["t3"]) - int(r["tc"])) / 100.0
            if i + 1 < len(rec):
                d["gap"] += (int(rec[i + 1]["t0"]) - int(r["t4"])) / 100.0
            d["bytes"] += int(r["bytes"])
    out = {}
    for k, d in rows.items():
        n = d["n"]
        out[k] = {"n": n, **{f: round(d[f] / n, 2) for f in ("wait", "release", "copy", "issue", "drain", "post",
                                                              "gap")},
                  "payload_GBs_in_copy": round(d["bytes"] / (d["copy"] * 1e3), 1) if d["copy"] else None}
    return out


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
