#!/usr/bin/env python3
"""Ring all-reduce parameter sweep (run under torch.distributed.run).

For each (NTHREADS, CHANNELS_PER_RING, SLOT_BYTES, FENCES) a fresh comm is
created (the library reads the env at init), an fp32 sum all-reduce of
SWEEP_BYTES per rank is checked bit-exactly (integer-valued inputs: exact in
any fold order) and timed; rank 0 prints one JSON line per config.
"""
import itertools
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vccl_amd import nccl  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    dist.init_process_group("gloo")
    if world > torch.cuda.device_count():
        os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"
    nbytes = int(os.environ.get("SWEEP_BYTES", 256 << 20))
    steps = int(os.environ.get("SWEEP_STEPS", 10))
    n = nbytes // 4
    gens = [torch.Generator(device="cuda").manual_seed(77 + r) for r in range(world)]
    ins = [torch.randint(-64, 64, (n,), device="cuda", generator=g).float() for g in gens]
    x = ins[rank]
    ref = torch.stack(ins).sum(0)
    del ins
    y = torch.empty_like(x)
    sp = torch.cuda.current_stream().cuda_stream
    grid = list(itertools.product(
        [int(v) for v in os.environ.get("SWEEP_THREADS", "512,1024").split(",")],
        [int(v) for v in os.environ.get("SWEEP_CPR", "4,8,16").split(",")],
        [int(v) for v in os.environ.get("SWEEP_SLOT", "131072,262144,524288,1048576").split(",")],
        [int(v) for v in os.environ.get("SWEEP_FENCES", "0,1").split(",")]))
    for nthr, cpr, slot, fences in grid:
        os.environ.update(VCCL_NTHREADS=str(nthr), VCCL_CHANNELS_PER_RING=str(cpr),
                          VCCL_SLOT_BYTES=str(slot), VCCL_FENCES=str(fences))
        obj = [nccl.unique_id_to_bytes(nccl.get_unique_id()) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm = nccl.Comm.init_rank(world, nccl.unique_id_from_bytes(obj[0]), rank)
        y.zero_()
        comm.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum, sp)
        torch.cuda.synchronize()
        ok = bool(torch.equal(y, ref)) and comm.async_error() == 0
        for _ in range(2):
            comm.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum, sp)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            comm.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum, sp)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        t = torch.tensor([dt, 0.0 if ok else 1.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        comm.destroy()
        if rank == 0:
            busbw = nbytes * steps / t[0].item() / 1e9 * 2 * (world - 1) / world
            print(json.dumps({"world": world, "threads": nthr, "ch_per_ring": cpr, "slot": slot,
                              "fences": fences, "busbw": round(busbw, 2),
                              "correct": t[1].item() == 0.0}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
