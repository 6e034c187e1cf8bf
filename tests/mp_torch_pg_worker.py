#!/usr/bin/env python3
"""One rank of the PyTorch drop-in test (tests/test_gpu_collectives.py).

Run with LD_PRELOAD = torch's libamdhip64.so (so one HIP runtime serves
both) then libvccl.so: torch.distributed's "nccl" backend (ProcessGroupNCCL,
the reference's own caller) then resolves ncclCommInitRank*,
ncclAllReduce, ncclReduceScatter, ncclAllGather, ncclGroupStart/End, ... to
this library instead of RCCL.  Both ranks share cuda:0, which RCCL itself
refuses; VCCL_ALLOW_SHARED_DEVICE=1 lets this library run it.  Checks
all_reduce (sum, avg, max), reduce_scatter_tensor and all_gather_into_tensor
exactly, broadcast, reduce, a DistributedDataParallel step (state broadcast at
construction, gradient-bucket all-reduce in backward) and an all_reduce on a
sub-group (new_group); exit 0 on success.  Rendezvous: RANK, WORLD_SIZE, MASTER_ADDR /
MASTER_PORT (TCPStore carries ncclUniqueId)."""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    # one rank per GPU where the box has them (rank % devices); ranks
    # beyond the device count share (VCCL_ALLOW_SHARED_DEVICE, tests/_mp.py)
    ndev = max(1, torch.cuda.device_count())
    dev = rank % ndev
    if world > ndev:
        os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"
    else:
        os.environ.pop("VCCL_ALLOW_SHARED_DEVICE", None)
    torch.cuda.set_device(dev)
    # lazy communicator init: sub-groups get their own ncclCommInitRankConfig;
    # eager (device_id=): torch splits the default communicator (ncclCommSplit)
    if os.environ.get("VCCL_TEST_TORCH_INIT", "lazy") == "eager":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group("nccl", rank=rank, world_size=world)
    bad = []
    # integer-valued inputs: exact in any fold order
    for n in (3, 4096, 1 << 20, 3 << 20):
        x = torch.arange(n, device="cuda", dtype=torch.float32) % 97 + rank
        want = (torch.arange(n, device="cuda", dtype=torch.float32) % 97) * world + world * (world - 1) / 2
        dist.all_reduce(x)
        if not torch.equal(x, want):
            bad.append(("all_reduce", n))
    y = torch.full((1000,), float(4 * (rank + 1)), device="cuda", dtype=torch.bfloat16)
    dist.all_reduce(y, op=dist.ReduceOp.AVG)
    if not torch.equal(y, torch.full_like(y, 2.0 * (world + 1))):
        bad.append(("avg", 1000))
    z = torch.full((777,), rank, device="cuda", dtype=torch.int32)
    dist.all_reduce(z, op=dist.ReduceOp.MAX)
    if not torch.equal(z, torch.full_like(z, world - 1)):
        bad.append(("max", 777))
    blk = 1 << 16
    src = torch.arange(blk * world, device="cuda", dtype=torch.float32) % 13 + rank
    out = torch.empty(blk, device="cuda")
    dist.reduce_scatter_tensor(out, src)
    ref = (torch.arange(blk * world, device="cuda", dtype=torch.float32) % 13)[rank * blk:(rank + 1) * blk]
    if not torch.equal(out, ref * world + world * (world - 1) / 2):
        bad.append(("reduce_scatter", blk))
    part = torch.full((blk,), float(rank), device="cuda")
    full = torch.empty(blk * world, device="cuda")
    dist.all_gather_into_tensor(full, part)
    if not torch.equal(full, torch.arange(world, device="cuda", dtype=torch.float32).repeat_interleave(blk)):
        bad.append(("all_gather", blk))
    # broadcast (ncclBroadcast) and DDP: construction broadcasts rank 0's
    # module state, backward all-reduces the gradient buckets (the path this
    # library is built for); grads of sum(model(x_r)) with x_r = r + 1 average
    # to exact values
    b = torch.full((1234,), float(rank * 10 + 1), device="cuda")
    dist.broadcast(b, src=world - 1)
    if not torch.equal(b, torch.full_like(b, float((world - 1) * 10 + 1))):
        bad.append(("broadcast", 1234))
    # reduce (ncclReduce) to the last rank: only the destination changes
    rd = torch.arange(4099, device="cuda", dtype=torch.float32) % 31 + rank
    dist.reduce(rd, dst=world - 1)
    base = torch.arange(4099, device="cuda", dtype=torch.float32) % 31
    if not torch.equal(rd, base * world + world * (world - 1) / 2 if rank == world - 1 else base + rank):
        bad.append(("reduce", 4099))
    # uneven lists: torch runs these as grouped ncclBroadcast / ncclReduce
    sizes = [1000 + 37 * r for r in range(world)]
    mine = torch.full((sizes[rank],), float(rank + 1), device="cuda")
    outs = [torch.empty(sz, device="cuda") for sz in sizes]
    dist.all_gather(outs, mine)
    if not all(torch.equal(o, torch.full_like(o, float(r + 1))) for r, o in enumerate(outs)):
        bad.append(("all_gather uneven", sizes))
    ins = [torch.full((sz,), float(rank + r), device="cuda") for r, sz in enumerate(sizes)]
    got = torch.empty(sizes[rank], device="cuda")
    dist.reduce_scatter(got, ins)
    if not torch.equal(got, torch.full_like(got, float(world * rank + world * (world - 1) / 2))):
        bad.append(("reduce_scatter uneven", sizes))
    torch.manual_seed(rank)
    model = torch.nn.Linear(64, 32).cuda()
    torch.manual_seed(0)
    ref = torch.nn.Linear(64, 32).cuda()  # rank 0's initial state
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0])
    if not (torch.equal(ddp.module.weight, ref.weight) and torch.equal(ddp.module.bias, ref.bias)):
        bad.append(("ddp broadcast", 0))
    ddp(torch.full((8, 64), float(rank + 1), device="cuda")).sum().backward()
    gw = torch.full((32, 64), 8.0 * (world + 1) / 2, device="cuda")
    if not (torch.equal(ddp.module.weight.grad, gw) and torch.equal(ddp.module.bias.grad, torch.full((32,), 8.0, device="cuda"))):
        bad.append(("ddp grads", 0))
    # a sub-group (its own communicator; reversed rank order inside it)
    sub = dist.new_group(list(range(world))[::-1])
    w = torch.full((4099,), float(rank + 1), device="cuda")
    dist.all_reduce(w, group=sub)
    if not torch.equal(w, torch.full_like(w, world * (world + 1) / 2)):
        bad.append(("sub_group", 4099))
    torch.cuda.synchronize()
    dist.destroy_process_group()
    if bad:
        print(f"rank {rank}: wrong {bad}", flush=True)
        sys.exit(1)
    print(f"rank {rank}: ok", flush=True)


if __name__ == "__main__":
    main()
