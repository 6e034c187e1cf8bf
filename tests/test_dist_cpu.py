"""World-size-2 gloo tests of the N>1 host path on CPU (no GPU).

* the communicator rendezvous: rank 0 creates the unique id (its process
  hosts the bootstrap root, as ncclGetUniqueId does), ships it through
  torch.distributed (gloo) exactly as bench.py does, and both ranks run
  all-gather rounds through the library's TCP bootstrap;
* bench.py's max-over-ranks timing reduction.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vccl_amd import nccl
        obj = [nccl.unique_id_to_bytes(nccl.get_unique_id()) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = nccl.unique_id_from_bytes(obj[0])
        mine = bytes([rank + 1]) * 100 + rank.to_bytes(4, "little")
        got = nccl.bootstrap_allgather(uid, rank, world, mine)
        ok = all(got[r] == bytes([r + 1]) * 100 + r.to_bytes(4, "little") for r in range(world))
        t = torch.tensor([0.5 + rank], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py _time_coll reduction
        ok &= t.item() == 0.5 + world - 1
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_rendezvous(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = dict(q.get(timeout=5) for _ in range(world))
    assert all(p.exitcode == 0 for p in procs)
    assert res == {r: True for r in range(world)}
