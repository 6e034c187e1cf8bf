#!/usr/bin/env python3
"""One rank of a multi-process ring test (spawned by tests/test_gpu_collectives.py).

argv: rank nranks device uid_hex outdir
Runs every case of tests/ring_cases.py through ncclAllReduce /
ncclReduceScatter / ncclAllGather and saves its outputs to outdir/rank<r>.npz.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests import ring_cases as RC  # noqa: E402
from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402


def main():
    rank, nranks = int(sys.argv[1]), int(sys.argv[2])  # argv[3]: device (unused: rank % devices)
    uid = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[4]))
    outdir = sys.argv[5]
    _mp.bind(rank, nranks)
    comm = nccl.Comm.init_rank(nranks, uid, rank)
    if os.environ.get("VCCL_TEST_SET_ALGO"):  # vcclCommSetAlgo for every call
        comm.set_algo(os.environ["VCCL_TEST_SET_ALGO"])
    s = torch.cuda.current_stream().cuda_stream
    res = {}
    for ci, (name, coll, op, dt, count) in enumerate(RC.CASES):
        x = RC.gen_input(ci, rank, nranks)
        xb = torch.from_numpy(x.view(np.uint8).copy()).cuda()
        nout = RC.out_count(ci, nranks)
        yb = torch.empty(nout * x.dtype.itemsize, dtype=torch.uint8, device="cuda")
        if coll == "ar":
            comm.all_reduce(xb.data_ptr(), yb.data_ptr(), count, dt, op, s)
        elif coll == "ar_inplace":
            comm.all_reduce(xb.data_ptr(), xb.data_ptr(), count, dt, op, s)
            yb = xb
        elif coll == "ar_mis":
            so, ro = RC.mis_offsets(dt)
            xm = torch.zeros(xb.numel() + 16, dtype=torch.uint8, device="cuda")
            xm[so:so + xb.numel()] = xb
            ym = torch.zeros(yb.numel() + 16, dtype=torch.uint8, device="cuda")
            comm.all_reduce(xm.data_ptr() + so, ym.data_ptr() + ro, count, dt, op, s)
            yb = ym[ro:ro + yb.numel()]
        elif coll == "rs":
            comm.reduce_scatter(xb.data_ptr(), yb.data_ptr(), count, dt, op, s)
        else:
            comm.all_gather(xb.data_ptr(), yb.data_ptr(), count, dt, s)
        torch.cuda.synchronize()
        res[name] = yb.cpu().numpy().view(x.dtype)
    # one group of GROUP_CASES on two streams (LL runs fused into one launch)
    streams = [torch.cuda.current_stream()]
    if int(os.environ.get("VCCL_TEST_GROUP_STREAMS", "2")) > 1:
        streams.append(torch.cuda.Stream())
    g = RC.run_group([(comm, streams)], [rank], nranks)[0]
    res.update(g)
    # every call's path in the group: its aggregate's (RC.group_algos)
    res["group_algos"] = np.array(RC.group_algos(comm.coll_algo, nranks))
    # ... and as the library reports it (vcclCommGroupAlgos)
    res["lib_group_algos"] = np.array(comm.group_algos([(0, c, dt, op) for _, op, dt, c in RC.GROUP_CASES]))
    before = comm.launch_stats()
    res["launch_stats"] = np.array(before, dtype=np.int64)
    res["net_stats"] = np.array(comm.net_stats(), dtype=np.int64)
    res["wave_launches"] = np.int64(comm.set_ring_wave(None))  # ring launches on the per-wave kernel
    err = comm.async_error()
    comm.destroy()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **res)
    sys.exit(0 if err == 0 else 3)


if __name__ == "__main__":
    main()
