#!/usr/bin/env python3
"""One rank of the full-size BASELINE workload test (tests/test_gpu_workloads.py).

argv: rank nranks uid_hex outdir nch slot nthreads case[,case...]
cases:
  c4 / c4_direct     reduce-scatter then all-gather of a 4 GiB bf16 bucket
                     (BASELINE config 4) on the default path / the direct path
  c3_ring / c3_direct / c3_default
                     all-reduce of 1 GiB fp32 (BASELINE config 3, headline
                     bucket) on the ring / the direct path / the library's choice
Each case runs twice: with the integer pattern (exact in any fold order,
checked here over the whole output) and with hashed fp inputs (the output at
the sampled windows of tests/_workload.py is saved for the test to check
bit-exactly against the oracle's fold in VCCL's ring order).
Exit 0 = every collective ran without a spin timeout (verdicts in the npz).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402  (pattern_fill / pattern_ok: the N>1 line's own checker)
from tests import _workload as W  # noqa: E402
from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402

C4_BYTES = 4 << 30
C3_BYTES = 1 << 30


def _to_np(t, dt):
    t = t.cpu()
    return t.view(torch.int16).numpy().view(np.uint16) if dt == 9 else t.numpy().copy()


def run_c4(comm, rank, n, algo, geo, res, tag):
    dt, tdt = 9, torch.bfloat16
    total = C4_BYTES // 2
    rc = total // n
    s = torch.cuda.current_stream().cuda_stream
    comm.set_algo(algo)
    res[f"{tag}_algo_rs"] = comm.coll_algo(1, rc, dt)
    res[f"{tag}_algo_ag"] = comm.coll_algo(2, rc, dt)
    x = torch.empty(total, dtype=tdt, device="cuda")
    shard = torch.empty(rc, dtype=tdt, device="cuda")
    for mode in ("pattern", "hash"):
        if mode == "pattern":
            bench.pattern_fill(x, rank, n)
        else:
            W.device_fill(x, dt, rank)
        shard.fill_(float("nan"))
        torch.cuda.synchronize()
        comm.reduce_scatter(x.data_ptr(), shard.data_ptr(), rc, dt, nccl.ncclSum, s)
        torch.cuda.synchronize()
        x.fill_(float("nan"))  # reused as the all-gather output
        comm.all_gather(shard.data_ptr(), x.data_ptr(), rc, dt, s)
        torch.cuda.synchronize()
        if comm.async_error() != 0:
            return False
        if mode == "pattern":
            res[f"{tag}_pattern_rs"] = bench.pattern_ok(shard, n, base=rank * rc)
            res[f"{tag}_pattern_ag"] = bench.pattern_ok(x, n)
        else:
            win, _ = W.rs_windows(rc, 2, n, *geo)
            wt = torch.from_numpy(win).cuda()
            res[f"{tag}_rs_win"] = _to_np(shard[wt], dt)
            agw = torch.cat([wt + q * rc for q in range(n)])
            res[f"{tag}_ag_win"] = _to_np(x[agw], dt)
    comm.set_algo(None)
    del x, shard
    torch.cuda.empty_cache()
    return True


def run_c3(comm, rank, n, algo, geo, res, tag):
    dt, tdt = 7, torch.float32
    count = C3_BYTES // 4
    s = torch.cuda.current_stream().cuda_stream
    comm.set_algo(algo)
    res[f"{tag}_algo"] = comm.coll_algo(0, count, dt)
    x = torch.empty(count, dtype=tdt, device="cuda")
    y = torch.empty(count, dtype=tdt, device="cuda")
    for mode in ("pattern", "hash"):
        if mode == "pattern":
            bench.pattern_fill(x, rank, n)
        else:
            W.device_fill(x, dt, rank)
        y.fill_(float("nan"))
        torch.cuda.synchronize()
        comm.all_reduce(x.data_ptr(), y.data_ptr(), count, dt, nccl.ncclSum, s)
        torch.cuda.synchronize()
        if comm.async_error() != 0:
            return False
        if mode == "pattern":
            res[f"{tag}_pattern"] = bench.pattern_ok(y, n)
        else:
            win, _ = W.ar_windows(count, 4, n, *geo)
            res[f"{tag}_win"] = _to_np(y[torch.from_numpy(win).cuda()], dt)
    comm.set_algo(None)
    del x, y
    torch.cuda.empty_cache()
    return True


def main():
    rank, n = int(sys.argv[1]), int(sys.argv[2])
    uid = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[3]))
    outdir = sys.argv[4]
    geo = (int(sys.argv[5]), int(sys.argv[6]), int(sys.argv[7]))  # nch, slot, nthreads
    cases = sys.argv[8].split(",")
    _mp.bind(rank, n)
    comm = nccl.Comm.init_rank(n, uid, rank)
    res = {}
    ok = True
    for case in cases:
        algo = {"c4": None, "c4_direct": "direct", "c3_ring": "ring", "c3_direct": "direct",
                "c3_default": None}[case]
        fn = run_c4 if case.startswith("c4") else run_c3
        ok = fn(comm, rank, n, algo, geo, res, case)
        print(f"rank {rank} {case}: {'ran' if ok else 'ASYNC ERROR'}", flush=True)
        if not ok:
            break
    comm.destroy()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **{k: np.asarray(v) for k, v in res.items()})
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
