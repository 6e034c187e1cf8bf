#!/usr/bin/env python3
"""One rank of the > 2 GiB collective test (spawned by tests/test_gpu_collectives.py).

argv: rank nranks device uid_hex
Per-rank buffers past 2 GiB for ring all-reduce, direct all-reduce, ring
reduce-scatter and ring all-gather.  Inputs are integer-valued f32 drawn from
a per-rank seeded GPU generator, so every fold order is exact and each rank
regenerates its peers' inputs to compute the expected output with torch.
Exit 0 = every case matched, 4 = mismatch, 3 = async error (spin timeout).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402

BIG = (1 << 29) + 1037  # f32 elements: 2 GiB + 4148 B
CASES = [("ar", "ring"), ("ar", "direct"), ("rs", "ring"), ("ag", "ring")]


def gen(rank, n_elts):
    g = torch.Generator(device="cuda").manual_seed(1000 + rank)
    return torch.randint(-64, 64, (n_elts,), device="cuda", generator=g).float()


def main():
    rank, nranks = int(sys.argv[1]), int(sys.argv[2])  # argv[3]: device (unused: rank % devices)
    uid = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[4]))
    _mp.bind(rank, nranks)
    comm = nccl.Comm.init_rank(nranks, uid, rank)
    s = torch.cuda.current_stream().cuda_stream
    bad = []
    for coll, algo in CASES:
        comm.set_algo(algo)
        ci = {"ar": 0, "rs": 1, "ag": 2}[coll]
        count = BIG if coll == "ar" else BIG // 2
        got_algo = comm.coll_algo(ci, count, 7)
        if got_algo != algo:
            bad.append(f"{coll}: algo {got_algo} != {algo}")
            continue
        insz = count * nranks if coll == "rs" else count
        outsz = count * nranks if coll == "ag" else count
        x = gen(rank, insz)
        y = torch.full((outsz,), float("nan"), device="cuda")
        if coll == "ar":
            comm.all_reduce(x.data_ptr(), y.data_ptr(), count, 7, 0, s)
        elif coll == "rs":
            comm.reduce_scatter(x.data_ptr(), y.data_ptr(), count, 7, 0, s)
        else:
            comm.all_gather(x.data_ptr(), y.data_ptr(), count, 7, s)
        torch.cuda.synchronize()
        if comm.async_error() != 0:
            print(f"rank {rank} {coll}/{algo}: async error", flush=True)
            comm.destroy()
            sys.exit(3)
        del x
        if coll == "ag":
            ref = torch.cat([gen(r, count) for r in range(nranks)])
        else:
            ref = gen(0, insz)
            for r in range(1, nranks):
                ref += gen(r, insz)
            if coll == "rs":
                ref = ref[rank * count:(rank + 1) * count]
        ok = torch.equal(y, ref)
        print(f"rank {rank} {coll}/{algo}: {'ok' if ok else 'MISMATCH'}", flush=True)
        if not ok:
            bad.append(f"{coll}/{algo}")
        del y, ref
        torch.cuda.empty_cache()
    comm.destroy()
    sys.exit(4 if bad else 0)


if __name__ == "__main__":
    main()
