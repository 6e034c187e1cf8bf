#!/usr/bin/env python3
"""One rank of the group-plan stress test (tests/test_gpu_collectives.py).

argv: rank nranks uid_hex outdir
One ncclGroupStart/End of STRESS_CALLS — all-reduces, reduce-scatters and
all-gathers of f32 / bf16 / i32 (sum, avg, max) from 1 KiB to 6 MiB, issued on
two streams in turn — so the group plan spans several (func, op, type) bins,
aggregates, and launches of up to 16 parts with channels skipped per part.
Saves every output and the path the library chose for each call
(its aggregate's, vcclCommCollAlgo on the summed count) for the test's
expectation; the group runs twice (outputs
NaN-filled before each) and the second run must equal the first bit for bit.
"""
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from tests import _ring  # noqa: E402
from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402

COLLS = ("ar", "rs", "ag")


def stress_calls(n, k=36, seed=4242):
    """[(name, coll, dtype, op, count)]: count = AR count, RS recvcount, AG
    sendcount (elements)."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(k):
        coll = COLLS[int(rng.integers(0, 3))]
        dt = int(rng.choice([7, 9, 2]))
        u = rng.random()
        op = 2 if dt == 2 and u < 0.4 else 4 if u > 0.7 else 0  # max (i32), avg, sum
        nbytes = int(2 ** rng.uniform(10, np.log2(6 << 20)))
        esz = 2 if dt == 9 else 4
        count = max(1, nbytes // esz)
        if coll in ("rs", "ag"):
            count = max(1, count // n)
        out.append((f"s{i}_{coll}", coll, dt, op, count))
    return out


def group_calls(calls):
    """(coll, op, dtype, count) per call, as _ring.group_works takes them."""
    return [(coll, op, dt, count) for _, coll, dt, op, count in calls]


def gen(name, dt, total, rank):
    rng = np.random.default_rng(zlib.crc32(name.encode()) * 16 + rank)
    if dt == 2:
        return rng.integers(-1000, 1000, total).astype(np.int32)
    x = rng.uniform(-1, 1, total).astype(np.float32)
    return O.f32_to_bf16_bits(x) if dt == 9 else x


def in_count(coll, count, n):
    return count * n if coll == "rs" else count


def out_count(coll, count, n):
    return count * n if coll == "ag" else count


def main():
    rank, n = int(sys.argv[1]), int(sys.argv[2])
    uid = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[3]))
    outdir = sys.argv[4]
    _mp.bind(rank, n)
    comm = nccl.Comm.init_rank(n, uid, rank)
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    calls = stress_calls(n)
    bufs = {}
    for name, coll, dt, op, count in calls:
        x = gen(name, dt, in_count(coll, count, n), rank)
        xb = torch.from_numpy(x.view(np.uint8).copy()).cuda()
        yb = torch.empty(out_count(coll, count, n) * x.dtype.itemsize, dtype=torch.uint8, device="cuda")
        bufs[name] = (xb, yb, x.dtype)
    # every call's path: its aggregate's (ncclPrepareTasks, _ring.group_algos)
    algos = _ring.group_algos(group_calls(calls), n, comm.coll_algo)
    lib_algos = comm.group_algos([(COLLS.index(c), cnt, dt, op) for _, c, dt, op, cnt in calls])
    res = {}
    for rep in range(2):
        for xb, yb, _ in bufs.values():
            yb.fill_(0xFF)
        torch.cuda.synchronize()
        nccl.group_start()
        for i, (name, coll, dt, op, count) in enumerate(calls):
            xb, yb, _ = bufs[name]
            sp = streams[i % 2].cuda_stream
            if coll == "ar":
                comm.all_reduce(xb.data_ptr(), yb.data_ptr(), count, dt, op, sp)
            elif coll == "rs":
                comm.reduce_scatter(xb.data_ptr(), yb.data_ptr(), count, dt, op, sp)
            else:
                comm.all_gather(xb.data_ptr(), yb.data_ptr(), count, dt, sp)
        nccl.group_end()
        torch.cuda.synchronize()
        for name, (xb, yb, npdt) in bufs.items():
            out = yb.cpu().numpy().view(npdt)
            if rep == 0:
                res[name] = out
            elif not np.array_equal(out.view(np.uint8), res[name].view(np.uint8)):
                res[name + "_differs"] = np.array(rep)
    res["algos"] = np.array(algos)
    res["lib_algos"] = np.array(lib_algos)
    err = comm.async_error()
    comm.destroy()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **res)
    sys.exit(0 if err == 0 else 3)


if __name__ == "__main__":
    main()
