#!/usr/bin/env python3
"""One rank of the ring hand-off switch test (tests/test_gpu_collectives.py).

argv: rank nranks uid_hex outdir
The SIMPLE ring forced (vcclCommSetAlgo) for a set of calls — f32 sum
all-reduce (ragged), f16 sum all-reduce in place, bf16 sum reduce-scatter,
byte all-gather, broadcast, and an f32 prod all-reduce (no per-wave kernel:
it keeps the workgroup hand-off) — run three times on ONE comm with the
slot hand-off switched between calls (vcclCommSetRingWave: workgroup, per
wave, workgroup).  Both hand-offs share the FIFOs, step counters, partition
and fold, so every output must be bitwise equal across the three passes,
and the per-wave launch count must grow by exactly the eligible calls of
the per-wave pass.  Writes outdir/rank<r>.json; exit 0 when the checks pass."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402

F32, F16, BF16, U8 = nccl.ncclFloat32, nccl.ncclFloat16, nccl.ncclBfloat16, nccl.ncclUint8
SUM, PROD = nccl.ncclSum, nccl.ncclProd
# (name, collective, dtype, op, count per rank, eligible for the per-wave kernel)
CALLS = [("ar_f32_sum", "ar", F32, SUM, 3 * (1 << 18) + 5, True),
         ("ar_f16_sum_inplace", "ar_inplace", F16, SUM, 1 << 20, True),
         ("rs_bf16_sum", "rs", BF16, SUM, 300001, True),
         ("ag_u8", "ag", U8, SUM, 1000003, True),
         ("bcast_u8", "bcast", U8, SUM, 777777, True),
         ("ar_f32_prod", "ar", F32, PROD, 1 << 18, False)]
TDT = {F32: torch.float32, F16: torch.float16, BF16: torch.bfloat16, U8: torch.uint8}


def run_pass(comm, rank, n, sp):
    outs = {}
    for k, (name, coll, dt, op, count, _) in enumerate(CALLS):
        g = torch.Generator(device="cuda").manual_seed(1000 * k + rank)
        nin = count * n if coll == "rs" else count
        if dt == U8:
            x = torch.randint(0, 256, (nin,), dtype=torch.uint8, device="cuda", generator=g)
        else:
            x = (torch.rand(nin, device="cuda", generator=g) * 2 - 1).to(TDT[dt])
        y = torch.empty(count * n if coll == "ag" else count, dtype=TDT[dt], device="cuda")
        if coll == "ar":
            comm.all_reduce(x.data_ptr(), y.data_ptr(), count, dt, op, sp)
        elif coll == "ar_inplace":
            comm.all_reduce(x.data_ptr(), x.data_ptr(), count, dt, op, sp)
            y = x
        elif coll == "rs":
            comm.reduce_scatter(x.data_ptr(), y.data_ptr(), count, dt, op, sp)
        elif coll == "ag":
            comm.all_gather(x.data_ptr(), y.data_ptr(), count, dt, sp)
        else:
            comm.broadcast(x.data_ptr(), y.data_ptr(), count, dt, 0, sp)
        torch.cuda.synchronize()
        outs[name] = y.view(torch.uint8).clone()
    return outs


def main():
    rank, n = int(sys.argv[1]), int(sys.argv[2])
    uid = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[3]))
    outdir = sys.argv[4]
    _mp.bind(rank, n)
    comm = nccl.Comm.init_rank(n, uid, rank)
    sp = torch.cuda.current_stream().cuda_stream
    comm.set_algo("ring")
    passes, counts = [], []
    for wave in (False, True, False):
        before = comm.set_ring_wave(wave)
        passes.append(run_pass(comm, rank, n, sp))
        counts.append(comm.set_ring_wave(None) - before)
    comm.set_ring_wave(False)
    comm.set_algo(None)
    res = {"rank": rank, "wave_launches_per_pass": counts,
           "eligible": sum(1 for c in CALLS if c[5]),
           "equal": {name: bool(torch.equal(passes[0][name], passes[1][name]) and
                                torch.equal(passes[0][name], passes[2][name])) for name, *_ in CALLS},
           "async_error": comm.async_error()}
    comm.destroy()
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    ok = all(res["equal"].values()) and counts == [0, res["eligible"], 0] and res["async_error"] == 0
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
