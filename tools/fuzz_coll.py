#!/usr/bin/env python3
"""Randomised transport soak of the collective paths (stress tool, not
product code).  Run under torch.distributed.run (ranks may share one GPU).

Every rank draws the same sequence from FUZZ_SEED: the collective (all-reduce,
reduce-scatter, all-gather, broadcast, reduce), the element type (every
ncclDataType_t torch can hold: int8, uint8, int32, int64, f16, f32, f64, bf16,
fp8 e4m3 / e5m2), the reduction (sum, prod for the integer types, max, min;
max / min only for fp8), the count (log-uniform up to FUZZ_MAX_BYTES, ragged),
in place or not, the root, the path (automatic, or forced ring, direct, LL,
LL128 ring through vcclCommSetAlgo) and runs of 1-4 calls inside one
ncclGroupStart/End.  Inputs are bench.py's small-integer pattern; the expected
output is folded on the device from every rank's pattern in a wide type and
narrowed once, which is exact for every (type, op) drawn here (sums of at
most 8 values in [-16, 15] are exact in f16 / bf16, integer sums and
products wrap the way the kernels' two's-complement arithmetic does), so the
comparison is bit for bit: a lost, stale, duplicated or misplaced byte on any
path shows.  Rank 0 prints a progress line per FUZZ_REPORT iterations and a
summary; every rank that sees a mismatch prints the group and the per-call
verdicts, and all ranks exit 1."""
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from vccl_amd import nccl  # noqa: E402

# name -> (torch dtype, ncclDataType_t, reductions drawn)
TYPES = {
    "i8": (torch.int8, nccl.ncclInt8, ("sum", "prod", "max", "min")),
    "u8": (torch.uint8, nccl.ncclUint8, ("sum", "prod", "max", "min")),
    "i32": (torch.int32, nccl.ncclInt32, ("sum", "prod", "max", "min")),
    "i64": (torch.int64, nccl.ncclInt64, ("sum", "prod", "max", "min")),
    "f16": (torch.float16, nccl.ncclFloat16, ("sum", "sum", "max", "min")),
    "f32": (torch.float32, nccl.ncclFloat32, ("sum", "sum", "max", "min")),
    "f64": (torch.float64, nccl.ncclFloat64, ("sum", "sum", "max", "min")),
    "bf16": (torch.bfloat16, nccl.ncclBfloat16, ("sum", "sum", "max", "min")),
    "e4m3": (torch.float8_e4m3fn, nccl.ncclFloat8e4m3, ("max", "min")),
    "e5m2": (torch.float8_e5m2, nccl.ncclFloat8e5m2, ("max", "min")),
}
TYPE_P = np.array([1, 1, 1, 1, 3, 4, 1, 3, 1, 1], dtype=float)
OPS = {"sum": nccl.ncclSum, "prod": nccl.ncclProd, "max": nccl.ncclMax, "min": nccl.ncclMin}
ALGOS = (None, None, "ring", "direct", "ll", "ll128")


def draw(rng, world, max_bytes):
    coll = str(rng.choice(["ar", "rs", "ag", "bcast", "reduce"], p=[0.35, 0.2, 0.2, 0.125, 0.125]))
    dt = str(rng.choice(list(TYPES), p=TYPE_P / TYPE_P.sum()))
    op = str(rng.choice(TYPES[dt][2]))
    esz = torch.tensor([], dtype=TYPES[dt][0]).element_size()
    nbytes = int(np.exp(rng.uniform(np.log(8), np.log(max_bytes))))
    count = max(1, nbytes // esz + int(rng.integers(0, 7)))  # ragged
    return {"coll": coll, "dt": dt, "op": op, "count": count, "inplace": bool(rng.random() < 0.3),
            "algo": ALGOS[int(rng.integers(0, len(ALGOS)))], "root": int(rng.integers(0, world))}


def mine(n, r, world, dt, base):
    """Rank r's input for global indices [base, base + n) in type dt."""
    t = torch.empty(n, dtype=torch.int64, device="cuda")
    bench.pattern_fill(t, r, world, base)
    tdt = TYPES[dt][0]
    return t.to(tdt) if not tdt.is_floating_point else t.to(torch.float32).to(tdt)


def _wide(x):
    return x.to(torch.float64) if x.dtype.is_floating_point else x.to(torch.int64)


def expected(n, world, dt, op, base):
    acc = _wide(mine(n, 0, world, dt, base))
    for r in range(1, world):
        v = _wide(mine(n, r, world, dt, base))
        acc = {"sum": torch.add, "prod": torch.mul, "max": torch.maximum, "min": torch.minimum}[op](acc, v)
    tdt = TYPES[dt][0]
    return acc.to(tdt) if not tdt.is_floating_point else acc.to(torch.float32).to(tdt)


def same(a, b):
    # bitwise: fp8 has no torch.equal kernel, and -0 / +0 must not pass for each other
    return bool(torch.equal(a.view(torch.uint8), b.view(torch.uint8)))


def run_call(comm, c, rank, world, sp, base):
    """Issue call c; returns (check closure, buffers).  Every buffer must stay
    alive until the call has run: inside a group that is after ncclGroupEnd,
    so the caller holds them (a freed send buffer would be handed to the next
    call's fill by the caching allocator before the collective reads it)."""
    tdt, code, op, n = TYPES[c["dt"]][0], TYPES[c["dt"]][1], OPS[c["op"]], c["count"]
    dt = c["dt"]

    def blank(m):
        return torch.full((m * tdt.itemsize,), 0x5A, dtype=torch.uint8, device="cuda").view(tdt)

    if c["coll"] == "ar":
        x = mine(n, rank, world, dt, base)
        y = x if c["inplace"] else blank(n)
        comm.all_reduce(x.data_ptr(), y.data_ptr(), n, code, op, sp)
        return (lambda: same(y, expected(n, world, dt, c["op"], base))), (x, y)
    if c["coll"] == "rs":
        x = mine(n * world, rank, world, dt, base)
        y = x[rank * n:(rank + 1) * n] if c["inplace"] else blank(n)
        comm.reduce_scatter(x.data_ptr(), y.data_ptr(), n, code, op, sp)
        return (lambda: same(y, expected(n, world, dt, c["op"], base + rank * n))), (x, y)
    if c["coll"] == "ag":
        out = blank(n * world)
        if c["inplace"]:
            src = out[rank * n:(rank + 1) * n]
            src.copy_(mine(n, rank, world, dt, base))
        else:
            src = mine(n, rank, world, dt, base)
        comm.all_gather(src.data_ptr(), out.data_ptr(), n, code, sp)
        return (lambda: all(same(out[r * n:(r + 1) * n], mine(n, r, world, dt, base))
                            for r in range(world))), (src, out)
    root = c["root"]
    x = mine(n, rank, world, dt, base)
    y = x if c["inplace"] else blank(n)
    if c["coll"] == "bcast":
        comm.broadcast(x.data_ptr(), y.data_ptr(), n, code, root, sp)
        return (lambda: same(y, mine(n, root, world, dt, base))), (x, y)
    comm.reduce(x.data_ptr(), y.data_ptr(), n, code, op, root, sp)
    return (lambda: rank != root or same(y, expected(n, world, dt, c["op"], base))), (x, y)


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    if world > torch.cuda.device_count():
        os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"
    os.environ.setdefault("VCCL_LL128_ALLOC", "1")
    dist.init_process_group("gloo")
    obj = [nccl.unique_id_to_bytes(nccl.get_unique_id()) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    comm = nccl.Comm.init_rank(world, nccl.unique_id_from_bytes(obj[0]), rank)
    sp = torch.cuda.current_stream().cuda_stream
    seed = int(os.environ.get("FUZZ_SEED", 1))
    iters = int(os.environ.get("FUZZ_ITERS", 200))
    max_bytes = int(os.environ.get("FUZZ_MAX_BYTES", 32 << 20))
    report = int(os.environ.get("FUZZ_REPORT", 200))
    budget_s = float(os.environ.get("FUZZ_SECONDS", 1e9))
    rng = np.random.default_rng(seed)
    t0 = time.monotonic()
    stats = {"calls": 0, "groups": 0, "bytes": 0, "by_path": {}, "by_type": {}, "by_op": {}}
    done = 0
    for it in range(iters):
        k = int(rng.choice([1, 1, 1, 2, 3, 4]))
        calls = [draw(rng, world, max_bytes) for _ in range(k)]
        # one forced path per group (the forced path is read per call at enqueue)
        comm.set_algo(calls[0]["algo"])
        checks, held = [], []
        try:
            if k > 1:
                nccl.group_start()
            for j, c in enumerate(calls):
                ch, bufs = run_call(comm, c, rank, world, sp, base=((it * 4 + j) % 512) << 20)
                checks.append(ch)
                held.append(bufs)
            if k > 1:
                nccl.group_end()
        finally:
            comm.set_algo(None)
        torch.cuda.synchronize()
        per_call = [bool(ch()) for ch in checks]
        aerr = comm.async_error()
        ok = all(per_call) and aerr == 0
        del held
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        stats["calls"] += k
        stats["groups"] += k > 1
        for c in calls:
            path = f"{c['coll']}:{calls[0]['algo'] or 'auto'}"
            stats["by_path"][path] = stats["by_path"].get(path, 0) + 1
            stats["by_type"][c["dt"]] = stats["by_type"].get(c["dt"], 0) + 1
            stats["by_op"][c["op"]] = stats["by_op"].get(c["op"], 0) + 1
            stats["bytes"] += c["count"] * TYPES[c["dt"]][0].itemsize
        done = it + 1
        if not t.item():
            if not ok:
                print(json.dumps({"mismatch_at": it, "rank": rank, "calls": calls, "call_ok": per_call,
                                  "async_error": aerr, "world": world, "seed": seed}), flush=True)
            comm.destroy()
            dist.destroy_process_group()
            sys.exit(1)
        if rank == 0 and done % report == 0:
            print(json.dumps({"iter": done, "calls": stats["calls"], "s": round(time.monotonic() - t0, 1)}),
                  flush=True)
        stop = torch.tensor([1 if time.monotonic() - t0 > budget_s else 0], dtype=torch.int32)
        dist.all_reduce(stop, op=dist.ReduceOp.MAX)
        if stop.item():
            break
    stats["net_stats"] = list(comm.net_stats())
    comm.destroy()
    if rank == 0:
        print(json.dumps({"summary": True, "world": world, "seed": seed, "iters": done, **stats,
                          "s": round(time.monotonic() - t0, 1), "all_exact": True}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
