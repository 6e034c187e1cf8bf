#!/usr/bin/env python3
"""bench.py's per-dtype leg (bench_rc_dtypes) three times in one process,
each followed by the same E5M2 kernel on buffers made the way
tools/rc_data.py makes them, to locate a measurement-only effect on the
E5M2 row.  Measurement tool."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from vccl_amd import nccl  # noqa: E402


def e5m2_rate(a, b, d, n, K=20):
    s = torch.cuda.current_stream()
    for _ in range(3):
        nccl.reduce_copy(0, nccl.ncclFloat8e5m2, 0, [a.data_ptr(), b.data_ptr()], [d.data_ptr()], n, s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(K):
        nccl.reduce_copy(0, nccl.ncclFloat8e5m2, 0, [a.data_ptr(), b.data_ptr()], [d.data_ptr()], n, s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    return round(3 * n * K / (e0.elapsed_time(e1) / 1e3) / 1e9, 1)


def main():
    nbytes = 256 << 20
    g = torch.Generator(device="cuda").manual_seed(9)
    for r in range(3):
        rows = {x["dtype"]: x["GB/s"] for x in bench.bench_rc_dtypes(nbytes)}
        a = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g) & 0x77
        b = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g) & 0x77
        d = torch.empty_like(a)
        gen_rate = e5m2_rate(a, b, d, nbytes)
        a2 = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
        b2 = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
        a2 &= 0x77
        b2 &= 0x77
        bench_like = e5m2_rate(a2, b2, d, nbytes)
        same_bufs = e5m2_rate(a2, b2, d, nbytes)
        print(json.dumps({"round": r, "bench_rows": rows, "e5m2_generator_bufs": gen_rate,
                          "e5m2_bench_style_bufs": bench_like, "e5m2_again": same_bufs}), flush=True)
        del a, b, d, a2, b2




def first_use(order=("f8e5m2", "f32", "f8e4m3", "f8e5m2")):
    """A fresh process: each kernel's first 8 event-timed batches of 20
    launches (E5M2 first, then f32, E4M3, E5M2 again): where a first-use
    slowdown sits and how long it lasts."""
    nbytes = 256 << 20
    g = torch.Generator(device="cuda").manual_seed(9)
    a = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g) & 0x77
    b = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g) & 0x77
    d = torch.empty_like(a)
    s = torch.cuda.current_stream()
    codes = {"f8e5m2": (nccl.ncclFloat8e5m2, nbytes), "f32": (nccl.ncclFloat32, nbytes // 4),
             "f8e4m3": (nccl.ncclFloat8e4m3, nbytes), "u8": (nccl.ncclUint8, nbytes),
             "bf16": (nccl.ncclBfloat16, nbytes // 2)}
    seen = set()
    for name in order:
        dt, n = codes[name]
        if name in seen:
            name += "_again"
        seen.add(name)
        rates = []
        for _ in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                nccl.reduce_copy(0, dt, 0, [a.data_ptr(), b.data_ptr()], [d.data_ptr()], n, s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            rates.append(round(3 * nbytes * 20 / (e0.elapsed_time(e1) / 1e3) / 1e9))
        print(json.dumps({"first_use": name, "batches_of_20_gbs": rates}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "first_use":
        first_use(*(sys.argv[2:3] and [tuple(sys.argv[2].split(","))]))
    else:
        main()
