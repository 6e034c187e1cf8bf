#!/usr/bin/env python3
"""Does the reduce-copy rate depend on the DATA?  Config 2's byte shape
(2 x 256 MiB -> 256 MiB) for E4M3 / E5M2 / u8 / f32 sum on several input
patterns (zeros, random bytes masked 0x77 as in bench.py's per-dtype leg,
masked 0x33, a byte ramp; for f32 also config 2's own uniform[-1,1)),
interleaved in one process; median GB/s per (dtype, pattern).  Measurement
tool."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vccl_amd import nccl  # noqa: E402


def main():
    nbytes = 256 << 20
    g = torch.Generator(device="cuda").manual_seed(9)
    rnd_a = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)
    rnd_b = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)
    ramp = (torch.arange(nbytes, device="cuda") & 0x77).to(torch.uint8)
    pats = {"zeros": (torch.zeros_like(rnd_a), torch.zeros_like(rnd_b)),
            "rand&77": (rnd_a & 0x77, rnd_b & 0x77),
            "rand&33": (rnd_a & 0x33, rnd_b & 0x33),
            "ramp&77": (ramp, ramp.roll(1))}
    u = torch.rand(nbytes // 4, device="cuda", generator=g) * 2 - 1
    pats["uniform_f32"] = (u.view(torch.uint8), (torch.rand(nbytes // 4, device="cuda", generator=g) * 2 - 1).view(torch.uint8))
    d = torch.empty_like(rnd_a)
    s = torch.cuda.current_stream()
    dts = {"f8e4m3": nccl.ncclFloat8e4m3, "f8e5m2": nccl.ncclFloat8e5m2, "u8": nccl.ncclUint8,
           "f32": nccl.ncclFloat32}
    times = {(k, p): [] for k in dts for p in pats if k == "f32" or p != "uniform_f32"}
    for r in range(6):
        for (k, p) in times:
            a, b = pats[p]
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(8)]
            for e0, e1 in ev:
                e0.record(s)
                nccl.reduce_copy(0, dts[k], 0, [a.data_ptr(), b.data_ptr()], [d.data_ptr()],
                                 nbytes // (4 if k == "f32" else 1), s.cuda_stream)
                e1.record(s)
            torch.cuda.synchronize()
            if r:
                times[(k, p)] += [e0.elapsed_time(e1) for e0, e1 in ev]
    for (k, p), t in times.items():
        t = np.array(t)
        print(json.dumps({"dtype": k, "pattern": p, "median_gbs": round(float(np.median(3 * nbytes / (t / 1e3) / 1e9)), 1),
                          "median_us": round(float(np.median(t)) * 1e3, 2)}), flush=True)
    # Sustained: K launches back to back under ONE event pair (bench.py's
    # per-dtype leg uses K = 20), after 3 warmup launches, 3 repetitions.
    for k in dts:
        a, b = pats["uniform_f32" if k == "f32" else "rand&77"]
        n = nbytes // (4 if k == "f32" else 1)
        for K in (8, 20, 60):
            res = []
            for _ in range(3):
                for _ in range(3):
                    nccl.reduce_copy(0, dts[k], 0, [a.data_ptr(), b.data_ptr()], [d.data_ptr()], n, s.cuda_stream)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(K):
                    nccl.reduce_copy(0, dts[k], 0, [a.data_ptr(), b.data_ptr()], [d.data_ptr()], n, s.cuda_stream)
                e1.record(s)
                torch.cuda.synchronize()
                res.append(round(3 * nbytes * K / (e0.elapsed_time(e1) / 1e3) / 1e9, 1))
            print(json.dumps({"dtype": k, "sustained_launches": K, "gbs": res}), flush=True)


if __name__ == "__main__":
    main()
