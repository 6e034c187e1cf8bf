#!/usr/bin/env python3
"""The two-destination reduce-copy (2 x n f32 -> 2 x n: the ring step that
writes the next rank's FIFO slot beside the own output) timed the way
bench.py times config 2: K back-to-back launches through the C ABI between
one HIP-event pair on the launch stream, after W warmup launches, so the
figure compares directly with the N = 1 line (per-launch event pairs, as in
tools/sweep_rc.py, add ~1.5 us of event overhead per launch).  Blocks of the
2 -> 2 and 2 -> 1 (config 2) shapes alternate, ROUNDS times; prints one JSON
line with the median average launch time and GB/s of each, and the fraction
of the 8 TB/s HBM peak.  Outputs are checked bit-exactly.
Measurement tool, not product code."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vccl_amd import nccl  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    n = 1 << 26  # 256 MiB per buffer (BASELINE config 2)
    steps, warmup, rounds = 20, 5, int(os.environ.get("ROUNDS", 8))
    g = torch.Generator(device="cuda").manual_seed(1)
    a = torch.rand(n, device="cuda", generator=g) * 2 - 1
    b = torch.rand(n, device="cuda", generator=g) * 2 - 1
    d0, d1 = torch.empty_like(a), torch.empty_like(a)
    ref = a + b
    s = torch.cuda.current_stream()
    shapes = {"2to2": [d0.data_ptr(), d1.data_ptr()], "2to1": [d0.data_ptr()]}
    avg = {k: [] for k in shapes}
    for r in range(rounds):
        for name in (shapes if r % 2 == 0 else reversed(list(shapes))):
            dsts = shapes[name]

            def launch():
                nccl.reduce_copy(0, 7, 0, [a.data_ptr(), b.data_ptr()], dsts, n, s.cuda_stream)
            for _ in range(warmup):
                launch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(steps):
                launch()
            e1.record(s)
            torch.cuda.synchronize()
            avg[name].append(e0.elapsed_time(e1) * 1e3 / steps)
    assert torch.equal(d0, ref) and torch.equal(d1, ref)
    out = {"workload": "f32 sum, 2 x 2^26 elements in, 1 or 2 outputs, device-resident",
           "steps": steps, "warmup": warmup, "rounds": rounds}
    for name, nd in (("2to2", 2), ("2to1", 1)):
        us = float(np.median(avg[name]))
        gbs = (2 + nd) * n * 4 / (us * 1e-6) / 1e9
        out[name] = {"avg_launch_us": round(us, 2), "gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                     "per_round_us": [round(v, 2) for v in avg[name]]}
    out["ratio_2to2_over_2to1"] = round(out["2to2"]["gbs"] / out["2to1"]["gbs"], 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
