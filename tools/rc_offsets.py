#!/usr/bin/env python3
"""Config-2 reduce-copy (2 x 256 MiB f32 -> 256 MiB) vs the relative placement
of its three buffers: HBM channel interleaving can make equal-offset streams
collide.  Places a, b, d inside one pool at chosen byte offsets, times 50
launches per layout (HIP events on the launch stream, after a 0.3 s pre-roll),
repeats the set 3 times interleaved.  Prints one JSON line per layout.
Measurement tool, not product code."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vccl_amd import nccl  # noqa: E402

MB = 1 << 20
N = 64 * MB  # f32 elements per buffer (256 MiB)
LAYOUTS = {
    "contiguous": (0, 256 * MB, 512 * MB),
    "stagger_4K": (0, 256 * MB + 4096, 512 * MB + 8192),
    "stagger_64K": (0, 256 * MB + 64 * 1024, 512 * MB + 128 * 1024),
    "stagger_1M": (0, 257 * MB, 514 * MB),
    "stagger_2M+4K": (0, 258 * MB + 4096, 516 * MB + 8192),
    "gap_64M": (0, 320 * MB, 640 * MB),
}


def main():
    # every layout must fit the pool (checked here, before any launch)
    need = max(max(offs) for offs in LAYOUTS.values()) + N * 4
    pool = torch.empty(need // 4 + 1024, dtype=torch.float32, device="cuda")
    for offs in LAYOUTS.values():
        assert all(o % 4 == 0 and o + N * 4 <= pool.numel() * 4 for o in offs), offs
    base = pool.data_ptr()
    sp = torch.cuda.current_stream().cuda_stream
    pool.uniform_(-1, 1)
    sep = [torch.rand(N, device="cuda") for _ in range(3)]
    res = {k: [] for k in list(LAYOUTS) + ["torch_separate"]}

    def run(ptrs, iters=50):
        def step():
            nccl.reduce_copy(0, 7, 0, ptrs[:2], ptrs[2:], N, sp)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            for _ in range(32):
                step()
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            step()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / iters
        return 3 * N * 4 / t / 1e9

    for _ in range(3):
        for name, offs in LAYOUTS.items():
            res[name].append(run([base + o for o in offs]))
        res["torch_separate"].append(run([t.data_ptr() for t in sep]))
    for name, v in res.items():
        offs = LAYOUTS.get(name)
        ptrs = [hex(base + o) for o in offs] if offs else [hex(t.data_ptr()) for t in sep]
        print(json.dumps({"layout": name, "GBs": [round(x, 1) for x in v],
                          "frac_best": round(max(v) / 8000, 4), "ptrs": ptrs}), flush=True)


if __name__ == "__main__":
    main()
