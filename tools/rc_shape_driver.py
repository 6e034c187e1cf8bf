#!/usr/bin/env python3
"""Launch driver for PMC passes over reduce-copy shapes (run under rocprofv3
by tools/pmc_shapes.py; never profiles itself).

argv: [shape ...] with shape in 2to2 (2 x 256 MiB f32 -> 2 x 256 MiB, library
default), 2to2_o3 / 2to2_plain1 (sweep variants), copy (1 -> 1), 2to1 (config 2).
Each shape: 3 warm-up + 10 launches, checked once.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vccl_amd import nccl  # noqa: E402

N = 1 << 26
HUNK2 = 256 * 2 * 16
SHAPES = {
    "2to2": (2, 2, None),
    "2to2_o3": (2, 2, {"blockSize": 256, "unroll": 2, "gridBlocks": N * 4 // HUNK2, "ntLoads": 1,
                       "ntStores": 16 | 2 | 2 << 2, "order": 3}),
    "2to2_plain1": (2, 2, {"blockSize": 256, "unroll": 2, "gridBlocks": N * 4 // HUNK2, "ntLoads": 1,
                           "ntStores": 16 | 2 | 0 << 2, "order": 0}),
    "copy": (1, 1, None),
    "2to1": (2, 1, None),
}


def main():
    a = torch.rand(N, device="cuda") * 2 - 1
    b = torch.rand(N, device="cuda") * 2 - 1
    d0, d1 = torch.empty_like(a), torch.empty_like(a)
    sp = torch.cuda.current_stream().cuda_stream
    for shape in sys.argv[1:] or ["2to2"]:
        ns, nd, cfg = SHAPES[shape]
        srcs = [a.data_ptr(), b.data_ptr()][:ns]
        dsts = [d0.data_ptr(), d1.data_ptr()][:nd]
        for _ in range(13):
            nccl.reduce_copy(0, 7, 0, srcs, dsts, N, sp, config=cfg)
        torch.cuda.synchronize()
        want = a + b if ns == 2 else a
        assert torch.equal(d0, want) and (nd == 1 or torch.equal(d1, want)), shape
        print(shape, "ok", flush=True)


if __name__ == "__main__":
    main()
