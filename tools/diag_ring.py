#!/usr/bin/env python3
"""Step-by-step diagnostic of the multi-rank path on one GPU (progress to stdout)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"  # ranks share the one GPU

from vccl_amd import nccl  # noqa: E402

def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
log("init_all", n)
comms = nccl.Comm.init_all([0] * n)
log("init done", [c.rank for c in comms])
streams = [torch.cuda.Stream() for _ in range(n)]
for count in (4, 4096, 1 << 20):
    xs = [torch.full((count,), float(r + 1), device="cuda") for r in range(n)]
    ys = [torch.zeros(count, device="cuda") for _ in range(n)]
    torch.cuda.synchronize()
    log("launch AR count", count)
    nccl.group_start()
    for r, c in enumerate(comms):
        c.all_reduce(xs[r].data_ptr(), ys[r].data_ptr(), count, nccl.ncclFloat32, nccl.ncclSum,
                     streams[r].cuda_stream)
    nccl.group_end()
    log("launched; syncing")
    for r in range(n):
        streams[r].synchronize()
        log("stream", r, "done; err", comms[r].async_error(), "y[:4]", ys[r][:4].tolist(),
            "expect", n * (n + 1) / 2)
for c in comms:
    c.destroy()
log("destroyed")
