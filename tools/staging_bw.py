#!/usr/bin/env python3
"""Inter-node staging analogue: the rate of moving a
256 MiB fp32 bucket through host-pinned proxy/NIC-style buffers.

VCCL's net transport stages FIFO slots through host-pinned buffers when GDR is
off (src/transport/net.cc:830-835, proxy thread net.cc:1293-1482).  Measured:
  D2H      device bucket -> pinned host (hipMemcpyAsync)
  H2D      pinned host -> device
  staged   D2H -> host reduce with a "received" peer bucket (oracle C code,
           16 threads) -> H2D, end to end
Writes gpurun_out/staging.json.  Test/measurement tool, not product code.
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    n = 1 << 26
    nbytes = n * 4
    dev = torch.rand(n, device="cuda")
    out = torch.empty_like(dev)
    host = torch.empty(n, dtype=torch.float32, pin_memory=True)
    peer = torch.rand(n, dtype=torch.float32).pin_memory()  # the bucket "from the network"
    red = torch.empty(n, dtype=torch.float32, pin_memory=True)
    threads = min(16, os.cpu_count() or 1)
    t_d2h = timed(lambda: host.copy_(dev, non_blocking=True))
    t_h2d = timed(lambda: out.copy_(host, non_blocking=True))
    hn, pn, rn = host.numpy(), peer.numpy(), red.numpy()

    def staged():
        host.copy_(dev, non_blocking=True)
        torch.cuda.synchronize()
        O.reduce_copy(0, 7, 0, [hn, pn], out=[rn], nthreads=threads)
        out.copy_(red, non_blocking=True)

    t_st = timed(staged, reps=3)
    assert torch.equal(out.cpu(), dev.cpu() + peer), "staged reduce mismatch"
    res = {"bucket_bytes": nbytes, "d2h_GBs": round(nbytes / t_d2h / 1e9, 2),
           "h2d_GBs": round(nbytes / t_h2d / 1e9, 2),
           "staged_reduce_GBs": round(nbytes / t_st / 1e9, 2), "host_threads": threads,
           "note": "staged = D2H + host 2-src f32 sum (oracle C, pthreads) + H2D, end to end"}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "staging.json"), "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
