#!/usr/bin/env python3
"""Diagnostic: two comms of one process on one GPU (init_all), re-initialised
several times with different channel counts; every round an all-reduce on
two streams.  Mode 'fresh': new torch streams per round; 'reused': one pair;
'raw': streams from hipStreamCreate via torch.cuda.Stream(priority)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/sessions/..
sys.path.insert(0, ROOT)
os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"
os.environ.setdefault("VCCL_SPIN_TIMEOUT_S", "5")
import torch  # noqa: E402

from vccl_amd import nccl  # noqa: E402

mode = sys.argv[1]
n = (3 << 20) + 5
reused = [torch.cuda.Stream() for _ in range(2)]
for it, nch in enumerate([16, 12, 16, 12, 8, 20]):
    os.environ["NCCL_NCHANNELS"] = str(nch)
    comms = nccl.Comm.init_all([0, 0])
    if mode == "sync":
        torch.cuda.synchronize()
    streams = reused if mode in ("reused", "sync") else [torch.cuda.Stream() for _ in range(2)]
    xs = [((torch.arange(n, device="cuda") * (r + 3)) % 101).float() for r in range(2)]
    ys = [torch.empty(n, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    t = time.time()
    nccl.group_start()
    for c, x, y, st in zip(comms, xs, ys, streams):
        c.set_algo("ring")
        c.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum, st.cuda_stream)
    nccl.group_end()
    torch.cuda.synchronize()
    ok = all(torch.equal(y, xs[0] + xs[1]) for y in ys)
    print(f"{mode} it {it} nch {nch} ok {ok} err {[c.async_error() for c in comms]} "
          f"{time.time() - t:.2f}s streams {[hex(s.cuda_stream) for s in streams]}", flush=True)
    for c in comms:
        c.destroy()
