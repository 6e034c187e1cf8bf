#!/usr/bin/env python3
"""Protocol A/B on one GPU: single-process n ranks, many all-reduces, for each
(VCCL_FENCES, VCCL_POLL_MODE); reports hangs (spin timeouts) and mismatches."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"  # ranks share the one GPU

from vccl_amd import nccl  # noqa: E402

n = int(sys.argv[1])
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
count = 4 << 20
os.environ.update(VCCL_SPIN_TIMEOUT_S="4", VCCL_NCHANNELS="14", VCCL_NTHREADS="512",
                  VCCL_SLOT_BYTES=str(256 << 10))
streams = [torch.cuda.Stream() for _ in range(n)]
xs = [torch.randint(-64, 64, (count,), device="cuda").float() for _ in range(n)]
ref = torch.stack(xs).sum(0)
ys = [torch.empty_like(ref) for _ in range(n)]
for fences in (1, 0):
    for poll in (0, 1):
        os.environ.update(VCCL_FENCES=str(fences), VCCL_POLL_MODE=str(poll))
        comms = nccl.Comm.init_all([0] * n)
        bad = hang = 0
        t0 = time.time()
        for it in range(iters):
            nccl.group_start()
            for r, c in enumerate(comms):
                c.all_reduce(xs[r].data_ptr(), ys[r].data_ptr(), count, 7, 0, streams[r].cuda_stream)
            nccl.group_end()
            torch.cuda.synchronize()
            if any(c.async_error() for c in comms):
                hang += 1
                break
            bad += sum(0 if torch.equal(y, ref) else 1 for y in ys)
        for c in comms:
            c.destroy()
        print(json.dumps({"n": n, "fences": fences, "poll": poll, "iters": it + 1, "hang": hang,
                          "mismatch": bad, "s": round(time.time() - t0, 2)}), flush=True)
