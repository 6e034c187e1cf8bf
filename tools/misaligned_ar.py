#!/usr/bin/env python3
"""All-reduce on 16-byte-aligned vs misaligned user buffers (send +4 B, recv
+12 B), 2 ranks sharing the one GPU (rehearsal: "xGMI" is local HBM), per
algorithm.  busbw = S/t * 2(n-1)/n.  JSON line per (algo, size, alignment)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"
import torch  # noqa: E402

from vccl_amd import nccl  # noqa: E402

n = 2
comms = nccl.Comm.init_all([0] * n)
streams = [torch.cuda.Stream() for _ in range(n)]
for algo in ("direct", "ring"):
    for c in comms:
        c.set_algo(algo)
    for S in (4 << 20, 64 << 20):
        cnt = S // 4
        for so, ro in ((0, 0), (4, 12)):
            xs = [torch.rand(cnt + 4, device="cuda") for _ in range(n)]
            ys = [torch.zeros(cnt + 4, device="cuda") for _ in range(n)]
            torch.cuda.synchronize()

            def run():
                nccl.group_start()
                for r, c in enumerate(comms):
                    c.all_reduce(xs[r].data_ptr() + so, ys[r].data_ptr() + ro, cnt, nccl.ncclFloat32,
                                 nccl.ncclSum, streams[r].cuda_stream)
                nccl.group_end()

            for _ in range(3):
                run()
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
            iters = 10
            for r in range(n):
                ev[r][0].record(streams[r])
            for _ in range(iters):
                run()
            for r in range(n):
                ev[r][1].record(streams[r])
            torch.cuda.synchronize()
            t = max(a.elapsed_time(b) for a, b in ev) / 1e3 / iters
            exp = xs[0][so // 4:so // 4 + cnt] + xs[1][so // 4:so // 4 + cnt]
            got = ys[0].view(torch.uint8)[ro:ro + S].view(torch.float32)
            print(json.dumps({"algo": algo, "bytes": S, "send_off": so, "recv_off": ro,
                              "us": round(t * 1e6, 1), "busbw_GBs": round(S / t * 2 * (n - 1) / n / 1e9, 1),
                              "max_err": float((got - exp).abs().max()),
                              "async_error": comms[0].async_error()}), flush=True)
for c in comms:
    c.destroy()
