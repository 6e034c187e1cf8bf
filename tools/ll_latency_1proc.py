#!/usr/bin/env python3
"""The config-5 LL all-reduce with every rank in ONE process:
n comms on device 0 from ncclCommInitAll (VCCL_ALLOW_SHARED_DEVICE=1), one
stream each, one host thread issuing each call on every comm in turn — the
same kernels as tools/ll_latency.py's n processes, without cross-process GPU
queue scheduling.  Each size is timed REPS times (back-to-back eager calls,
one synchronize at the end), so a bimodal rate shows.  Prints one JSON line.

    VCCL_ALLOW_SHARED_DEVICE=1 python tools/ll_latency_1proc.py [n]

Measurement tool, not product code."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from vccl_amd import nccl  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    os.environ.setdefault("VCCL_ALLOW_SHARED_DEVICE", "1")
    comms = nccl.Comm.init_all([0] * n)
    torch.cuda.set_device(0)
    streams = [torch.cuda.Stream() for _ in range(n)]
    steps, reps = int(os.environ.get("LAT_STEPS", 200)), int(os.environ.get("LAT_REPS", 5))
    out = {"ranks_in_one_process": n, "rows": []}
    for S in (8, 1024, 4096):
        m = max(1, S // 2)
        xs = [torch.ones(m, dtype=torch.float16, device="cuda") for _ in range(n)]
        ys = [torch.empty_like(x) for x in xs]

        def call():
            for c, s, x, y in zip(comms, streams, xs, ys):
                c.all_reduce(x.data_ptr(), y.data_ptr(), m, nccl.ncclFloat16, nccl.ncclSum, s.cuda_stream)
        for _ in range(20):
            call()
        torch.cuda.synchronize()
        us = []
        for _ in range(reps):
            t0 = time.perf_counter()
            for _ in range(steps):
                call()
            th = time.perf_counter() - t0
            torch.cuda.synchronize()
            us.append((round((time.perf_counter() - t0) / steps * 1e6, 2), round(th / steps * 1e6, 2)))
        ok = all(bool((y == n).all()) for y in ys)
        row = {"bytes": S, "eager_us": [u for u, _ in us], "host_us_all_ranks": [h for _, h in us], "exact": ok,
               "algo": comms[0].coll_algo(0, m, nccl.ncclFloat16)}
        out["rows"].append(row)
        print(f"# {row}", file=sys.stderr, flush=True)
    out["async_error"] = [c.async_error() for c in comms]
    for c in comms:
        c.destroy()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
