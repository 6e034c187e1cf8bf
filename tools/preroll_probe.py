"""How the config-2 reduce-copy rate depends on what precedes the timed
region (bench.py N=1): idle gap, pre-roll length, sustained load.

For each pre-roll length (after a fixed idle gap) the 20-launch timed region
of bench.py is repeated; then one long back-to-back run is cut into windows
of 50 launches to show the sustained rate over time.  Prints JSON lines.
"""
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vccl_amd import nccl  # noqa: E402


def main():
    n = (256 << 20) // 4
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    a = torch.rand(n, device="cuda") * 2 - 1
    b = torch.rand(n, device="cuda") * 2 - 1
    d = torch.empty_like(a)
    L = nccl.lib()
    srcs = (ctypes.c_void_p * 2)(a.data_ptr(), b.data_ptr())
    dsts = (ctypes.c_void_p * 1)(d.data_ptr())

    def step():
        assert L.vcclReduceCopy(0, nccl.ncclFloat32, 0, 0, 0, 2, srcs, 1, dsts, n, sp) == 0

    def timed(k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(k):
            step()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / k

    bytes_per = 3 * n * 4
    for rnd in range(2):
        for pre_s in (0.0, 0.02, 0.1, 0.5, 2.0):
            time.sleep(2.0)
            t0 = time.perf_counter()
            npre = 0
            while time.perf_counter() - t0 < pre_s:
                for _ in range(16):
                    step()
                torch.cuda.synchronize()
                npre += 16
            for _ in range(5):
                step()
            torch.cuda.synchronize()
            us = timed(20)
            print(json.dumps({"round": rnd, "idle_s": 2.0, "preroll_s": pre_s, "preroll_launches": npre,
                              "us": round(us, 2), "frac": round(bytes_per / us / 1e3 / 8000, 4)}),
                  flush=True)
    time.sleep(2.0)
    rows = []
    for w in range(60):  # ~0.33 s of sustained load
        us = timed(50)
        rows.append(round(us, 2))
    print(json.dumps({"sustained_window_us": rows}), flush=True)


if __name__ == "__main__":
    main()
