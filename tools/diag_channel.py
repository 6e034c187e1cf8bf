#!/usr/bin/env python3
"""Per-channel bandwidth diagnostic: what one ring channel (one workgroup) can
move, by memory kind of the FIFO operands and by cache policy.

A ring step is a 2-source reduce-copy (own input + received slot) into the
peer's slot.  Here the same 2-src f32 sum runs as a reduce-copy launch with a
fixed number of workgroups, B (the "received slot") and D (the "peer slot")
allocated as ordinary hipMalloc memory, hipDeviceMallocUncached, or
hipDeviceMallocFinegrained.  Prints GB/s per workgroup (3 x bytes / time).
Measurement tool only.
"""
import ctypes
import itertools
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vccl_amd import nccl  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipFree.argtypes = [ctypes.c_void_p]
KINDS = {"hbm": None, "uncached": 0x3, "fine": 0x1}


def alloc(kind, nbytes, keep):
    if KINDS[kind] is None:
        t = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
        keep.append(t)
        return t.data_ptr()
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, KINDS[kind])
    assert rc == 0, (kind, rc)
    keep.append(p)
    return p.value


def main():
    per_wg = int(os.environ.get("DIAG_BYTES_PER_WG", 4 << 20))
    grids = [int(x) for x in os.environ.get("DIAG_GRIDS", "1,8,64").split(",")]
    reps = int(os.environ.get("DIAG_REPS", 20))
    s = torch.cuda.current_stream()
    keep = []
    gmax = max(grids)
    nbytes = per_wg * gmax
    a = torch.rand(nbytes // 4, device="cuda")
    bufs = {}
    for k in KINDS:
        bufs[k] = (alloc(k, nbytes, keep), alloc(k, nbytes, keep))
        torch.cuda.synchronize()
    for kb in KINDS:  # fill B with data via a copy from a
        nccl.reduce_copy(15, 0, 0, [a.data_ptr()], [bufs[kb][0]], nbytes, s.cuda_stream)
    torch.cuda.synchronize()
    for g, bk, dk, ld, st, threads in itertools.product(grids, KINDS, KINDS, (1, 2), (0, 2), (1024,)):
        n = per_wg * g // 4
        cfg = {"blockSize": threads, "unroll": 2, "gridBlocks": g, "ntLoads": ld, "ntStores": st,
               "order": 0}
        srcs = [a.data_ptr(), bufs[bk][0]]
        dsts = [bufs[dk][1]]
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(reps)]
        for e0, e1 in ev:
            e0.record(s)
            nccl.reduce_copy(0, 7, 0, srcs, dsts, n, s.cuda_stream, config=cfg)
            e1.record(s)
        torch.cuda.synchronize()
        t = np.array([e0.elapsed_time(e1) for e0, e1 in ev][2:]) / 1e3
        gbs = 3 * n * 4 / np.median(t) / 1e9
        print(json.dumps({"grid": g, "B": bk, "D": dk, "ld": ld, "st": st, "threads": threads,
                          "GBs": round(gbs, 1), "GBs_per_wg": round(gbs / g, 1),
                          "us": round(float(np.median(t)) * 1e6, 1)}), flush=True)
    for p in keep:
        if isinstance(p, ctypes.c_void_p):
            hip.hipFree(p)


if __name__ == "__main__":
    main()
