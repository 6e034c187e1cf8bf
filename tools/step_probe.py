#!/usr/bin/env python3
"""Per-channel copy rate of the ring primitive's shapes without the protocol
(tools/step_probe.hip): nWG workgroups of 512 threads, each repeating one
shape over its own 512 KiB slot with the per-slot drain + barrier.  Prints
one JSON line per (shape, unroll, output policy, nWG): per-workgroup GB/s
(operand bytes per slot / time per slot) and the aggregate.  Measurement
tool, not product code."""
import ctypes
import itertools
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "vccl_amd", "lib", "libvccl_stepprobe.so"))
vp = ctypes.c_void_p
lib.step_probe_alloc_uncached.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t]
lib.step_probe_free.argtypes = [vp]
lib.step_probe_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp,
                               ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long, vp]
NAMES = ["S->F", "S+F->F2", "S+F->O", "S->F+O", "F->O", "F->F2+O", "S+F->F2+O"]
OPS = [(1, 1), (2, 1), (2, 1), (1, 2), (1, 1), (1, 2), (2, 2)]
SLOT = 512 << 10


def main():
    nwgs = [int(x) for x in os.environ.get("PROBE_NWG", "96").split(",")]
    unrolls = [int(x) for x in os.environ.get("PROBE_UNROLL", "4,8").split(",")]
    reps = int(os.environ.get("PROBE_REPS", "64"))
    span = int(os.environ.get("PROBE_SPAN", str(1 << 30)))  # own input / output streamed
    nmax = max(nwgs)
    S = torch.rand(span // 4, device="cuda")
    O = torch.empty_like(S)
    F, F2 = vp(), vp()
    assert lib.step_probe_alloc_uncached(ctypes.byref(F), nmax * SLOT) == 0
    assert lib.step_probe_alloc_uncached(ctypes.byref(F2), nmax * SLOT) == 0
    st = torch.cuda.current_stream()
    for nwg, shape, u in itertools.product(nwgs, range(7), unrolls):
        for opol, spol in itertools.product((1, 2) if shape in (2, 4) else (1,),
                                            (1, 0) if shape not in (4, 5) else (1,)):
            def run():
                rc = lib.step_probe_run(shape, u, opol, spol, vp(S.data_ptr()), F, F2, vp(O.data_ptr()), SLOT,
                                        nwg, 512, reps, span, vp(st.cuda_stream))
                assert rc == 0, rc
            run()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                run()
                e1.record(st)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e-3)
            t = sorted(ts)[len(ts) // 2]
            ns, nd = OPS[shape]
            per_slot_us = t / reps * 1e6
            wg_gbs = (ns + nd) * SLOT / (t / reps) / 1e9
            print(json.dumps({"shape": NAMES[shape], "unroll": u, "out_pol": "nt" if opol == 1 else "sys",
                              "src_pol": "nt" if spol == 1 else "plain",
                              "nwg": nwg, "us_per_slot": round(per_slot_us, 2),
                              "wg_GBs": round(wg_gbs, 1), "total_GBs": round(wg_gbs * nwg, 1)}), flush=True)
    lib.step_probe_free(F)
    lib.step_probe_free(F2)


if __name__ == "__main__":
    sys.exit(main())
