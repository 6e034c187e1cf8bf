#!/usr/bin/env python3
"""Single-process multi-GPU check: ncclCommInitAll over every visible GPU.

argv: ndev | comma-separated device list (e.g. "0,0" with
VCCL_ALLOW_SHARED_DEVICE=1 rehearses the path on a one-GPU box)
The reference's own test-harness shape (init.cc:1750-1814):
one thread drives ndev communicators, one per GPU, so peers are mapped with
hipDeviceEnablePeerAccess + raw pointers (init.cc map_peer) instead of IPC.
Runs, inside ncclGroupStart/End, the one-shot LL (64 KiB), the library's
default (64 MiB) and the forced ring (64 MiB) all-reduce, and a bf16
reduce-scatter + all-gather, all on bench.py's integer pattern (exact in any
fold order).  Prints one JSON line {"ok": ..., "checks": {...}}; exit 0.
Launched as a child process by bench.py (rank 0 of an N > 1 run) and by
tests/test_gpu_collectives.py when the box has more than one GPU.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from vccl_amd import nccl  # noqa: E402


def main():
    arg = sys.argv[1]
    dev_of = [int(v) for v in arg.split(",")] if "," in arg else list(range(int(arg)))
    ndev = len(dev_of)
    devs = list(range(ndev))  # rank indices; rank d runs on GPU dev_of[d]
    comms = nccl.Comm.init_all(dev_of)
    streams = []
    for d in devs:
        torch.cuda.set_device(dev_of[d])
        streams.append(torch.cuda.Stream())
    checks = {}

    def run_ar(name, nbytes, dtype, algo):
        n = nbytes // torch.tensor([], dtype=bench._TDT[dtype]).element_size()
        xs, ys = [], []
        for d in devs:
            torch.cuda.set_device(dev_of[d])
            x = torch.empty(n, dtype=bench._TDT[dtype], device="cuda")
            bench.pattern_fill(x, d, ndev)
            xs.append(x)
            ys.append(torch.full((n,), float("nan"), dtype=x.dtype, device="cuda"))
            comms[d].set_algo(algo)
            torch.cuda.synchronize()
        nccl.group_start()
        for d in devs:
            comms[d].all_reduce(xs[d].data_ptr(), ys[d].data_ptr(), n, bench._CODE[dtype],
                                nccl.ncclSum, streams[d].cuda_stream)
        nccl.group_end()
        ok = True
        for d in devs:
            torch.cuda.set_device(dev_of[d])
            torch.cuda.synchronize()
            ok &= bench.pattern_ok(ys[d], ndev) and comms[d].async_error() == 0
            comms[d].set_algo(None)
        checks[name] = {"ok": bool(ok), "algo": comms[0].coll_algo(0, n, bench._CODE[dtype])
                        if algo is None else algo}

    def run_rs_ag(nbytes):
        n = nbytes // 2
        rc = n // ndev
        xs, shards = [], []
        for d in devs:
            torch.cuda.set_device(dev_of[d])
            x = torch.empty(rc * ndev, dtype=torch.bfloat16, device="cuda")
            bench.pattern_fill(x, d, ndev)
            xs.append(x)
            shards.append(torch.full((rc,), float("nan"), dtype=torch.bfloat16, device="cuda"))
            torch.cuda.synchronize()
        nccl.group_start()
        for d in devs:
            comms[d].reduce_scatter(xs[d].data_ptr(), shards[d].data_ptr(), rc, nccl.ncclBfloat16,
                                    nccl.ncclSum, streams[d].cuda_stream)
        nccl.group_end()
        rs_ok = True
        for d in devs:
            torch.cuda.set_device(dev_of[d])
            torch.cuda.synchronize()
            rs_ok &= bench.pattern_ok(shards[d], ndev, base=d * rc)
            xs[d].fill_(float("nan"))
            torch.cuda.synchronize()
        nccl.group_start()
        for d in devs:
            comms[d].all_gather(shards[d].data_ptr(), xs[d].data_ptr(), rc, nccl.ncclBfloat16,
                                streams[d].cuda_stream)
        nccl.group_end()
        ag_ok = True
        for d in devs:
            torch.cuda.set_device(dev_of[d])
            torch.cuda.synchronize()
            ag_ok &= bench.pattern_ok(xs[d], ndev) and comms[d].async_error() == 0
        checks[f"rs_bf16_{nbytes}"] = {"ok": bool(rs_ok)}
        checks[f"ag_bf16_{nbytes}"] = {"ok": bool(ag_ok)}

    try:
        run_ar("ar_ll_64KiB", 64 << 10, "f32", None)
        run_ar("ar_default_64MiB", 64 << 20, "f32", None)
        run_ar("ar_ring_64MiB", 64 << 20, "f32", "ring")
        run_ar("ar_f16_16KiB", 16 << 10, "f16", None)
        run_rs_ag(64 << 20)
        err = None
    except Exception as e:  # noqa: BLE001 - reported in the verdict
        err = repr(e)
    for c in comms:
        c.destroy()
    ok = err is None and all(v["ok"] for v in checks.values())
    print(json.dumps({"ok": ok, "ndev": ndev, "devices": dev_of, "peer_access": "hipDeviceEnablePeerAccess",
                      "checks": checks, **({"error": err} if err else {})}), flush=True)


if __name__ == "__main__":
    main()
