#!/usr/bin/env python3
"""One rank of tests/test_gpu_nonblocking.py (non-blocking communicators,
SURVEY.md §8b; the reference's group.cc:553-576, init.cc:1836-1860).

argv: rank nranks outdir uid_hex uid2_hex
1. ncclCommInitRankConfig with config.blocking = 0 returns ncclInProgress;
   ncclCommGetAsyncError reports ncclInProgress until the initialisation has
   ended, then ncclSuccess; an all-reduce on the comm is then exact.
2. NCCL_COMM_BLOCKING=0 makes a plain ncclCommInitRank non-blocking the same
   way (the environment wins over the config, envConfigOverride).
Verdict to <outdir>/rank<r>.json."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402


def poll(h):
    st, polls, t0 = ctypes.c_int(nccl.ncclInProgress), 0, time.monotonic()
    while st.value == nccl.ncclInProgress and time.monotonic() - t0 < 120:
        nccl.check(nccl.lib().ncclCommGetAsyncError(h, ctypes.byref(st)), "ncclCommGetAsyncError")
        polls += 1
        if st.value == nccl.ncclInProgress:
            time.sleep(1e-3)
    return st.value, polls


def exact_allreduce(comm, rank, n):
    x = torch.empty(1 << 20, device="cuda")
    y = torch.full_like(x, float("nan"))
    bench.pattern_fill(x, rank, n)
    comm.all_reduce(x.data_ptr(), y.data_ptr(), x.numel(), nccl.ncclFloat32, nccl.ncclSum,
                    torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return bench.pattern_ok(y, n)


def main():
    rank, n, outdir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    uids = [nccl.unique_id_from_bytes(bytes.fromhex(h)) for h in sys.argv[4:6]]
    _mp.bind(rank, n)
    res = {"rank": rank}
    cfg = nccl.ncclConfig_t.initializer(blocking=0)
    h = ctypes.c_void_p()
    res["config_rc"] = nccl.lib().ncclCommInitRankConfig(ctypes.byref(h), n, uids[0], rank, ctypes.byref(cfg))
    res["config_state"], res["config_polls"] = poll(h)
    c = nccl.Comm(h.value)
    res["config_exact"] = exact_allreduce(c, rank, n)
    c.destroy()
    os.environ["NCCL_COMM_BLOCKING"] = "0"
    h2 = ctypes.c_void_p()
    res["env_rc"] = nccl.lib().ncclCommInitRank(ctypes.byref(h2), n, uids[1], rank)
    res["env_state"], _ = poll(h2)
    c2 = nccl.Comm(h2.value)
    res["env_exact"] = exact_allreduce(c2, rank, n)
    c2.destroy()
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
