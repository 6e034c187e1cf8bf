#!/usr/bin/env python3
"""Host cost per call of the HIP runtime pieces under a collective call:
hipEventRecord, hipStreamWaitEvent, a 1 KiB byte-copy launch through the C
ABI (vcclReduceCopy) and a world-size-1 out-of-place ncclAllReduce (1 KiB).
Prints one JSON line (us per call, host wall over N back-to-back calls)."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vccl_amd import nccl  # noqa: E402


def per_call(fn, n=5000):
    for _ in range(100):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    dt = time.perf_counter() - t0
    torch.cuda.synchronize()
    return round(dt / n * 1e6, 3)


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    torch.cuda.set_device(0)
    s = torch.cuda.current_stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    ev = ctypes.c_void_p()
    assert hip.hipEventCreateWithFlags(ctypes.byref(ev), 2) == 0  # hipEventDisableTiming
    x = torch.rand(256, device="cuda")
    y = torch.empty_like(x)
    s2 = torch.cuda.Stream()
    res = {
        "python_ctypes_noop": per_call(lambda: hip.hipGetDevice(ctypes.byref(ctypes.c_int()))),
        "hipEventRecord": per_call(lambda: hip.hipEventRecord(ev, sp)),
        "hipEventRecord+hipStreamWaitEvent": per_call(
            lambda: (hip.hipEventRecord(ev, sp), hip.hipStreamWaitEvent(ctypes.c_void_p(s2.cuda_stream), ev, 0))),
        "reduce_copy_1KiB_launch": per_call(lambda: nccl.reduce_copy(
            nccl.vcclDevCopy, nccl.ncclUint8, 0, [x.data_ptr()], [y.data_ptr()], 1024, s.cuda_stream)),
        "hipMemcpyAsync_1KiB": per_call(lambda: hip.hipMemcpyAsync(
            ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(x.data_ptr()), ctypes.c_size_t(1024), 3, sp)),
    }
    comm = nccl.Comm.init_rank(1, nccl.get_unique_id(), 0)
    res["ncclAllReduce_1KiB_world1_oop"] = per_call(
        lambda: comm.all_reduce(x.data_ptr(), y.data_ptr(), 256, nccl.ncclFloat32, nccl.ncclSum, s.cuda_stream))
    comm.destroy()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
