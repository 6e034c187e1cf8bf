#!/usr/bin/env python3
"""One rank of the broadcast test (tests/test_gpu_collectives.py).

argv: rank nranks uid_hex
ncclBroadcast / ncclBcast (broadcast.h: the ring from the root, byte copies)
over sizes 1 B - 24 MiB, every root, out of place and in place, then ONE
group of broadcasts from different roots of different types plus an
all-reduce (fused ring parts with per-part roots).  Every byte checked:
exit 0 on success."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402


def payload(nbytes, root, tag):
    g = torch.Generator(device="cpu").manual_seed(1000 * tag + root)
    return torch.randint(0, 256, (nbytes,), dtype=torch.uint8, generator=g).cuda()


def main():
    rank, n = int(sys.argv[1]), int(sys.argv[2])
    uid = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[3]))
    _mp.bind(rank, n)
    comm = nccl.Comm.init_rank(n, uid, rank)
    sp = torch.cuda.current_stream().cuda_stream
    bad = []
    tag = 0
    for nbytes in (1, 7, 4099, (1 << 20) + 5, 24 << 20):
        for root in range(n):
            for inplace in (False, True):
                tag += 1
                want = payload(nbytes, root, tag)
                if inplace:
                    buf = want.clone() if rank == root else torch.full((nbytes,), 0xAB, dtype=torch.uint8,
                                                                      device="cuda")
                    L = nccl.lib()
                    nccl.check(L.ncclBcast(ctypes.c_void_p(buf.data_ptr()), ctypes.c_size_t(nbytes), nccl.ncclUint8,
                                           root, comm.handle, ctypes.c_void_p(sp)), "ncclBcast")
                    out = buf
                else:
                    src = want if rank == root else torch.zeros(1, dtype=torch.uint8, device="cuda")
                    out = torch.full((nbytes,), 0xCD, dtype=torch.uint8, device="cuda")
                    comm.broadcast(src.data_ptr() if rank == root else 0, out.data_ptr(), nbytes,
                                   nccl.ncclUint8, root, sp)
                torch.cuda.synchronize()
                if not torch.equal(out, want):
                    bad.append((nbytes, root, inplace))
    # one group: broadcasts of f32 / bf16 / i32 from different roots + an all-reduce
    specs = [(torch.float32, 7, 300_001), (torch.bfloat16, 9, 70_000), (torch.int32, 2, 5_000), (torch.float32, 7, 77)]
    outs, wants = [], []
    for i, (tdt, code, cnt) in enumerate(specs):
        g = torch.Generator(device="cpu").manual_seed(77 + i)
        w = torch.randint(-100, 100, (cnt,), generator=g).to(tdt).cuda()
        root = i % n
        outs.append(torch.zeros(cnt, dtype=tdt, device="cuda") if rank != root else w.clone())
        wants.append((w, root))
    x = torch.empty(1 << 20, device="cuda")
    bench.pattern_fill(x, rank, n, base=5 << 20)
    y = torch.full_like(x, float("nan"))
    torch.cuda.synchronize()
    nccl.group_start()
    for i, (tdt, code, cnt) in enumerate(specs):
        root = wants[i][1]
        comm.broadcast(outs[i].data_ptr(), outs[i].data_ptr(), cnt, code, root, sp)
    comm.all_reduce(x.data_ptr(), y.data_ptr(), x.numel(), nccl.ncclFloat32, nccl.ncclSum, sp)
    nccl.group_end()
    torch.cuda.synchronize()
    for i, (w, root) in enumerate(wants):
        if not torch.equal(outs[i], w):
            bad.append(("group", i, root))
    if not bench.pattern_ok(y, n, base=5 << 20):
        bad.append(("group all-reduce",))
    err = comm.async_error()
    comm.destroy()
    if bad or err:
        print(f"rank {rank}: {bad} async error {err}", flush=True)
        sys.exit(1)


if __name__ == "__main__":
    main()
