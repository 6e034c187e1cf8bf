#!/usr/bin/env python3
"""One rank of the HIP-graph capture/replay test (tests/test_gpu_collectives.py).

argv: rank nranks uid_hex
Captures [LL all-reduce (small), direct all-reduce (mid), ring all-reduce
(large), ring reduce-scatter]
into one graph on a side stream (after an eager call on the current stream,
and followed by another), replays it 4 times with new integer-valued inputs (exact in any
fold order) and checks every output; then two captures interleaved on the
same comm (interleaved_captures); a group of ring and direct calls on two
streams inside one capture (group_in_capture); a reduce, a broadcast and an
all-gather in one capture (rooted_in_capture); then collectives that fail
inside a capture (failing_calls_in_capture); exit code 0 = all replays
correct."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from tests import _mp  # noqa: E402
from vccl_amd import nccl  # noqa: E402


def interleaved_captures(comm, rank, n):
    """two captures on one comm, interleaved.  Capture A forks a
    second stream sA2 before its first collective (X1 on sA), then capture B
    records Y on sB, then A's second collective X2 goes onto sA2.  X2 must
    wait for X1 inside graph A (the comm's ordering is kept per capture id),
    or the replay runs two collectives of the comm at once."""
    big = 3 << 20  # the ring / direct paths: concurrent calls would share FIFOs
    x1, x2, xb = (torch.empty(big, device="cuda") for _ in range(3))
    y1, y2, yb = (torch.empty(big, device="cuda") for _ in range(3))
    sA, sA2, sB = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    gA, gB = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    f32, add = nccl.ncclFloat32, nccl.ncclSum
    torch.cuda.synchronize()
    with torch.cuda.stream(sA):
        gA.capture_begin(capture_error_mode="relaxed")
    sA2.wait_stream(sA)  # sA2 joins capture A before X1 exists
    comm.all_reduce(x1.data_ptr(), y1.data_ptr(), big, f32, add, sA.cuda_stream)
    with torch.cuda.stream(sB):
        gB.capture_begin(capture_error_mode="relaxed")
    comm.all_reduce(xb.data_ptr(), yb.data_ptr(), big, f32, add, sB.cuda_stream)
    comm.all_reduce(x2.data_ptr(), y2.data_ptr(), big, f32, add, sA2.cuda_stream)
    sA.wait_stream(sA2)
    with torch.cuda.stream(sB):
        gB.capture_end()
    with torch.cuda.stream(sA):
        gA.capture_end()
    ok = True
    for it in range(3):
        def val(r, k):
            return ((torch.arange(big, device="cuda") * (r + 5 + k) + 11 * it) % 89).float()
        x1.copy_(val(rank, 1))
        x2.copy_(val(rank, 2))
        xb.copy_(val(rank, 3))
        torch.cuda.synchronize()
        gA.replay()
        gB.replay()
        torch.cuda.synchronize()
        for y, k in ((y1, 1), (y2, 2), (yb, 3)):
            ok &= torch.equal(y, sum(val(r, k) for r in range(n)))
    if not ok:
        print(f"rank {rank}: interleaved captures mismatch", flush=True)
    return ok


def rooted_in_capture(comm, rank, n):
    """A reduce (into rank 0), a broadcast (from the last rank) and an
    all-gather captured in one graph on one stream replay exactly with fresh
    inputs each time: the rooted rings keep their roots and partitions in the
    captured kernel arguments."""
    cnt = 700_001
    x, y = torch.empty(cnt, device="cuda"), torch.full((cnt,), float("nan"), device="cuda")
    b = torch.empty(cnt, device="cuda")
    ag_in, ag_out = torch.empty(4099, device="cuda"), torch.empty(4099 * n, device="cuda")
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    f32 = nccl.ncclFloat32
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        g.capture_begin(capture_error_mode="relaxed")
        comm.reduce(x.data_ptr(), y.data_ptr() if rank == 0 else 0, cnt, f32, nccl.ncclSum, 0, s.cuda_stream)
        comm.broadcast(b.data_ptr(), b.data_ptr(), cnt, f32, n - 1, s.cuda_stream)
        comm.all_gather(ag_in.data_ptr(), ag_out.data_ptr(), 4099, f32, s.cuda_stream)
        g.capture_end()
    ok = True
    for it in range(3):
        def val(r, m, k):
            return ((torch.arange(m, device="cuda") * (r + 7 + k) + 3 * it) % 79).float()
        x.copy_(val(rank, cnt, 0))
        b.copy_(val(rank, cnt, 1))
        ag_in.copy_(val(rank, 4099, 2))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        if rank == 0:
            ok &= torch.equal(y, sum(val(r, cnt, 0) for r in range(n)))
        ok &= torch.equal(b, val(n - 1, cnt, 1))
        ok &= torch.equal(ag_out, torch.cat([val(r, 4099, 2) for r in range(n)]))
    if not ok:
        print(f"rank {rank}: rooted collectives in capture mismatch", flush=True)
    return ok


def group_in_capture(comm, rank, n):
    """A group of ring and direct calls on two streams inside one capture:
    the planned sequence (VCCL's group plan, several launches joined onto one
    stream) is captured as a fork / join in the graph and replays exactly."""
    sizes = [(0, 5 << 20), (0, 300_001), (1, 1 << 20), (0, 9 << 20), (0, 500_001)]  # (coll, count)
    xs = [torch.empty(c * n if coll == 1 else c, device="cuda") for coll, c in sizes]
    ys = [torch.empty(c, device="cuda") for _, c in sizes]
    sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    f32, add = nccl.ncclFloat32, nccl.ncclSum
    torch.cuda.synchronize()
    with torch.cuda.stream(sA):
        g.capture_begin(capture_error_mode="relaxed")
    sB.wait_stream(sA)
    nccl.group_start()
    for i, ((coll, c), x, y) in enumerate(zip(sizes, xs, ys)):
        st = (sA if i % 2 == 0 else sB).cuda_stream
        if coll == 0:
            comm.all_reduce(x.data_ptr(), y.data_ptr(), c, f32, add, st)
        else:
            comm.reduce_scatter(x.data_ptr(), y.data_ptr(), c, f32, add, st)
    nccl.group_end()
    sA.wait_stream(sB)
    with torch.cuda.stream(sA):
        g.capture_end()
    ok = True
    for it in range(3):
        def val(r, m, k):
            return ((torch.arange(m, device="cuda") * (r + 3 + k) + 5 * it) % 83).float()
        for k, ((coll, c), x) in enumerate(zip(sizes, xs)):
            x.copy_(val(rank, x.numel(), k))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        for k, ((coll, c), y) in enumerate(zip(sizes, ys)):
            full = sum(val(r, c * n if coll == 1 else c, k) for r in range(n))
            ok &= torch.equal(y, full[rank * c:(rank + 1) * c] if coll == 1 else full)
    if not ok:
        print(f"rank {rank}: group in capture mismatch", flush=True)
    return ok


def captures_on_destroyed_streams(comm, rank, n):
    """The capture-ordering pool after 16 captures whose streams were
    destroyed: each entry's capture has ended and its stream is gone, so a
    new capture must find a free entry (the liveness query on a destroyed
    stream handle reads as ended, host/enqueue.cc capture_live) — no crash, no
    refusal — and replay exactly."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    vp = ctypes.c_void_p
    small = 2048
    x = torch.arange(small, device="cuda", dtype=torch.float32) + rank
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    for i in range(16):
        st, graph = vp(), vp()
        assert hip.hipStreamCreate(ctypes.byref(st)) == 0
        assert hip.hipStreamBeginCapture(st, 2) == 0  # hipStreamCaptureModeRelaxed
        comm.all_reduce(x.data_ptr(), y.data_ptr(), small, nccl.ncclFloat32, nccl.ncclSum, st.value)
        assert hip.hipStreamEndCapture(st, ctypes.byref(graph)) == 0
        assert hip.hipGraphDestroy(graph) == 0
        assert hip.hipStreamDestroy(st) == 0
    s, g = torch.cuda.Stream(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        comm.all_reduce(x.data_ptr(), y.data_ptr(), small, nccl.ncclFloat32, nccl.ncclSum, s.cuda_stream)
    y.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    ok = torch.equal(y, sum(torch.arange(small, device="cuda", dtype=torch.float32) + r for r in range(n)))
    if not ok:
        print(f"rank {rank}: capture after destroyed-stream captures mismatch", flush=True)
    return ok


def failing_calls_in_capture(comm, rank, n):
    """collectives that fail inside a HIP graph capture return
    an ncclResult_t and leave the capture and the process usable.
    (a) inside one capture: a valid all-reduce, then calls the library
        refuses (invalid datatype; a PreMulSum op of another datatype,
        enqueue.cc:2301-2305), then another valid all-reduce — the capture
        ends cleanly and its replay is exact;
    (b) 17 captures live on one comm at once: the 17th call finds every
        ordering entry taken by a live capture and is refused with
        ncclInvalidUsage instead of silently dropping a live capture's
        ordering; all captures then end cleanly, and an eager
        call afterwards is exact."""
    m = 3 << 20
    xa, xb = torch.empty(m, device="cuda"), torch.empty(m, device="cuda")
    ya, yb = torch.empty_like(xa), torch.empty_like(xb)
    scal = torch.ones(1, dtype=torch.float16, device="cuda")
    uop = comm.create_premulsum(scal.data_ptr(), nccl.ncclFloat16, nccl.ncclScalarDevice)
    s, g = torch.cuda.Stream(), torch.cuda.CUDAGraph()
    codes = []
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        sp = s.cuda_stream
        comm.all_reduce(xa.data_ptr(), ya.data_ptr(), m, nccl.ncclFloat32, nccl.ncclSum, sp)
        for dt, op in ((99, nccl.ncclSum), (nccl.ncclFloat32, uop)):
            try:
                comm.all_reduce(xa.data_ptr(), ya.data_ptr(), m, dt, op, sp)
                codes.append(0)
            except nccl.VcclError as e:
                codes.append(e.code)
        comm.all_reduce(xb.data_ptr(), yb.data_ptr(), m, nccl.ncclFloat32, nccl.ncclSum, sp)
    ok = codes == [nccl.ncclInvalidArgument, nccl.ncclInvalidArgument]
    for it in range(2):
        def val(r, k):
            return ((torch.arange(m, device="cuda") * (r + 2 + k) + 5 * it) % 61).float()
        xa.copy_(val(rank, 0))
        xb.copy_(val(rank, 1))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        ok &= torch.equal(ya, sum(val(r, 0) for r in range(n)))
        ok &= torch.equal(yb, sum(val(r, 1) for r in range(n)))
    comm.destroy_op(uop)
    # (b) 17 live captures on one comm (the ordering pool holds 16)
    k = 17
    small = 1024
    xs = [torch.full((small,), float(i + rank), device="cuda") for i in range(k)]
    ys = [torch.empty(small, device="cuda") for _ in range(k)]
    streams = [torch.cuda.Stream() for _ in range(k)]
    graphs = [torch.cuda.CUDAGraph() for _ in range(k)]
    res = []
    torch.cuda.synchronize()
    for i in range(k):
        with torch.cuda.stream(streams[i]):
            graphs[i].capture_begin(capture_error_mode="relaxed")
        try:
            comm.all_reduce(xs[i].data_ptr(), ys[i].data_ptr(), small, nccl.ncclFloat32, nccl.ncclSum,
                            streams[i].cuda_stream)
            res.append(0)
        except nccl.VcclError as e:
            res.append(e.code)
    for i in reversed(range(k)):
        with torch.cuda.stream(streams[i]):
            graphs[i].capture_end()
    ok &= res == [0] * 16 + [nccl.ncclInvalidUsage]
    # the process is usable: an eager call, exact
    x = torch.arange(4099, device="cuda", dtype=torch.float32) + rank
    y = torch.empty_like(x)
    comm.all_reduce(x.data_ptr(), y.data_ptr(), 4099, nccl.ncclFloat32, nccl.ncclSum,
                    torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ok &= torch.equal(y, sum(torch.arange(4099, device="cuda", dtype=torch.float32) + r for r in range(n)))
    if not ok:
        print(f"rank {rank}: failing calls in capture: codes {codes}, pool {res}", flush=True)
    return ok


def main():
    rank, n = int(sys.argv[1]), int(sys.argv[2])
    uid = nccl.unique_id_from_bytes(bytes.fromhex(sys.argv[3]))
    _mp.bind(rank, n)
    comm = nccl.Comm.init_rank(n, uid, rank)
    small, mid, large, rc = 10_001, 600_001, 3 << 20, 100_003
    xs = torch.empty(small, device="cuda")
    xm = torch.empty(mid, device="cuda")
    ym = torch.empty_like(xm)
    xl = torch.empty(large, device="cuda")
    xr = torch.empty(rc * n, device="cuda")
    ys, yl, yr = torch.empty_like(xs), torch.empty_like(xl), torch.empty(rc, device="cuda")
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    # An eager call on ANOTHER stream right before the capture: the capture
    # must not wait on (or overwrite) the comm's eager ordering event, which
    # was recorded outside it (enqueue.cc stream_order / stream_mark).
    eager_x = torch.arange(4099, device="cuda", dtype=torch.float32) + rank
    eager_y = torch.empty_like(eager_x)
    comm.all_reduce(eager_x.data_ptr(), eager_y.data_ptr(), 4099, nccl.ncclFloat32, nccl.ncclSum,
                    torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        sp = s.cuda_stream
        comm.all_reduce(xs.data_ptr(), ys.data_ptr(), small, nccl.ncclFloat32, nccl.ncclSum, sp)
        comm.all_reduce(xm.data_ptr(), ym.data_ptr(), mid, nccl.ncclFloat32, nccl.ncclSum, sp)
        comm.all_reduce(xl.data_ptr(), yl.data_ptr(), large, nccl.ncclFloat32, nccl.ncclSum, sp)
        comm.reduce_scatter(xr.data_ptr(), yr.data_ptr(), rc, nccl.ncclFloat32, nccl.ncclSum, sp)
    ok = True
    for it in range(4):
        def val(r, m):
            return ((torch.arange(m, device="cuda") * (r + 3) + 7 * it) % 97).float()
        xs.copy_(val(rank, small))
        xm.copy_(val(rank, mid))
        xl.copy_(val(rank, large))
        xr.copy_(val(rank, rc * n))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        ok &= torch.equal(ys, sum(val(r, small) for r in range(n)))
        ok &= torch.equal(ym, sum(val(r, mid) for r in range(n)))
        ok &= torch.equal(yl, sum(val(r, large) for r in range(n)))
        ok &= torch.equal(yr, sum(val(r, rc * n) for r in range(n))[rank * rc:(rank + 1) * rc])
    # eager again on the first stream after the replays
    exp_eager = sum(torch.arange(4099, device="cuda", dtype=torch.float32) + r for r in range(n))
    ok &= torch.equal(eager_y, exp_eager)
    eager_y.zero_()
    comm.all_reduce(eager_x.data_ptr(), eager_y.data_ptr(), 4099, nccl.ncclFloat32, nccl.ncclSum,
                    torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ok &= torch.equal(eager_y, exp_eager)
    ok &= interleaved_captures(comm, rank, n)
    ok &= group_in_capture(comm, rank, n)
    ok &= rooted_in_capture(comm, rank, n)
    ok &= failing_calls_in_capture(comm, rank, n)
    ok &= captures_on_destroyed_streams(comm, rank, n)
    ok &= comm.async_error() == 0
    comm.destroy()
    sys.exit(0 if ok else 4)


if __name__ == "__main__":
    main()
