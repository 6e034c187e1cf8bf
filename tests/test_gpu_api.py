"""NCCL C API on one rank (BASELINE config 1) and API-level error behaviour.

Reference paths: ncclEnqueueCheck (enqueue.cc:2448-2525), ArgsCheck
(misc/argcheck.cc:45-86), nRanks==1 -> ncclLaunchOneRank (onerank.cu:47-83),
ncclRedOpCreatePreMulSum (enqueue.cc:2528-2567).
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from tests.gpu_util import stream_ptr  # noqa: E402
from vccl_amd import nccl  # noqa: E402


@pytest.fixture(scope="module")
def comm1():
    uid = nccl.get_unique_id()
    c = nccl.Comm.init_rank(1, uid, 0)
    yield c
    c.destroy()


def test_comm_queries(comm1):
    assert comm1.count == 1 and comm1.rank == 0 and comm1.device == 0
    assert comm1.async_error() == nccl.ncclSuccess


def test_config1_allreduce_1kib_identity(comm1):
    """ncclAllReduce fp32 sum, 1 KiB, world 1: output bitwise equal to input."""
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.rand(256, device="cuda", generator=g) * 2 - 1
    y = torch.full_like(x, float("nan"))
    comm1.all_reduce(x.data_ptr(), y.data_ptr(), 256, nccl.ncclFloat32, nccl.ncclSum, stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(x.view(torch.int32), y.view(torch.int32))
    x0 = x.clone()
    comm1.all_reduce(x.data_ptr(), x.data_ptr(), 256, nccl.ncclFloat32, nccl.ncclSum, stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(x0.view(torch.int32), x.view(torch.int32))


@pytest.mark.parametrize("dt,tdt", [(nccl.ncclFloat32, torch.float32), (nccl.ncclFloat16, torch.float16),
                                    (nccl.ncclBfloat16, torch.bfloat16), (nccl.ncclFloat64, torch.float64),
                                    (nccl.ncclInt32, torch.int32), (nccl.ncclUint8, torch.uint8),
                                    (nccl.ncclFloat8e4m3, torch.float8_e4m3fn),
                                    (nccl.ncclFloat8e5m2, torch.float8_e5m2)])
@pytest.mark.parametrize("op", [0, 1, 2, 3, 4])
def test_one_rank_all_ops(comm1, dt, tdt, op):
    n = 4099
    if tdt in (torch.float8_e4m3fn, torch.float8_e5m2):  # finite codes only (avg: x * 1.0)
        x = torch.randn(n).to(tdt).cuda()
    elif tdt.is_floating_point:
        x = torch.randn(n, device="cuda").to(tdt)
    else:
        x = torch.randint(0, 100, (n,), device="cuda").to(tdt)
    y = torch.empty_like(x)
    comm1.all_reduce(x.data_ptr(), y.data_ptr(), n, dt, op, stream_ptr())
    torch.cuda.synchronize()
    # avg on floats runs the PreMulSum kernel with scalar 1/1 = 1: x*1 == x
    assert torch.equal(x.view(torch.uint8), y.view(torch.uint8))
    z = torch.empty_like(x)
    comm1.reduce_scatter(x.data_ptr(), z.data_ptr(), n, dt, op, stream_ptr())
    w = torch.empty_like(x)
    comm1.all_gather(x.data_ptr(), w.data_ptr(), n, dt, stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(x.view(torch.uint8), z.view(torch.uint8))
    assert torch.equal(x.view(torch.uint8), w.view(torch.uint8))


@pytest.mark.parametrize("nbytes", [1, 1023, 1024, 4097, (1 << 20) - 3, (1 << 20) + 5, 3 << 20])
@pytest.mark.parametrize("shift", [0, 3])
def test_one_rank_copy_sizes(comm1, nbytes, shift):
    """World-size-1 copies on both sides of the kernel-copy / hipMemcpy
    threshold (1 MiB), misaligned by `shift` bytes: AR, RS and AG."""
    src = torch.randint(0, 256, (nbytes + shift,), dtype=torch.uint8, device="cuda")[shift:]
    for coll in ("ar", "rs", "ag"):
        dst = torch.zeros(nbytes + 2 * shift + 1, dtype=torch.uint8, device="cuda")
        d = dst[shift:shift + nbytes]
        if coll == "ar":
            comm1.all_reduce(src.data_ptr(), d.data_ptr(), nbytes, nccl.ncclUint8, 0, stream_ptr())
        elif coll == "rs":
            comm1.reduce_scatter(src.data_ptr(), d.data_ptr(), nbytes, nccl.ncclUint8, 2, stream_ptr())
        else:
            comm1.all_gather(src.data_ptr(), d.data_ptr(), nbytes, nccl.ncclUint8, stream_ptr())
        torch.cuda.synchronize()
        assert torch.equal(d, src), coll
        assert int(dst[:shift].sum()) == 0 and int(dst[shift + nbytes:].sum()) == 0, coll


def test_user_premulsum(comm1):
    n = 1000
    x = torch.randn(n, device="cuda")
    y = torch.empty_like(x)
    half = ctypes.c_float(0.5)
    op = comm1.create_premulsum(ctypes.addressof(half), nccl.ncclFloat32, nccl.ncclScalarHostImmediate)
    assert op >= nccl.ncclAvg + 1
    comm1.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, op, stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(y, x * 0.5)
    # device-resident scalar, read by the kernel
    s = torch.tensor([3.0], device="cuda")
    op2 = comm1.create_premulsum(s.data_ptr(), nccl.ncclFloat32, nccl.ncclScalarDevice)
    comm1.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, op2, stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(y, x * 3.0)
    # type mismatch with the op's datatype -> invalid argument (enqueue.cc:2301-2305)
    with pytest.raises(nccl.VcclError) as e:
        comm1.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat64, op, stream_ptr())
    assert e.value.code == nccl.ncclInvalidArgument
    comm1.destroy_op(op)
    comm1.destroy_op(op2)
    with pytest.raises(nccl.VcclError):
        comm1.destroy_op(op)


def test_user_premulsum_fp8(comm1):
    """ncclRedOpCreatePreMulSum on fp8 (scalar = 1 fp8 byte; preOp =
    fp8(half(x) * half(scalar)), reduce_kernel.h:586-624) vs the oracle."""
    codes = torch.arange(256, dtype=torch.uint8)
    for dt in (nccl.ncclFloat8e4m3, nccl.ncclFloat8e5m2):
        x = codes.cuda()
        y = torch.empty_like(x)
        scalar = ctypes.c_uint8(0x2B if dt == nccl.ncclFloat8e4m3 else 0x35)  # ~1/3
        op = comm1.create_premulsum(ctypes.addressof(scalar), dt, nccl.ncclScalarHostImmediate)
        comm1.all_reduce(x.data_ptr(), y.data_ptr(), 256, dt, op, stream_ptr())
        torch.cuda.synchronize()
        exp = O.reduce_copy(3, dt, scalar.value, [codes.numpy()], pre_op_args=[scalar.value])[0]
        got = y.cpu().numpy()
        nan = O.fp8_bits_to_f32(dt, exp) != O.fp8_bits_to_f32(dt, exp)
        assert np.array_equal(got[~nan], exp[~nan])
        assert np.all(np.isnan(O.fp8_bits_to_f32(dt, got[nan])))
        comm1.destroy_op(op)


def test_arg_errors(comm1):
    L = nccl.lib()
    x = torch.zeros(16, device="cuda")
    p = x.data_ptr()
    assert L.ncclAllReduce(p, p, 16, 12, 0, comm1.handle, None) == nccl.ncclInvalidArgument  # bad type
    assert L.ncclAllReduce(p, p, 16, 7, 17, comm1.handle, None) == nccl.ncclInvalidArgument  # unknown op
    assert L.ncclAllReduce(p, p, 16, 7, -1, comm1.handle, None) == nccl.ncclInvalidArgument
    assert L.ncclAllReduce(p, p, 16, 7, 0, None, None) == nccl.ncclInvalidArgument  # NULL comm
    # fp8 is native on gfx950 (the reference rejects it below sm90, enqueue.cc:2379-2384)
    assert L.ncclAllReduce(p, p, 16, nccl.ncclFloat8e4m3, 0, comm1.handle, None) == nccl.ncclSuccess
    assert L.ncclAllReduce(p, p, 0, 7, 0, comm1.handle, None) == nccl.ncclSuccess  # empty: no-op
    assert L.ncclGroupEnd() == nccl.ncclInvalidUsage  # not in a group
    assert nccl.lib().ncclGetErrorString(4) == b"invalid argument (run with NCCL_DEBUG=WARN for details)"


def test_group_calls(comm1):
    xs = [torch.randn(1000 + i, device="cuda") for i in range(4)]
    ys = [torch.empty_like(x) for x in xs]
    nccl.group_start()
    nccl.group_start()  # nested
    for x, y in zip(xs, ys):
        comm1.all_reduce(x.data_ptr(), y.data_ptr(), x.numel(), nccl.ncclFloat32, nccl.ncclSum, stream_ptr())
    nccl.group_end()
    nccl.group_end()
    torch.cuda.synchronize()
    for x, y in zip(xs, ys):
        assert torch.equal(x, y)


def test_oracle_allreduce_one_rank_semantics():
    # the oracle's API-level restatement agrees (world 1: copy / x*1)
    x = np.arange(10, dtype=np.float32)
    assert np.array_equal(O.allreduce(4, 7, [x]), x)


def test_debug_subsys_filters_info_lines():
    """NCCL_DEBUG_SUBSYS (debug.cc:30, 57-111): with NCCL_DEBUG=INFO the
    default mask (INIT, BOOTSTRAP, ENV) prints the init lines but not the
    per-call COLL trace; COLL alone prints only the trace; ^INIT prints every
    subsystem but INIT."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from vccl_amd import nccl
c = nccl.Comm.init_rank(1, nccl.get_unique_id(), 0)
x = torch.ones(256, device="cuda"); y = torch.empty_like(x)
c.all_reduce(x.data_ptr(), y.data_ptr(), 256, nccl.ncclFloat32, nccl.ncclSum,
             torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize(); c.destroy()
"""
    base = {k: v for k, v in os.environ.items()
            if k not in ("NCCL_DEBUG", "VCCL_DEBUG", "NCCL_DEBUG_SUBSYS", "VCCL_DEBUG_SUBSYS")}
    seen = {}
    for sub in (None, "COLL", "^INIT"):
        env = dict(base, NCCL_DEBUG="INFO")
        if sub:
            env["NCCL_DEBUG_SUBSYS"] = sub
        r = subprocess.run([sys.executable, "-c", code, root], capture_output=True, text=True, env=env,
                           timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        seen[sub] = ("dev 0: bootstrap" in r.stderr, "AllReduce: opCount" in r.stderr)
    assert seen == {None: (True, False), "COLL": (False, True), "^INIT": (False, True)}, seen
