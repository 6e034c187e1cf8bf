"""Parity of the HIP reduce-copy engine (vcclReduceCopy C ABI) on MI355X.

* every golden vector (10 types x 5 ops x {2,3,8} sources), bit-exact;
* the same against the CPU oracle at ragged sizes, misaligned pointers,
  several destinations, in-place operation;
* full-size (256 MiB, BASELINE config 2) 2-source f32 sum: bit-exact to
  numpy's a + b;
* C-ABI error behaviour (invalid op/type/counts).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests._util import FLOAT_TYPES, assert_bitexact, golden_rc_cases

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU, skipped there
    pytest.skip("needs a GPU", allow_module_level=True)

from tests.gpu_util import empty_dev, from_dev, stream_ptr, to_dev  # noqa: E402
from vccl_amd import nccl  # noqa: E402


def _run(dev_op, t, arg, srcs_np, n_dsts=1, pre=0, post=False, offsets=None, config=None):
    n = srcs_np[0].size
    dt = srcs_np[0].dtype
    offsets = offsets or [0] * (len(srcs_np) + n_dsts)
    keep, sp, dp = [], [], []
    for i, s in enumerate(srcs_np):
        tt, p = to_dev(s, offset=offsets[i])
        keep.append(tt)
        sp.append(p)
    outs = []
    for j in range(n_dsts):
        tt, p = empty_dev(n * dt.itemsize, offset=offsets[len(srcs_np) + j])
        outs.append((tt, offsets[len(srcs_np) + j]))
        dp.append(p)
    nccl.reduce_copy(dev_op, t, arg, sp, dp, n, stream_ptr(), pre_op_srcs=pre, post_op=post,
                     config=config)
    torch.cuda.synchronize()
    return [from_dev(tt, dt, n, off) for tt, off in outs]


def _dev_args(op, t, nsrc):
    dev_op, arg = nccl.host_to_dev_redop(op, t, nsrc)
    assert (dev_op, arg) == O.host_to_dev_redop(op, t, nsrc)
    pre = nsrc if dev_op == nccl.vcclDevPreMulSum else 0
    return dev_op, arg, pre, dev_op == nccl.vcclDevSumPostDiv


def test_golden_vectors_bitexact(golden):
    n = 0
    for key, t, op, nsrc, inp, exp in golden_rc_cases(golden):
        dev_op, arg, pre, post = _dev_args(op, t, nsrc)
        got = _run(dev_op, t, arg, [inp[i] for i in range(nsrc)], pre=pre, post=post)[0]
        assert_bitexact(t, got, exp, minmax=op in (2, 3), what=key)
        n += 1
    assert n == 150


def _rand(rng, t, n):
    if t in (0, 1, 2, 3, 4, 5):
        dt = O.NP_DTYPE[t]
        return rng.integers(0, 2**63, size=n, dtype=np.int64).astype(np.uint64).view(np.int64).astype(dt)
    if t == 9:
        return O.f32_to_bf16_bits(rng.uniform(-2, 2, n).astype(np.float32))
    if t in (10, 11):  # every fp8 code: NaN, saturating magnitudes, subnormals
        return rng.integers(0, 256, n).astype(np.uint8)
    return rng.uniform(-2, 2, n).astype(O.NP_DTYPE[t])


@pytest.mark.parametrize("t", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11])
@pytest.mark.parametrize("op", [0, 1, 2, 3, 4])
def test_ragged_sizes_vs_oracle(t, op):
    rng = np.random.default_rng(100 * t + op)
    for n in (1, 7, 16, 1000, 4099, 65536 + 13, 1 << 20):
        nsrc = 2 if n % 2 else 3
        srcs = [_rand(rng, t, n) for _ in range(nsrc)]
        dev_op, arg, pre, post = _dev_args(op, t, nsrc)
        got = _run(dev_op, t, arg, srcs, pre=pre, post=post)[0]
        exp = O.reduce_copy(dev_op, t, arg, srcs, pre_op_args=[arg] * pre, post_op=post)[0]
        assert_bitexact(t, got, exp, minmax=op in (2, 3), what=f"t{t} op{op} n{n}")


@pytest.mark.parametrize("t", [1, 6, 7, 8, 9, 10])
def test_misaligned_and_multi_dst(t):
    rng = np.random.default_rng(7 + t)
    n = 100_003
    sz = np.dtype(O.NP_DTYPE[t]).itemsize
    srcs = [_rand(rng, t, n) for _ in range(3)]
    exp = O.reduce_copy(0, t, 0, srcs)[0]
    # same misalignment on every pointer, then different misalignments
    for offs in ([sz] * 6, [0, sz, 2 * sz, 0, sz, 3 * sz]):
        outs = _run(0, t, 0, srcs, n_dsts=3, offsets=offs)
        for o in outs:
            assert_bitexact(t, o, exp, what=f"t{t} offs{offs}")


# Sources misaligned relative to destinations that share one misalignment:
# the body moves in 16-byte packs realigned by wavefront shuffle + funnel
# shift (reduce_copy_misaligned).  Sizes hit head-only, tail-only, one
# partial wave, whole hunks; bytes around every destination stay untouched.
SHIFT_OFFSETS = {1: ([1, 7, 15], [3, 3]), 2: ([2, 6, 14], [10, 10]),
                 4: ([0, 4, 12], [8, 8]), 8: ([8, 0, 8], [8, 8])}


@pytest.mark.parametrize("t", [0, 1, 2, 4, 6, 7, 8, 9, 10, 11])
@pytest.mark.parametrize("op", [0, 1, 2, 4])
def test_shifted_sources(t, op):
    rng = np.random.default_rng(900 + 10 * t + op)
    sz = np.dtype(O.NP_DTYPE[t]).itemsize
    soffs, doffs = SHIFT_OFFSETS[sz]
    for n in (1, 3, 17, 63, 1000, 4096 + 5, 100_003, (1 << 20) + 7):
        nsrc = 3 if n % 2 else 2
        srcs = [_rand(rng, t, n) for _ in range(nsrc)]
        dev_op, arg, pre, post = _dev_args(op, t, nsrc)
        exp = O.reduce_copy(dev_op, t, arg, srcs, pre_op_args=[arg] * pre, post_op=post)[0]
        offs = soffs[:nsrc] + doffs
        keep, sp = [], []
        for i, x in enumerate(srcs):
            tt, ptr = to_dev(x, offset=offs[i])
            keep.append(tt)
            sp.append(ptr)
        outs = [empty_dev(n * sz, offset=o) for o in doffs]
        nccl.reduce_copy(dev_op, t, arg, sp, [ptr for _, ptr in outs], n, stream_ptr(),
                         pre_op_srcs=pre, post_op=post)
        torch.cuda.synchronize()
        for (tt, _), o in zip(outs, doffs):
            got = from_dev(tt, O.NP_DTYPE[t], n, o)
            assert_bitexact(t, got, exp, minmax=op == 2, what=f"t{t} op{op} n{n} offs{offs}")
            raw = tt.cpu().numpy()
            assert (raw[:o] == 0xA5).all() and (raw[o + n * sz:] == 0xA5).all(), "guard bytes written"


def test_eight_sources_and_geometry_sweep():
    rng = np.random.default_rng(11)
    n = (1 << 22) + 5
    srcs = [rng.standard_normal(n).astype(np.float32) for _ in range(8)]
    exp = O.reduce_copy(0, 7, 0, srcs)[0]
    got = _run(0, 7, 0, srcs)[0]
    assert_bitexact(7, got, exp, what="8 srcs")
    two = srcs[:2]
    exp2 = two[0] + two[1]
    for cfg in ({"blockSize": 256, "unroll": 4, "gridBlocks": 0, "ntLoads": 0, "ntStores": 0},
                {"blockSize": 512, "unroll": 8, "gridBlocks": 1024, "ntLoads": 1, "ntStores": 1},
                {"blockSize": 1024, "unroll": 2, "gridBlocks": 7, "ntLoads": 0, "ntStores": 1},
                {"blockSize": 256, "unroll": 8, "gridBlocks": 0, "ntLoads": 1, "ntStores": 0}):
        got = _run(0, 7, 0, two, config=cfg)[0]
        assert np.array_equal(got.view(np.uint32), exp2.view(np.uint32)), cfg


def test_in_place():
    rng = np.random.default_rng(5)
    n = 1 << 20
    a = rng.standard_normal(n).astype(np.float32)
    b = rng.standard_normal(n).astype(np.float32)
    ta, pa = to_dev(a)
    tb, pb = to_dev(b)
    nccl.reduce_copy(0, 7, 0, [pa, pb], [pa], n, stream_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(from_dev(ta, np.float32, n), a + b)


def test_full_size_config2_bitexact():
    """BASELINE config 2: 2 x 256 MiB f32 -> 256 MiB, seeds 1 and 2."""
    n = 1 << 26
    g1 = torch.Generator(device="cuda").manual_seed(1)
    g2 = torch.Generator(device="cuda").manual_seed(2)
    a = torch.rand(n, device="cuda", generator=g1) * 2 - 1
    b = torch.rand(n, device="cuda", generator=g2) * 2 - 1
    d = torch.empty_like(a)
    nccl.reduce_copy(0, 7, 0, [a.data_ptr(), b.data_ptr()], [d.data_ptr()], n, stream_ptr())
    torch.cuda.synchronize()
    ref = a + b  # IEEE f32 add, same single rounding
    assert torch.equal(d.view(torch.int32), ref.view(torch.int32))


@pytest.mark.parametrize("offs", [(0, 0, 0), (0, 1, 0), (1, 1, 1), (0, 0, 1)],
                         ids=["aligned", "shifted_src1", "common_misalign", "element_dst"])
def test_beyond_2gib(offs):
    """Buffers past 2 GiB: every access policy (nt, write-through sc0 sc1 buffer
    stores, shifted-source realignment, element path) must address bytes beyond
    a 32-bit signed offset.  offs = f32-element offsets of (src0, src1, dst)."""
    n = (1 << 29) + 1037  # 2 GiB + 4148 B per buffer
    g = torch.Generator(device="cuda").manual_seed(7)
    bufs = []
    for o in offs:
        t = torch.empty(n + o, device="cuda")
        bufs.append(t[o:])
    a, b, d = bufs
    a.uniform_(-1, 1, generator=g)
    b.uniform_(-1, 1, generator=g)
    d.fill_(float("nan"))
    nccl.reduce_copy(0, 7, 0, [a.data_ptr(), b.data_ptr()], [d.data_ptr()], n, stream_ptr())
    torch.cuda.synchronize()
    ref = a + b
    assert torch.equal(d.view(torch.int32), ref.view(torch.int32))
    del a, b, d, ref, bufs
    torch.cuda.empty_cache()


def test_abi_errors():
    L = nccl.lib()
    import ctypes
    s = (ctypes.c_void_p * 1)(0x1000)
    d = (ctypes.c_void_p * 1)(0x2000)
    # SumPostDiv on float, copy on non-byte type, 0 / 9 sources
    assert L.vcclReduceCopy(4, 7, 0, 0, 0, 1, s, 1, d, 16, None) == nccl.ncclInvalidArgument
    assert L.vcclReduceCopy(15, 7, 0, 0, 0, 1, s, 1, d, 16, None) == nccl.ncclInvalidArgument
    assert L.vcclReduceCopy(0, 7, 0, 0, 0, 0, s, 1, d, 16, None) == nccl.ncclInvalidArgument
    assert L.vcclReduceCopy(0, 12, 0, 0, 0, 1, s, 1, d, 16, None) == nccl.ncclInvalidArgument
    # count 0 is a successful no-op even with bogus pointers
    assert L.vcclReduceCopy(0, 7, 0, 0, 0, 1, s, 1, d, 0, None) == nccl.ncclSuccess


@pytest.mark.parametrize("t", [10, 11])
def test_fp8_all_code_pairs(t):
    """Every (a, b) fp8 code pair through the device for sum/prod/min/max and
    the avg preOp: bit-exact to the oracle (NaN by NaN-ness, +-0 for min/max)."""
    codes = np.arange(256, dtype=np.uint8)
    a, b = np.repeat(codes, 256), np.tile(codes, 256)
    for op in (0, 1, 2, 3, 4):
        dev_op, arg, pre, post = _dev_args(op, t, 2)
        got = _run(dev_op, t, arg, [a, b], pre=pre, post=post)[0]
        exp = O.reduce_copy(dev_op, t, arg, [a, b], pre_op_args=[arg] * pre, post_op=post)[0]
        assert_bitexact(t, got, exp, minmax=op in (2, 3), what=f"fp8 t{t} op{op}")


# Destinations at DIFFERENT misalignments (the reference falls back to element
# packs, common_kernel.h:237-241): the body is aligned on destination 0 and
# every other destination is realigned by wavefront shuffle + funnel shift,
# with <= 4 partial stores at each wave's two ends.  Sizes straddle the wave
# (64 packs), hunk and grid boundaries; bytes around each destination must
# stay untouched.
DST_OFFSETS = {1: [(0, 1), (3, 0), (5, 13), (0, 15, 7)], 2: [(0, 2), (6, 0), (2, 14), (0, 8, 4)],
               4: [(0, 4), (12, 0), (4, 8), (0, 12, 4)], 8: [(0, 8), (8, 0), (8, 8, 0)]}


@pytest.mark.parametrize("t", [1, 6, 7, 8, 9, 10])
@pytest.mark.parametrize("op", [0, 2])
def test_destination_realignment(t, op):
    rng = np.random.default_rng(2000 + 10 * t + op)
    sz = np.dtype(O.NP_DTYPE[t]).itemsize
    for doffs in DST_OFFSETS[sz]:
        for soffs in ([0, 0], [sz, 0], [(3 * sz) % 16, (5 * sz) % 16]):
            for n in (1, 5, 63, 64 * 16 // sz + 3, 4097, 100_003, (1 << 20) + 9):
                srcs = [_rand(rng, t, n) for _ in range(2)]
                dev_op, arg, pre, post = _dev_args(op, t, 2)
                exp = O.reduce_copy(dev_op, t, arg, srcs, pre_op_args=[arg] * pre, post_op=post)[0]
                keep, sp = [], []
                for i, x in enumerate(srcs):
                    tt, ptr = to_dev(x, offset=soffs[i])
                    keep.append(tt)
                    sp.append(ptr)
                outs = [empty_dev(n * sz, offset=o) for o in doffs]
                nccl.reduce_copy(dev_op, t, arg, sp, [ptr for _, ptr in outs], n, stream_ptr(),
                                 pre_op_srcs=pre, post_op=post)
                torch.cuda.synchronize()
                for (tt, _), o in zip(outs, doffs):
                    got = from_dev(tt, O.NP_DTYPE[t], n, o)
                    assert_bitexact(t, got, exp, minmax=op == 2,
                                    what=f"t{t} op{op} n{n} srcs{soffs} dsts{doffs}")
                    raw = tt.cpu().numpy()
                    assert (raw[:o] == 0xA5).all() and (raw[o + n * sz:] == 0xA5).all(), \
                        f"guard bytes written t{t} n{n} dsts{doffs}"


def test_lds_staged_variant():
    """The north-star's LDS double-buffered staging (k_reduce_copy_lds,
    rc_kernels.hip: global_load_lds_dwordx4 two tiles deep, ds_read back) —
    a benchmark variant selected by launch config order 2 — must be
    bit-exact like the register path it lost to.  Sizes are
    whole 8 KiB tiles (the launcher falls back to the register path
    otherwise, which the ragged size checks)."""
    rng = np.random.default_rng(31)
    for n, grid, st in ((1 << 22, 256, 1), (1 << 22, 1024, 2), ((1 << 20) + 2048, 97, 1),
                        (1 << 20, 4096, 2), ((1 << 20) + 5, 256, 1)):
        a = rng.standard_normal(n).astype(np.float32)
        b = rng.standard_normal(n).astype(np.float32)
        cfg = {"blockSize": 256, "unroll": 2, "gridBlocks": grid, "ntLoads": 1, "ntStores": st,
               "order": 2}
        got = _run(0, 7, 0, [a, b], config=cfg)[0]
        assert np.array_equal(got.view(np.uint32), (a + b).view(np.uint32)), (n, grid, st)
