"""Pin the CPU oracle (oracle/reduce_ref.c) before trusting it.

* against the independent golden vectors (numpy / torch-CPU IEEE semantics);
* against the reference's own generate.py dispatch table (functable.json);
* f16 / bf16 conversion exhaustively against numpy / torch.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests._util import (FLOAT_TYPES, assert_bitexact, golden_rc_cases)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _api_to_dev(op, t, n):
    dev_op, arg = O.host_to_dev_redop(op, t, n)
    pre = [arg] * n if dev_op == O.DEV_PREMULSUM else []
    return dev_op, arg, pre, dev_op == O.DEV_SUMPOSTDIV


def test_oracle_matches_golden_reduce_copy(golden):
    n_cases = 0
    for key, t, op, nsrc, inp, exp in golden_rc_cases(golden):
        dev_op, arg, pre, post = _api_to_dev(op, t, nsrc)
        srcs = [inp[i] for i in range(nsrc)]
        got = O.reduce_copy(dev_op, t, arg, srcs, pre_op_args=pre, post_op=post)[0]
        assert_bitexact(t, got, exp, minmax=op in (2, 3), what=key)
        n_cases += 1
    assert n_cases == 10 * 5 * 3


def test_oracle_ring_fold_matches_golden(golden):
    for k in golden.files:
        if not (k.startswith("ring_") and k.endswith("_in")):
            continue
        base = k[:-3]
        t = {"f32": 7, "f16": 6, "bf16": 9}[base.split("_")[1]]
        inp, owner, exp = golden[k], golden[base + "_owner"], golden[base + "_out"]
        got = O.ring_fold(O.DEV_SUM, t, 0, False, [inp[i] for i in range(inp.shape[0])], owner)
        assert_bitexact(t, got, exp, what=base)


def test_oracle_threads_agree():
    rng = np.random.default_rng(1)
    a = rng.standard_normal(100_003).astype(np.float32)
    b = rng.standard_normal(100_003).astype(np.float32)
    one = O.reduce_copy(O.DEV_SUM, 7, 0, [a, b], nthreads=1)[0]
    many = O.reduce_copy(O.DEV_SUM, 7, 0, [a, b], nthreads=7)[0]
    assert np.array_equal(one.view(np.uint32), many.view(np.uint32))
    assert np.array_equal(one, a + b)


def test_f16_conversion_exhaustive():
    L = O.lib()
    bits = np.arange(0, 1 << 16, dtype=np.uint32).astype(np.uint16)
    f = bits.view(np.float16).astype(np.float32)
    # f16 -> f32 -> f16 round trip is the identity (NaNs stay NaN)
    rt = np.array([L.ref_f32_to_f16(float(x)) for x in f[::7]], dtype=np.uint16)
    src = bits[::7]
    nan = np.isnan(f[::7])
    assert np.array_equal(rt[~nan], src[~nan])
    assert np.all(np.isnan(rt[nan].view(np.float16)))
    # f32 -> f16 rounding against numpy on random + boundary values
    rng = np.random.default_rng(2)
    xs = np.concatenate([rng.standard_normal(4000).astype(np.float32) * 10.0 ** rng.integers(-9, 6, 4000),
                         np.float32([65504, 65519.99, 65520, 6.1035156e-05, 5.96e-08, 2.98e-08,
                                     2.99e-08, 1e-30, -0.0])]).astype(np.float32)
    ours = np.array([L.ref_f32_to_f16(float(x)) for x in xs], dtype=np.uint16)
    assert np.array_equal(ours, xs.astype(np.float16).view(np.uint16))


def test_bf16_conversion_against_torch():
    L = O.lib()
    rng = np.random.default_rng(3)
    xs = np.concatenate([rng.standard_normal(4000).astype(np.float32) * 10.0 ** rng.integers(-30, 30, 4000),
                         np.float32([3.3895e38, 3.4e38, 1e-40, -0.0, np.inf])]).astype(np.float32)
    ours = np.array([L.ref_f32_to_bf16(float(x)) for x in xs], dtype=np.uint16)
    ref = torch.from_numpy(xs).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    assert np.array_equal(ours, ref)
    assert np.array_equal(O.f32_to_bf16_bits(xs), ref)


def test_host_to_dev_redop_encoding():
    # enqueue.cc:2240-2256 — xormask for min/max
    assert O.host_to_dev_redop(3, 2, 4) == (2, 0x80000000)        # min i32
    assert O.host_to_dev_redop(2, 2, 4) == (2, 0x7FFFFFFF)        # max i32
    assert O.host_to_dev_redop(3, 3, 4) == (2, 0)                 # min u32
    assert O.host_to_dev_redop(2, 5, 4) == (2, 0xFFFFFFFFFFFFFFFF)  # max u64
    assert O.host_to_dev_redop(2, 7, 4) == (2, 0xFFFFFFFF)        # max f32: bit0 = 1
    assert O.host_to_dev_redop(3, 9, 4) == (2, 0)                 # min bf16
    # avg: ints SumPostDiv nRanks<<1|signed, floats PreMulSum 1/n bits
    assert O.host_to_dev_redop(4, 0, 8) == (4, (8 << 1) | 1)
    assert O.host_to_dev_redop(4, 5, 3) == (4, 3 << 1)
    assert O.host_to_dev_redop(4, 7, 4) == (3, int(np.float32(0.25).view(np.uint32)))
    assert O.host_to_dev_redop(4, 6, 3) == (3, int(np.float16(1 / 3).view(np.uint16)))


def test_functable_signed_maps_to_unsigned():
    """Reference generate.py (run unmodified, tests/golden/gen_functable.py):
    rows sharing a primary id run one kernel.  Our dispatch
    (vcclKernelTypeOf, vccl_amd/csrc/device/dispatch.hpp) maps (devOp, type)
    to a kernel element type; two rows share a reference id iff they share
    our kernel type, and a row the reference does not build (id -1) is
    rejected by ours (-1).  Loads libvccl.so; makes no GPU call."""
    from vccl_amd import nccl
    table = json.load(open(os.path.join(ROOT, "tests", "golden", "functable.json")))
    devop = {"Sum": 0, "Prod": 1, "MinMax": 2, "PreMulSum": 3, "SumPostDiv": 4}
    tyid = {"i8": 0, "u8": 1, "i32": 2, "u32": 3, "i64": 4, "u64": 5, "f16": 6, "f32": 7,
            "f64": 8, "bf16": 9, "f8e4m3": 10, "f8e5m2": 11}
    by_key = {}
    for r in table["rows"]:
        if r["coll"] == "AllGather":
            continue
        by_key.setdefault((r["coll"], r["redop"], r["algo"], r["proto"]), []).append(r)
    kt = lambda r: nccl.kernel_type_of(devop[r["redop"]], tyid[r["type"]])  # noqa: E731
    checked = 0
    for rows in by_key.values():
        for r1 in rows:
            assert (kt(r1) >= 0) == (r1["id"] != -1), r1
            for r2 in rows:
                if r1["id"] == -1 or r2["id"] == -1:
                    continue
                assert (r1["id"] == r2["id"]) == (kt(r1) == kt(r2)), (r1, r2)
                checked += 1
    assert checked > 500


def test_oracle_chain_fold_order():
    """Chain-tree LL fold (all_reduce.h:148-229, prims_ll.h:258-266):
    x_0 (+) (x_1 (+) (... (+) x_{n-1})) with peer (+) own at every hop —
    restated with numpy's IEEE f32/f16 adds, element by element."""
    rng = np.random.default_rng(9)
    for dt, npdt in ((7, np.float32), (6, np.float16)):
        for n in (2, 3, 8):
            xs = [rng.uniform(-1, 1, 777).astype(npdt) for _ in range(n)]
            exp = xs[n - 1].copy()
            for p in range(n - 2, -1, -1):
                exp = (exp + xs[p]).astype(npdt)
            got = O.chain_fold(O.DEV_SUM, dt, 0, False, xs)
            assert np.array_equal(got.view(np.uint8), exp.view(np.uint8)), (dt, n)


def test_reduce_expectation_fold_order():
    """The ring reduce's expected output (tests/_ring.py expected_reduce,
    reduce.h:12-55) restated element by element with numpy's IEEE f32 adds:
    on one channel of ring R the chunk starts at root's successor, every
    next rank computes own + received, and the root ends with own + received
    — x_root + (x_{R[i-1]} + (... + x_{R[i+1]})) for root = R[i]."""
    from tests import _ring
    rng = np.random.default_rng(13)
    for n in (2, 3, 4, 5):
        xs = [rng.uniform(-1, 1, 1001).astype(np.float32) for _ in range(n)]
        ring = _ring.ring_orders(n)[0]
        for root in range(n):
            i = ring.index(root)
            acc = xs[ring[(i + 1) % n]].copy()
            for k in range(2, n + 1):
                acc = (xs[ring[(i + k) % n]] + acc).astype(np.float32)
            got = _ring.expected_reduce(0, 7, xs, root, 1)
            assert np.array_equal(got.view(np.uint8), acc.view(np.uint8)), (n, root)


# ---------------------------------------------------------------- fp8
# The reference reduces fp8 through __half (reduce_kernel.h:309-321) with
# CUDA's cuda_fp8.h conversions (absent here).  The oracle's conversions and
# its two-rounding arithmetic are pinned against torch-CPU's independent
# float8_e4m3fn / float8_e5m2 implementation (RN-even; torch does NOT saturate,
# so out-of-range results are checked against the satfinite rule separately).
FP8_TORCH = {10: torch.float8_e4m3fn, 11: torch.float8_e5m2}
FP8_MAX = {10: 448.0, 11: 57344.0}


@pytest.mark.parametrize("t", [10, 11])
def test_fp8_decode_all_codes_against_torch(t):
    codes = np.arange(256, dtype=np.uint8)
    ours = O.fp8_bits_to_f32(t, codes)
    ref = torch.from_numpy(codes).view(FP8_TORCH[t]).float().numpy()
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(ours), nan)
    assert np.array_equal(ours[~nan].view(np.uint32), ref[~nan].view(np.uint32))


@pytest.mark.parametrize("t", [10, 11])
def test_fp8_encode_every_half_against_torch(t):
    L = O.lib()
    h = np.arange(0, 1 << 16, dtype=np.uint32).astype(np.uint16).view(np.float16).astype(np.float32)
    ours = np.array([L.ref_f32_to_fp8(t, float(x)) for x in h], dtype=np.uint8)
    ref = torch.from_numpy(h).to(FP8_TORCH[t]).view(torch.uint8).numpy()
    fin = np.isfinite(h) & (np.abs(h) <= FP8_MAX[t])
    assert np.array_equal(ours[fin], ref[fin])
    big = np.isfinite(h) & (np.abs(h) > FP8_MAX[t]) | np.isinf(h)  # satfinite: +-max
    maxcode = 0x7E if t == 10 else 0x7B
    assert np.array_equal(ours[big], np.where(h[big] < 0, 0x80 | maxcode, maxcode).astype(np.uint8))
    assert np.all(ours[np.isnan(h)] == 0x7F)


@pytest.mark.parametrize("t", [10, 11])
@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_fp8_all_pairs_against_torch_half(t, op):
    """Every (a, b) code pair: oracle == fp8(half(a) (op) half(b)) computed
    with torch half arithmetic and torch's fp8 narrowing (+ satfinite)."""
    codes = np.arange(256, dtype=np.uint8)
    a = np.repeat(codes, 256)
    b = np.tile(codes, 256)
    dev_op, arg = O.host_to_dev_redop(op, t, 2)
    ours = O.reduce_copy(dev_op, t, arg, [a, b])[0]
    ta = torch.from_numpy(a).view(FP8_TORCH[t]).half()
    tb = torch.from_numpy(b).view(FP8_TORCH[t]).half()
    r = {0: ta + tb, 1: ta * tb, 2: torch.fmax(ta, tb), 3: torch.fmin(ta, tb)}[op].float()
    rn = r.numpy()
    ref = r.to(FP8_TORCH[t]).view(torch.uint8).numpy()
    fin = np.isfinite(rn) & (np.abs(rn) <= FP8_MAX[t])
    assert np.array_equal(ours[fin], ref[fin]) or (op in (2, 3) and np.array_equal(
        O.fp8_bits_to_f32(t, ours[fin]), O.fp8_bits_to_f32(t, ref[fin])))
    maxcode = 0x7E if t == 10 else 0x7B
    big = ~np.isnan(rn) & ~fin
    assert np.array_equal(ours[big], np.where(rn[big] < 0, 0x80 | maxcode, maxcode).astype(np.uint8))
    assert np.all(ours[np.isnan(rn)] == 0x7F)


def test_fp8_avg_scalar_encoding():
    # enqueue.cc:2265-2272: __nv_cvt_float_to_fp8(float(1.0/n), SATFINITE, fmt)
    for t in (10, 11):
        for n in (2, 3, 5, 7, 8):
            dev_op, arg = O.host_to_dev_redop(4, t, n)
            ref = torch.tensor([1.0 / n], dtype=torch.float32).to(FP8_TORCH[t]).view(torch.uint8).item()
            assert (dev_op, arg) == (3, ref)


# ---- the reference's two arithmetic branches agree ----------
# reduce_kernel.h computes f16 / bf16 sums and products either with the
# intrinsics (__hadd / __hmul: correctly rounded) or, on older architectures,
# as widen -> one binary32 op -> RN-even narrowing (:276-277, :294-296) — what
# the golden vectors and the oracle compute.  The two agree because double
# rounding through binary32 is innocuous for binary16 and bfloat16 (p' = 24 >=
# 2p + 2).  Checked here on every finite f16 / bf16 value against a spread of
# partners (subnormals, large exponent gaps, cancellation) and random pairs.
def _partners(vals, rng, k):
    fin = vals[np.isfinite(vals.astype(np.float64))]
    return np.concatenate([fin[rng.integers(0, fin.size, k - 8)],
                           np.array([0.0, -0.0, 1.0, -1.0, 65504.0, -65504.0, 6e-8, -6e-8],
                                    dtype=vals.dtype)])


def _rn_f16_from_f64(x):
    return x.astype(np.float16)  # numpy's double -> half conversion rounds once (RN-even)


def _round_to_odd_f32(x):
    """binary64 -> binary32 rounding to odd (exact, or the truncation with its
    last bit set): a following RN-even rounding to bf16 is then the correct
    rounding of x (24 >= 8 + 2)."""
    y = x.astype(np.float32)
    inexact = y.astype(np.float64) != x
    over = inexact & (np.abs(y.astype(np.float64)) > np.abs(x))
    y = np.where(over, np.nextafter(y, np.float32(0)), y)
    bits = y.view(np.uint32) | inexact.astype(np.uint32)
    return bits.view(np.float32)


def test_f16_fallback_equals_correct_rounding():
    rng = np.random.default_rng(77)
    allh = np.arange(1 << 16, dtype=np.uint16).view(np.float16)
    allh = allh[np.isfinite(allh)]
    b = _partners(allh, rng, 48)
    A = np.repeat(allh, b.size)
    B = np.tile(b, allh.size)
    with np.errstate(over="ignore", invalid="ignore"):
        for op in (np.add, np.multiply):
            fallback = op(A.astype(np.float32), B.astype(np.float32)).astype(np.float16)
            exact = _rn_f16_from_f64(op(A.astype(np.float64), B.astype(np.float64)))  # exact in binary64
            assert np.array_equal(fallback.view(np.uint16), exact.view(np.uint16)), op


def test_bf16_fallback_equals_correct_rounding():
    rng = np.random.default_rng(78)
    allb = torch.arange(1 << 16, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    allb = allb[torch.isfinite(allb)]
    vals = allb.float().numpy()
    idx = rng.integers(0, vals.size, 40)
    b = np.concatenate([vals[idx], np.array([0.0, -0.0, 1.0, -1.0, 1e-38, -1e-38, 3e38, -3e38], np.float32)])
    A = np.repeat(vals, b.size).astype(np.float64)
    B = np.tile(b, vals.size).astype(np.float64)
    with np.errstate(over="ignore", invalid="ignore"):
        for op in (np.add, np.multiply):
            fallback = torch.from_numpy(op(A.astype(np.float32), B.astype(np.float32))).to(torch.bfloat16)
            # binary64 holds the product exactly and the sum to 53 bits (> 2*8 + 2)
            exact = torch.from_numpy(_round_to_odd_f32(op(A, B))).to(torch.bfloat16)
            assert torch.equal(fallback.view(torch.int16), exact.view(torch.int16)), op
