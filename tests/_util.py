"""Shared comparison rules for parity tests.

* integers: bit-exact;
* floats, same fold order: bit-exact, except NaN compares by NaN-ness and, for
  min/max only, +0 == -0 (CUDA fminf / v_min_f32 leave the zero sign open);
* floats, different fold order (multi-rank collectives): the tolerance stated
  in SURVEY.md §8c against the exact value —  sum: |y - exact| <=
  (n-1)*u*sum|x_i| + ulp(y)/2, prod: <= ((1+u)^(n-1) - 1)*|exact| + ulp(y)/2 —
  and twice the fold term against another order's computed result (VCCL's).
"""
import numpy as np

TYPE_IDS = {"i8": 0, "u8": 1, "i32": 2, "u32": 3, "i64": 4, "u64": 5,
            "f16": 6, "f32": 7, "f64": 8, "bf16": 9,
            "f8e4m3": 10, "f8e5m2": 11}
OP_IDS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}
FLOAT_TYPES = (6, 7, 8, 9, 10, 11)
UNIT_ROUNDOFF = {6: 2.0**-11, 7: 2.0**-24, 8: 2.0**-53, 9: 2.0**-8, 10: 2.0**-4, 11: 2.0**-3}


def to_f64(t, a):
    a = np.asarray(a)
    if t == 9:
        return (a.astype(np.uint16).astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    if t in (10, 11):
        from oracle import oracle as O
        return O.fp8_bits_to_f32(t, a).astype(np.float64)
    return a.astype(np.float64)


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[a.dtype.itemsize])


def assert_bitexact(t, got, exp, minmax=False, what=""):
    got, exp = np.asarray(got), np.asarray(exp)
    assert got.shape == exp.shape, (got.shape, exp.shape)
    gb, eb = bits(got), bits(exp)
    if t not in FLOAT_TYPES:
        bad = np.nonzero(gb != eb)[0]
        assert bad.size == 0, f"{what}: {bad.size} mismatches, first at {bad[:5]}: got {got[bad[:5]]} exp {exp[bad[:5]]}"
        return
    gf, ef = to_f64(t, got), to_f64(t, exp)
    same = gb == eb
    same |= np.isnan(gf) & np.isnan(ef)
    if minmax:
        same |= (gf == 0) & (ef == 0)
    bad = np.nonzero(~same)[0]
    assert bad.size == 0, f"{what}: {bad.size} mismatches, first at {bad[:5]}: got {gf[bad[:5]]} exp {ef[bad[:5]]}"


def exact_f64(t, op, inputs):
    """The exactly rounded-once reference in f64 of a sum / prod of n inputs
    (exact for sums of <= 8 values of <= 24-bit significands; products carry
    a negligible ~n * 2^-53 relative error)."""
    xs = np.stack([to_f64(t, x) for x in inputs])
    return xs.prod(axis=0) if op == 1 else xs.sum(axis=0)


def assert_fold_tolerance(t, op, got, exp, inputs, what="", exp_is_exact=False):
    """Order-independent check for multi-rank fp sum/prod.

    Against the exact value (exp_is_exact=True, exp in f64): any fold order of
    n inputs lands within the forward-error bound
        sum:  |y - exact| <= (n-1) u sum|x_i| + ulp(y)/2
        prod: |y - exact| <= ((1+u)^(n-1) - 1) |exact| + ulp(y)/2.
    Against another fold order's computed result (e.g. VCCL's schedule on the
    same inputs; exp in the storage type): both sit within that bound of the
    exact value, so the allowed difference is twice the fold term."""
    if t not in FLOAT_TYPES or op in (2, 3):
        assert_bitexact(t, got, exp, minmax=op in (2, 3), what=what)
        return
    n = len(inputs)
    u = UNIT_ROUNDOFF[t]
    g = to_f64(t, got)
    e = np.asarray(exp, dtype=np.float64) if exp_is_exact else to_f64(t, exp)
    xs = np.stack([to_f64(t, x) for x in inputs])
    finite = np.isfinite(e) & np.isfinite(g)
    if op == 1:
        bound = ((1 + u) ** (n - 1) - 1) * np.abs(e)
    else:
        bound = (n - 1) * u * np.abs(xs).sum(axis=0)
    if not exp_is_exact:
        bound = 2 * bound
    bound = bound + np.maximum(np.abs(e), np.abs(g)) * u + 1e-300
    ok = ~finite | (np.abs(g - e) <= bound)
    ok &= ~(np.isnan(g) ^ np.isnan(e))
    bad = np.nonzero(~ok)[0]
    assert bad.size == 0, f"{what}: {bad.size} out of tolerance, first {bad[:5]}: got {g[bad[:5]]} exp {e[bad[:5]]}"


def golden_rc_cases(golden):
    """Yield (key, type_id, op_id, nsrc, inputs[nsrc], expected) from the npz."""
    for k in golden.files:
        if not (k.startswith("rc_") and k.endswith("_in")):
            continue
        _, tname, oname, nsrc = k[:-3].split("_")
        yield (k[:-3], TYPE_IDS[tname], OP_IDS[oname], int(nsrc), golden[k],
               golden[k[:-3] + "_out"])
