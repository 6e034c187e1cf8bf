"""ORACLE — test infrastructure only.

ctypes + numpy wrapper over ``oracle/build/liboracle.so`` (the C restatement of
VCCL's reduction semantics, see ``reduce_ref.h``).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module; the product path (``vccl_amd``) never does.

Parity status: dispatch table pinned by the reference's ``generate.py``; the
arithmetic is pinned to the reference's own fallback expressions (widen, one
binary32 op, RN-even narrowing; reduce_kernel.h:276-296) evaluated by numpy /
torch IEEE implementations — no reference-produced fixture exists (CUDA's
fp16/bf16 intrinsic headers are not in /root/reference); see DESIGN.md §2.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")

# ncclDataType_t (nccl.h.in:239-252) -> numpy storage dtype
NP_DTYPE = {
    0: np.int8, 1: np.uint8, 2: np.int32, 3: np.uint32, 4: np.int64, 5: np.uint64,
    6: np.float16, 7: np.float32, 8: np.float64, 9: np.uint16,  # bf16 stored as raw bits
    10: np.uint8, 11: np.uint8,  # fp8 e4m3 / e5m2 stored as raw bits
}
TYPE_NAMES = {0: "i8", 1: "u8", 2: "i32", 3: "u32", 4: "i64", 5: "u64",
              6: "f16", 7: "f32", 8: "f64", 9: "bf16",
              10: "f8e4m3", 11: "f8e5m2"}
OP_NAMES = {0: "sum", 1: "prod", 2: "max", 3: "min", 4: "avg"}
DEV_SUM, DEV_PROD, DEV_MINMAX, DEV_PREMULSUM, DEV_SUMPOSTDIV = range(5)

_lib = None


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u64, i32, vp = ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p
        L.ref_host_to_dev_redop.argtypes = [i32, i32, i32, ctypes.POINTER(i32), ctypes.POINTER(u64)]
        L.ref_reduce_copy.argtypes = [i32, i32, u64, ctypes.POINTER(u64), i32, i32, i32,
                                      ctypes.POINTER(vp), i32, ctypes.POINTER(vp), ctypes.c_size_t, i32]
        L.ref_ring_fold.argtypes = [i32, i32, u64, i32, i32, ctypes.POINTER(vp),
                                    vp, vp, ctypes.c_size_t]
        L.ref_chain_fold.argtypes = [i32, i32, u64, i32, i32, ctypes.POINTER(vp), vp, ctypes.c_size_t]
        L.ref_f32_to_f16.restype = ctypes.c_uint16
        L.ref_f32_to_f16.argtypes = [ctypes.c_float]
        L.ref_f32_to_bf16.restype = ctypes.c_uint16
        L.ref_f32_to_bf16.argtypes = [ctypes.c_float]
        L.ref_fp8_to_f32.restype = ctypes.c_float
        L.ref_fp8_to_f32.argtypes = [i32, ctypes.c_uint8]
        L.ref_f32_to_fp8.restype = ctypes.c_uint8
        L.ref_f32_to_fp8.argtypes = [i32, ctypes.c_float]
        _lib = L
    return _lib


def _bind_cpu_bench(L):
    sz, i32, vp, dbl = ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_double
    L.ref_cpu_bench_alloc.argtypes = [sz, i32, ctypes.POINTER(i32), ctypes.POINTER(vp),
                                      ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.ref_cpu_bench_run.argtypes = [vp, vp, vp, sz, i32, ctypes.POINTER(i32), dbl,
                                    ctypes.POINTER(ctypes.c_long), ctypes.POINTER(dbl)]
    L.ref_cpu_bench_free.argtypes = [vp, vp, vp, sz]
    L.ref_cpu_bench_rank_alloc.argtypes = [sz, i32, sz, i32, i32, ctypes.POINTER(i32), ctypes.POINTER(vp)]
    L.ref_cpu_bench_rank_run.argtypes = [ctypes.POINTER(vp), sz, i32, sz, i32, i32, ctypes.POINTER(i32), dbl,
                                         ctypes.POINTER(ctypes.c_long), ctypes.POINTER(dbl)]
    L.ref_cpu_bench_rank_free.argtypes = [ctypes.POINTER(vp), sz, i32, sz, i32]
    L.ref_reduce_copy.argtypes = [i32, i32, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), i32,
                                  i32, i32, ctypes.POINTER(vp), i32, ctypes.POINTER(vp), sz, i32]
    return L


_native = None


def native_lib(outdir: str | None = None):
    """The oracle's reduce_ref.c + cpu_bench.c compiled for THIS host
    (-O3 -march=native, same IEEE flags as the checker build) into a scratch
    directory — the CPU baseline's build; falls back to the
    portable checker build (-march=x86-64-v3) when no compiler is present.
    Returns (CDLL, march)."""
    global _native
    if _native is None:
        import tempfile
        d = outdir or tempfile.mkdtemp(prefix="vccl_cpu_native_")
        so = os.path.join(d, "liboracle_native.so")
        cmd = ["gcc", "-O3", "-march=native", "-fno-fast-math", "-ffp-contract=off", "-fPIC",
               "-std=gnu11", "-shared", "-o", so, os.path.join(_HERE, "reduce_ref.c"),
               os.path.join(_HERE, "cpu_bench.c"), "-lpthread", "-lm"]
        try:
            subprocess.run(cmd, check=True, capture_output=True, timeout=120)
            _native = (_bind_cpu_bench(ctypes.CDLL(so)), "native")
        except (OSError, subprocess.SubprocessError):
            _native = (_bind_cpu_bench(lib()), "x86-64-v3")
    return _native


def cpu_bench(n: int, cpus, seconds: float, register=None, native: bool = True) -> dict:
    """f32 d = a + b over n elements on len(cpus) persistent workers pinned to
    `cpus` (first-touched slices, see cpu_bench.c); `register(ptr, bytes)` /
    its returned undo callable may pin the pages for the device
    (hipHostRegister) between the first touch and the timed loop.  Returns
    GB/s (3 x 4 n bytes per pass), passes, seconds, and the bit-exact check."""
    L, march = native_lib() if native else (_bind_cpu_bench(lib()), "x86-64-v3")
    nt = len(cpus)
    cp = (ctypes.c_int * nt)(*cpus)
    a, b, d = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    if L.ref_cpu_bench_alloc(n, nt, cp, ctypes.byref(a), ctypes.byref(b), ctypes.byref(d)) != 0:
        raise MemoryError("cpu bench allocation")
    undo = []
    try:
        if register is not None:
            for p in (a, b, d):
                undo.append(register(p.value, n * 4))
        iters, el = ctypes.c_long(), ctypes.c_double()
        ok = L.ref_cpu_bench_run(a, b, d, n, nt, cp, seconds, ctypes.byref(iters), ctypes.byref(el))
    finally:
        for u in undo:
            if u:
                u()
        L.ref_cpu_bench_free(a, b, d, n)
    return {"GB/s": round(3 * n * 4 * iters.value / el.value / 1e9, 2), "threads": nt,
            "iters": iters.value, "s": round(el.value, 2), "correct": bool(ok), "march": march,
            "pinned": register is not None and all(undo)}


def cpu_bench_rank(m: int, nsrc: int, ncopy: int, cpus, seconds: float, register=None,
                   native: bool = True, dtype: int = 7) -> dict:
    """One rank's share of an nsrc-rank ring all-reduce as host work (see
    cpu_bench.c): an nsrc-source sum of `dtype` (f32 7, f16 6, bf16 9) over m
    elements into one shard, then a copy of ncopy elements, on len(cpus)
    pinned persistent workers, each pass checked bit-exactly at the end.
    Returns the seconds per pass, the memory rate ((nsrc + 1) m + 2 ncopy)
    elements per pass, and the check."""
    L, march = native_lib() if native else (_bind_cpu_bench(lib()), "x86-64-v3")
    esz = np.dtype(NP_DTYPE[dtype]).itemsize
    nt = len(cpus)
    cp = (ctypes.c_int * nt)(*cpus)
    bufs = (ctypes.c_void_p * (nsrc + 3))()
    if L.ref_cpu_bench_rank_alloc(m, nsrc, ncopy, dtype, nt, cp, bufs) != 0:
        raise MemoryError("cpu bench allocation")
    undo = []
    try:
        if register is not None:
            for i in range(nsrc + 3):
                if bufs[i]:
                    undo.append(register(bufs[i], (m if i <= nsrc else ncopy) * esz))
        iters, el = ctypes.c_long(), ctypes.c_double()
        ok = L.ref_cpu_bench_rank_run(bufs, m, nsrc, ncopy, dtype, nt, cp, seconds, ctypes.byref(iters),
                                      ctypes.byref(el))
    finally:
        for u in undo:
            if u:
                u()
        L.ref_cpu_bench_rank_free(bufs, m, nsrc, ncopy, dtype)
    per_pass = el.value / max(1, iters.value)
    return {"s_per_pass": per_pass, "mem_GB/s": round(((nsrc + 1) * m + 2 * ncopy) * esz / per_pass / 1e9, 2),
            "threads": nt, "iters": iters.value, "s": round(el.value, 2), "correct": bool(ok),
            "march": march, "pinned": register is not None and bool(undo) and all(undo)}


def host_to_dev_redop(op: int, dtype: int, nranks: int) -> tuple[int, int]:
    d, a = ctypes.c_int(), ctypes.c_uint64()
    rc = lib().ref_host_to_dev_redop(op, dtype, nranks, ctypes.byref(d), ctypes.byref(a))
    if rc != 0:
        raise ValueError(f"invalid op/type {op}/{dtype}")
    return d.value, a.value


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def reduce_copy(dev_op, dtype, red_arg, srcs, n_dsts=1, pre_op_args=(), post_op=False,
                nthreads=1, out=None):
    """dst = postOp(preOp(src0) (+) preOp(src1) (+) ...) elementwise."""
    srcs = [np.ascontiguousarray(s) for s in srcs]
    n = srcs[0].size
    if out is None:
        out = [np.empty_like(srcs[0]) for _ in range(n_dsts)]
    pre = (ctypes.c_uint64 * max(1, len(pre_op_args)))(*pre_op_args) if pre_op_args else None
    lib().ref_reduce_copy(dev_op, dtype, red_arg, pre, len(pre_op_args), int(post_op),
                          len(srcs), _ptrs(srcs), len(out), _ptrs(out), n, nthreads)
    return out


def ring_fold(dev_op, dtype, red_arg, pre_op, inputs_ring_order, owner):
    inputs = [np.ascontiguousarray(x) for x in inputs_ring_order]
    owner = np.ascontiguousarray(owner, dtype=np.int32)
    out = np.empty_like(inputs[0])
    lib().ref_ring_fold(dev_op, dtype, red_arg, int(pre_op), len(inputs), _ptrs(inputs),
                        owner.ctypes.data, out.ctypes.data, out.size)
    return out


def chain_fold(dev_op, dtype, red_arg, pre_op, inputs_chain_order):
    inputs = [np.ascontiguousarray(x) for x in inputs_chain_order]
    out = np.empty_like(inputs[0])
    lib().ref_chain_fold(dev_op, dtype, red_arg, int(pre_op), len(inputs), _ptrs(inputs),
                         out.ctypes.data, out.size)
    return out


def allreduce(op, dtype, inputs, owner_fn=None):
    """Full API-level all-reduce semantics: hostToDevRedOp + ring fold.

    ``inputs`` are per-rank arrays indexed by rank; ``owner_fn(n_elems)`` gives
    for each element the ring index that finishes it (ring = identity order
    unless the caller permutes ``inputs``)."""
    n = len(inputs)
    dev_op, arg = host_to_dev_redop(op, dtype, n)
    owner = owner_fn(inputs[0].size) if owner_fn else np.zeros(inputs[0].size, np.int32)
    if n == 1:  # ncclLaunchOneRank (onerank.cu:47-83): copy, or PreMulSum kernel
        x = inputs[0]
        if dev_op == DEV_PREMULSUM:
            return reduce_copy(dev_op, dtype, arg, [x], pre_op_args=[arg], post_op=True)[0]
        return x.copy()
    return ring_fold(dev_op, dtype, arg, dev_op == DEV_PREMULSUM, inputs, owner)


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """Vectorised RN-even f32 -> bf16 bits (NaN kept NaN), matches ref_f32_to_bf16."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.ascontiguousarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


_FP8_TABLES = {}


def fp8_bits_to_f32(t: int, b: np.ndarray) -> np.ndarray:
    """Exact fp8 (type 10 e4m3 / 11 e5m2) -> f32 through ref_fp8_to_f32."""
    if t not in _FP8_TABLES:
        _FP8_TABLES[t] = np.array([lib().ref_fp8_to_f32(t, i) for i in range(256)], np.float32)
    return _FP8_TABLES[t][np.asarray(b, dtype=np.uint8)]


def f32_to_fp8_bits(t: int, x: np.ndarray) -> np.ndarray:
    """RN-even satfinite f32 -> fp8 bits (ref_f32_to_fp8), element by element."""
    L = lib()
    x = np.asarray(x, dtype=np.float32).ravel()
    return np.array([L.ref_f32_to_fp8(t, float(v)) for v in x], dtype=np.uint8)
