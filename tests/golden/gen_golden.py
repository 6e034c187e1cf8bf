#!/usr/bin/env python3
"""Generate tests/golden/reduce_golden.npz — independent known-answer vectors.

The reference ships no tests or golden vectors and its
arithmetic lives in CUDA headers that are absent here, so the expected outputs
are computed by INDEPENDENT IEEE-754 implementations, never by our oracle:
  * integers, f16, f32, f64: numpy (wrap-around ints, np.fmin/np.fmax = minNum)
  * bf16: torch CPU bfloat16 (fp32 op + RN-even rounding, as __hadd/__hmul)
Semantics restated from reduce_kernel.h:174-323 (ops), :410-688 (PreMulSum,
SumPostDiv), common_kernel.h:84-152 (fold order: acc = preOp(src0); acc =
acc (+) src_s), enqueue.cc:2217-2310 (op encoding), all_reduce.h:42-64 (ring
fold order).

Each case: inputs (nsrc arrays of N elements) + expected output.
Run:  python tests/golden/gen_golden.py   (deterministic; seeds fixed)
"""
import os

import numpy as np
import torch

N = 515  # odd: exercises the 16-byte pack tail on every type
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reduce_golden.npz")

TYPES = {0: "i8", 1: "u8", 2: "i32", 3: "u32", 4: "i64", 5: "u64",
         6: "f16", 7: "f32", 8: "f64", 9: "bf16"}
INT_NP = {0: np.int8, 1: np.uint8, 2: np.int32, 3: np.uint32, 4: np.int64, 5: np.uint64}
FLT_NP = {6: np.float16, 7: np.float32, 8: np.float64}
OPS = {0: "sum", 1: "prod", 2: "max", 3: "min", 4: "avg"}


def gen_inputs(rng, t, nsrc):
    if t in INT_NP:
        dt = np.dtype(INT_NP[t])
        info = np.iinfo(dt)
        arrs = []
        for _ in range(nsrc):
            raw = rng.integers(0, np.iinfo(np.uint64).max, size=N, dtype=np.uint64, endpoint=True)
            a = raw.astype(np.uint64).view(np.int64).astype(dt) if dt.itemsize < 8 else raw.view(dt)
            a = np.array(a, dtype=dt)
            a[:6] = [info.min, info.max, 0, 1, info.max // 2, info.min // 2 if info.min else 7]
            arrs.append(a)
        return arrs
    arrs = []
    for _ in range(nsrc):
        f = rng.uniform(-1.0, 1.0, size=N).astype(np.float64)
        f[rng.integers(0, N, 40)] *= 1e4  # some larger magnitudes
        spec = [0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40, -3e-39, 6e-8, 1e-300, 65504.0,
                3.0e38, -3.0e38, 1.0, -1.0]
        k = int(rng.integers(0, len(spec)))
        spec = spec[k:] + spec[:k]  # rotate so sources differ at each special slot
        f[:len(spec)] = spec
        if t == 9:
            arrs.append(torch.tensor(f, dtype=torch.float32).to(torch.bfloat16))
        else:
            arrs.append(f.astype(FLT_NP[t]))
    return arrs


def fold(t, op, srcs):
    """Expected output for an nsrc-way reduce-copy (left fold)."""
    n = len(srcs)
    if t in INT_NP:
        dt = np.dtype(INT_NP[t])
        with np.errstate(over="ignore"):
            if op in (0, 4):
                acc = srcs[0].copy()
                for s in srcs[1:]:
                    acc = (acc + s).astype(dt)
                if op == 4:  # SumPostDiv: truncate toward zero
                    acc = np.array([int(x) for x in acc.tolist()], dtype=object)
                    acc = np.array([(abs(x) // n) * (1 if x >= 0 else -1) for x in acc],
                                   dtype=dt)
                return acc
            if op == 1:
                acc = srcs[0].copy()
                for s in srcs[1:]:
                    acc = (acc * s).astype(dt)
                return acc
            f = np.maximum if op == 2 else np.minimum
            acc = srcs[0].copy()
            for s in srcs[1:]:
                acc = f(acc, s)
            return acc
    if t == 9:
        scal = torch.tensor(1.0 / n, dtype=torch.float32).to(torch.bfloat16)
        pre = (lambda x: x * scal) if op == 4 else (lambda x: x)
        acc = pre(srcs[0])
        for s in srcs[1:]:
            s = pre(s)
            if op in (0, 4):
                acc = acc + s
            elif op == 1:
                acc = acc * s
            elif op == 2:
                acc = torch.fmax(acc, s)
            else:
                acc = torch.fmin(acc, s)
        return acc
    dt = FLT_NP[t]
    scal = dt(np.float32(1.0 / n)) if t != 8 else 1.0 / n
    pre = (lambda x: (x * scal).astype(dt)) if op == 4 else (lambda x: x)
    with np.errstate(all="ignore"):
        acc = pre(srcs[0])
        for s in srcs[1:]:
            s = pre(s)
            if op in (0, 4):
                acc = (acc + s).astype(dt)
            elif op == 1:
                acc = (acc * s).astype(dt)
            elif op == 2:
                acc = np.fmax(acc, s)
            else:
                acc = np.fmin(acc, s)
    return acc


def as_bits(t, a):
    if t == 9:
        return a.view(torch.int16).numpy().view(np.uint16).copy()
    return np.ascontiguousarray(a)


def ring_case(rng, t, n):
    """Ring all-reduce sum fold: owner ring index per element; ring = identity."""
    srcs = gen_inputs(rng, t, n)
    owner = rng.integers(0, n, size=N).astype(np.int32)
    exp = []
    for i in range(N):
        o = int(owner[i])
        order = [(o + j) % n for j in range(1, n + 1)]  # o+1, o+2, ..., o
        if t == 9:
            acc = srcs[order[0]][i]
            for k in order[1:]:
                acc = srcs[k][i] + acc
        else:
            dt = FLT_NP[t]
            with np.errstate(all="ignore"):
                acc = srcs[order[0]][i]
                for k in order[1:]:
                    acc = dt(srcs[k][i] + acc)
        exp.append(acc)
    if t == 9:
        exp = torch.stack(exp)
    else:
        exp = np.array(exp, dtype=FLT_NP[t])
    return srcs, owner, exp


def main():
    torch.manual_seed(0)
    rng = np.random.default_rng(20260206)
    out = {}
    for t in TYPES:
        for op in OPS:
            for nsrc in (2, 3, 8):
                srcs = gen_inputs(rng, t, nsrc)
                exp = fold(t, op, srcs)
                key = f"rc_{TYPES[t]}_{OPS[op]}_{nsrc}"
                out[key + "_in"] = np.stack([as_bits(t, s) for s in srcs])
                out[key + "_out"] = as_bits(t, exp)
    for t in (7, 6, 9):
        for n in (2, 4, 8):
            srcs, owner, exp = ring_case(rng, t, n)
            key = f"ring_{TYPES[t]}_sum_{n}"
            out[key + "_in"] = np.stack([as_bits(t, s) for s in srcs])
            out[key + "_owner"] = owner
            out[key + "_out"] = as_bits(t, exp)
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {len(out)} arrays, {os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    main()
