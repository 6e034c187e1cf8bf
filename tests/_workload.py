"""BASELINE workloads at full size for the GPU parity tests (config 3: 1 GiB
fp32 all-reduce; config 4: reduce-scatter + all-gather of a 4 GiB bf16
bucket), checked two ways:

* an integer-valued pattern whose reduction is exact in any fold order
  (bench.pattern_fill / pattern_ok), over the WHOLE output;
* hashed floating-point inputs with varied exponents (so the fold order
  shows in the rounding), whose values any process can regenerate for any
  index: the worker generates them on the GPU, the test regenerates the
  inputs of sampled windows on the host and folds them with the CPU oracle
  in VCCL's ring order (oracle/vccl_sched.py partition + ring_fold), bit-exact.
  Windows straddle every channel-part boundary and a sample of the chunk
  boundaries, plus random positions.

The hash is a 32-bit multiply-xorshift mixer evaluated in int64 with every
product below 2^63 (multipliers < 2^31, operands < 2^32), so numpy and torch
(CPU or GPU) give identical bits.
"""
import numpy as np

from oracle import oracle as O
from oracle import vccl_sched as S
from tests import _ring

M32 = 0xFFFFFFFF
WIN = 64            # elements on each side of a boundary
N_RANDOM = 64       # random windows per output


def _mix(h):
    h = h ^ (h >> 16)
    h = (h * 0x7FEB352D) & M32
    h = h ^ (h >> 15)
    h = (h * 0x2C1B3C6D) & M32
    h = h ^ (h >> 16)
    h = (h * 0x297A2D39) & M32
    h = h ^ (h >> 15)
    return h


def hash32(idx, rank, salt):
    """idx: int64 array (numpy or torch)."""
    h = (idx & M32) ^ ((rank * 0x3243F6A9 + salt * 0x2545F491) & M32)
    h = _mix(h)
    h = (h + (idx >> 32)) & M32
    return _mix(h)


def bits_of(dtype, idx, rank):
    """Raw bits of input element `idx` of `rank`: bf16 (uint16 pattern) or f32
    (uint32 pattern), sign random, exponent over 8 binades around 1, mantissa
    random — returned as int64 values."""
    h1 = hash32(idx, rank, 0)
    if dtype == 9:  # bf16
        sign = h1 >> 31
        exp = 121 + ((h1 >> 24) & 7)
        mant = (h1 >> 8) & 0x7F
        return (sign << 15) | (exp << 7) | mant
    h2 = hash32(idx, rank, 1)
    sign = h1 >> 31
    exp = 121 + ((h1 >> 24) & 7)
    mant = h2 & 0x7FFFFF
    return (sign << 31) | (exp << 23) | mant


def host_values(dtype, idx, rank):
    b = bits_of(dtype, np.asarray(idx, dtype=np.int64), rank)
    return b.astype(np.uint16) if dtype == 9 else b.astype(np.uint32).view(np.float32)


def device_fill(buf, dtype, rank, base=0, slice_elems=1 << 26):
    """Fill the 1-D torch tensor `buf` (bf16 or f32) with rank's hashed
    inputs for global indices [base, base + numel)."""
    import torch
    n = buf.numel()
    raw = buf.view(torch.int16 if dtype == 9 else torch.int32)
    for lo in range(0, n, slice_elems):
        hi = min(n, lo + slice_elems)
        idx = torch.arange(base + lo, base + hi, device=buf.device, dtype=torch.int64)
        b = bits_of(dtype, idx, rank)
        wrap = 1 << (16 if dtype == 9 else 32)
        b = torch.where(b >= wrap // 2, b - wrap, b)
        raw[lo:hi] = b.to(raw.dtype)
        del idx, b


def _windows(bounds, total, rng):
    pts = set()
    for b in bounds:
        for i in range(max(0, b - WIN), min(total, b + WIN)):
            pts.add(i)
    for s in rng.integers(0, max(1, total - 2 * WIN), N_RANDOM):
        pts.update(range(int(s), min(total, int(s) + 2 * WIN)))
    pts.update(range(max(0, total - WIN), total))
    return np.array(sorted(pts), dtype=np.int64)


def _part_bounds(work, chunk_sample=48, rng=None):
    """Channel-part starts and a sample of chunk starts inside the parts."""
    bounds = []
    for c in range(work.channel_lo, work.channel_hi + 1):
        off, length, chunk = work.part(c)
        bounds.append(off)
        starts = list(range(off + chunk, off + length, chunk))
        if len(starts) > chunk_sample:
            starts = [starts[i] for i in sorted(rng.choice(len(starts), chunk_sample, replace=False))]
        bounds += starts
    return bounds


def ar_windows(count, esz, n, nch, slot, nthreads, seed=0):
    """Sample indices of an all-reduce output: every channel-part and ring
    loop / chunk boundary (k * chunk inside each loop, incl. the short last
    loop) up to a sample, plus random windows."""
    rng = np.random.default_rng(seed)
    work = S.cbd_schedule("ar", count, esz, n, nch, buff_size=slot * S.NCCL_STEPS, nthreads=nthreads)
    bounds = []
    elt_align = max(1, 16 // esz)
    for c in range(work.channel_lo, work.channel_hi + 1):
        off, length, chunk = work.part(c)
        bounds.append(off)
        loop = n * chunk
        eo, cand = 0, []
        while eo < length:
            rem = length - eo
            ck = chunk if rem >= loop else (rem + n - 1) // n
            ck = (ck + elt_align - 1) // elt_align * elt_align  # all_reduce.h:36
            cand += [off + eo + k * ck for k in range(1, n)] + [off + eo]
            eo += loop
        if len(cand) > 48:
            cand = [cand[i] for i in sorted(rng.choice(len(cand), 48, replace=False))]
        bounds += cand
    return _windows(bounds, count, rng), work


def rs_windows(recvcount, esz, n, nch, slot, nthreads, seed=1):
    rng = np.random.default_rng(seed)
    work = S.cbd_schedule("rs", recvcount, esz, n, nch, buff_size=slot * S.NCCL_STEPS,
                          nthreads=nthreads)
    return _windows(_part_bounds(work, rng=rng), recvcount, rng), work


def expected_ar_windows(dtype, idx, n, work, rings=None, op=0):
    """VCCL's ring all-reduce result at indices `idx` (the channel's ring,
    folded from position owner+1 around to the owner)."""
    rings = rings or _ring.ring_orders(n)
    dev_op, arg = O.host_to_dev_redop(op, dtype, n)
    ins = [host_values(dtype, idx, r) for r in range(n)]
    chan, owner = S.allreduce_owner_at(work, int(idx.max()) + 1 if idx.size else 0, n, idx)
    out = np.empty_like(ins[0])
    for c in np.unique(chan):
        sel = np.nonzero(chan == c)[0]
        ring = rings[int(c) % len(rings)]
        out[sel] = O.ring_fold(dev_op, dtype, arg, dev_op == O.DEV_PREMULSUM,
                               [ins[q][sel] for q in ring], owner[sel])
    return out


def expected_rs_windows(dtype, idx, n, rank, recvcount, work, rings=None, op=0):
    """Rank `rank`'s reduce-scatter output at block indices `idx`: folded on
    the ring of each element's channel, finishing at `rank`."""
    rings = rings or _ring.ring_orders(n)
    dev_op, arg = O.host_to_dev_redop(op, dtype, n)
    gidx = rank * recvcount + idx
    ins = [host_values(dtype, gidx, r) for r in range(n)]
    chan = np.full(idx.size, -1, np.int64)
    for c in range(work.channel_lo, work.channel_hi + 1):
        off, length, _ = work.part(c)
        chan[(idx >= off) & (idx < off + length)] = c
    out = np.empty_like(ins[0])
    for c in np.unique(chan):
        sel = np.nonzero(chan == c)[0]
        ring = rings[int(c) % len(rings)]
        own = np.full(sel.size, ring.index(rank), np.int32)
        out[sel] = O.ring_fold(dev_op, dtype, arg, dev_op == O.DEV_PREMULSUM,
                               [ins[q][sel] for q in ring], own)
    return out
