#!/usr/bin/env python3
"""Interleaved launch-geometry sweep of the reduce-copy kernel (config 2 shape).

All variants run in ONE process, round-robin, each launch timed with its own
HIP event pair on the launch stream (cdna_hip_programming.md §5.4 rule 24).
Prints median / min GB/s per variant as JSON lines.
"""
import itertools
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vccl_amd import nccl  # noqa: E402


def main():
    n = int(os.environ.get("SWEEP_ELEMS", 1 << 26))
    rounds = int(os.environ.get("SWEEP_ROUNDS", 16))
    reps = int(os.environ.get("SWEEP_REPS", 10))
    a = torch.rand(n, device="cuda") * 2 - 1
    b = torch.rand(n, device="cuda") * 2 - 1
    d = torch.empty_like(a)
    ref = a + b
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    variants = []
    mode = os.environ.get("SWEEP_MODE", "policies")
    if mode == "misaligned":
        return misaligned(n, rounds, reps)
    if mode.startswith("dtype"):  # dtype<code>: geometry sweep of one element type's sum kernel
        return dtype_geometry(int(mode[5:]), n * 4, rounds, reps)
    if mode == "twodst":
        return two_dst(n, rounds, reps)
    if mode == "twodst_geom":
        return two_dst(n, rounds, reps, geom=True)
    if mode == "policies":
        # load/store policy: 0 plain, 1 nt, 2 sc0 sc1, 3 sc1 nt; order 1 = XCD-contiguous hunks
        for block, unroll, ld, st, order in itertools.product(
                (256,), (4, 8), (1, 2, 3), (0, 1, 2, 3), (0, 1)):
            hunk = block * unroll * 16
            grid = (n * 4 + hunk - 1) // hunk
            variants.append({"blockSize": block, "unroll": unroll, "gridBlocks": grid,
                             "ntLoads": ld, "ntStores": st, "order": order})
    elif mode == "lds":  # LDS-DMA double-buffered staging (order 2) vs the register path
        tiles = n * 4 // (256 * 2 * 16)
        for grid, st in itertools.product((256, 512, 1024, 1280, 2048, tiles), (1, 2)):
            variants.append({"blockSize": 256, "unroll": 2, "gridBlocks": grid,
                             "ntLoads": 1, "ntStores": st, "order": 2})
    elif mode == "fine":  # small hunks, one per workgroup (nt loads, sc0 sc1 stores)
        for block, unroll in itertools.product((64, 128, 256, 512), (1, 2, 4)):
            hunk = block * unroll * 16
            grid = (n * 4 + hunk - 1) // hunk
            variants.append({"blockSize": block, "unroll": unroll, "gridBlocks": grid,
                             "ntLoads": 1, "ntStores": 2, "order": 0})
    else:  # geometry around the tuned policies (nt loads, sc0 sc1 stores)
        for block, unroll, per in itertools.product((256, 512, 1024), (2, 4, 8), (1, 2, 4)):
            hunk = block * unroll * 16
            grid = max(1, (n * 4 + hunk - 1) // hunk // per)
            variants.append({"blockSize": block, "unroll": unroll, "gridBlocks": grid,
                             "ntLoads": 1, "ntStores": 2, "order": 0})
    variants.append(None)  # library default
    variants.append("torch_add")  # known-good reference on the same hardware: torch.add(a, b, out=d)
    times = {i: [] for i in range(len(variants))}
    for r in range(rounds):
        order = list(range(len(variants)))
        np.random.default_rng(r).shuffle(order)
        for i in order:
            cfg = variants[i]
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(reps)]
            for e0, e1 in ev:
                e0.record(s)
                if cfg == "torch_add":
                    torch.add(a, b, out=d)
                else:
                    nccl.reduce_copy(0, 7, 0, [a.data_ptr(), b.data_ptr()], [d.data_ptr()], n, sp,
                                     config=cfg)
                e1.record(s)
            torch.cuda.synchronize()
            times[i] += [e0.elapsed_time(e1) for e0, e1 in ev]
            if r == 0:
                assert torch.equal(d, ref), cfg
    rows = []
    for i, cfg in enumerate(variants):
        t = np.array(times[i][reps:])  # drop the first round (warm-up)
        gbs = 3 * n * 4 / (t / 1e3) / 1e9
        rows.append({"cfg": cfg or "default", "median_gbs": round(float(np.median(gbs)), 1),
                     "max_gbs": round(float(gbs.max()), 1), "median_us": round(float(np.median(t)) * 1e3, 2)})
    rows.sort(key=lambda x: -x["median_gbs"])
    for row in rows:
        print(json.dumps(row))


def misaligned(n, rounds, reps):
    """2-src f32 sum at the config-2 size with byte offsets (src0, src1, dst):
    aligned; a shifted source (lane-shift realignment); a common
    misalignment (head/tail elements + aligned body); two destinations, aligned
    and at different misalignments (destination realignment)."""
    base = [torch.empty(n * 4 + 64, dtype=torch.uint8, device="cuda") for _ in range(4)]
    for b in base[:2]:
        b.view(torch.float32)[:n] = torch.rand(n, device="cuda")
    s = torch.cuda.current_stream()
    variants = {"aligned": ((0, 0), (0,)), "shifted_src1_+4": ((0, 4), (0,)),
                "shifted_both_+4_+8": ((4, 8), (0,)), "common_+4": ((4, 4), (4,)),
                "aligned_2dst": ((0, 0), (0, 0)), "dsts_0_4": ((0, 0), (0, 4)),
                "dsts_0_12": ((0, 0), (0, 12)), "dsts_8_4": ((0, 0), (8, 4))}
    times = {k: [] for k in variants}
    for r in range(rounds):
        for name, (so, do) in variants.items():
            srcs = [base[i].data_ptr() + o for i, o in enumerate(so)]
            dsts = [base[2 + i].data_ptr() + o for i, o in enumerate(do)]
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(reps)]
            for e0, e1 in ev:
                e0.record(s)
                nccl.reduce_copy(0, 7, 0, srcs, dsts, n - 4, s.cuda_stream)
                e1.record(s)
            torch.cuda.synchronize()
            times[name] += [e0.elapsed_time(e1) for e0, e1 in ev]
    for name, (so, do) in variants.items():
        t = np.array(times[name][reps:])
        nbytes = (2 + len(do)) * (n - 4) * 4
        print(json.dumps({"cfg": name, "offsets": [so, do],
                          "median_gbs": round(float(np.median(nbytes / (t / 1e3) / 1e9)), 1),
                          "median_us": round(float(np.median(t)) * 1e3, 2)}))


POL = {"plain": 0, "nt": 1, "sys": 2, "sc1nt": 3}


def two_dst(n, rounds, reps, geom=False):
    """The two-destination shape (2 x n f32 -> 2 x n: the ring's final reduce
    step and every recv-copy-send step) against its read/write-mix reference,
    the 1 -> 1 copy (ours and torch's), interleaved in one process.  2 -> 2
    variants: unroll x per-destination store policy x store order (0
    destination-major, 3 interleaved, 4 pipelined).  GB/s = (srcs + dsts) x
    bytes / kernel time."""
    a = torch.rand(n, device="cuda") * 2 - 1
    b = torch.rand(n, device="cuda") * 2 - 1
    d0, d1 = torch.empty_like(a), torch.empty_like(a)
    ref = a + b
    s = torch.cuda.current_stream()
    hunk = lambda u: 256 * u * 16  # noqa: E731
    variants = []  # (name, nsrc, ndst, cfg)
    if geom:
        # round 5: workgroup size x hunks per workgroup (grid-stride) x
        # unroll x order for the two policy mixes that lead the round-3 sweep
        for blk, per, u, (p0, p1), order in itertools.product(
                (256, 512, 1024), (1, 2, 4), (2, 4), (("sys", "nt"), ("nt", "sys")), (0, 1, 4)):
            hk = blk * u * 16
            cfg = {"blockSize": blk, "unroll": u, "gridBlocks": max(1, (n * 4 + hk - 1) // hk // per),
                   "ntLoads": 1, "ntStores": 16 | POL[p0] | POL[p1] << 2, "order": order}
            variants.append((f"2to2_b{blk}_p{per}_u{u}_{p0}_{p1}_o{order}", 2, 2, cfg))
    for u, (p0, p1), order in itertools.product(
            (2, 4), (("sys", "sys"), ("nt", "nt"), ("plain", "plain"), ("sys", "nt"), ("nt", "sys"),
                     ("sys", "plain"), ("plain", "sys"), ("sc1nt", "sc1nt")), (0, 3, 4)):
        if geom:
            break
        cfg = {"blockSize": 256, "unroll": u, "gridBlocks": (n * 4 + hunk(u) - 1) // hunk(u),
               "ntLoads": 1, "ntStores": 16 | POL[p0] | POL[p1] << 2, "order": order}
        variants.append((f"2to2_u{u}_{p0}_{p1}_o{order}", 2, 2, cfg))
    variants.append(("2to2_default", 2, 2, None))
    for u, ld, st in itertools.product((2, 4), ("nt", "plain"), ("sys", "nt", "plain")):
        cfg = {"blockSize": 256, "unroll": u, "gridBlocks": (n * 4 + hunk(u) - 1) // hunk(u),
               "ntLoads": POL[ld], "ntStores": POL[st], "order": 0}
        variants.append((f"copy_u{u}_{ld}_{st}", 1, 1, cfg))
    variants.append(("copy_torch", 1, 1, "torch_copy"))
    variants.append(("2to1_default", 2, 1, None))
    times = {v[0]: [] for v in variants}
    for r in range(rounds):
        order = list(range(len(variants)))
        np.random.default_rng(r).shuffle(order)
        for i in order:
            name, ns, nd, cfg = variants[i]
            srcs = [a.data_ptr(), b.data_ptr()][:ns]
            dsts = [d0.data_ptr(), d1.data_ptr()][:nd]
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(reps)]
            for e0, e1 in ev:
                e0.record(s)
                if cfg == "torch_copy":
                    d0.copy_(a)
                else:
                    nccl.reduce_copy(0, 7, 0, srcs, dsts, n, s.cuda_stream, config=cfg)
                e1.record(s)
            torch.cuda.synchronize()
            times[name] += [e0.elapsed_time(e1) for e0, e1 in ev]
            if r == 0:
                want = ref if ns == 2 else a
                assert torch.equal(d0, want) and (nd == 1 or torch.equal(d1, want)), name
    rows = []
    for name, ns, nd, cfg in variants:
        t = np.array(times[name][reps:])
        gbs = (ns + nd) * n * 4 / (t / 1e3) / 1e9
        rows.append({"cfg": name, "median_gbs": round(float(np.median(gbs)), 1),
                     "max_gbs": round(float(gbs.max()), 1), "median_us": round(float(np.median(t)) * 1e3, 2)})
    rows.sort(key=lambda x: -x["median_gbs"])
    for row in rows:
        print(json.dumps(row))


def dtype_geometry(dt, nbytes, rounds, reps):
    """Config 2's byte shape (2 x nbytes -> nbytes) for element type `dt`:
    block size x unroll x hunks per workgroup, default policies (nt loads,
    sc0 sc1 stores), interleaved with the library default."""
    esz = {0: 1, 1: 1, 6: 2, 9: 2, 10: 1, 11: 1, 4: 8, 5: 8, 8: 8}.get(dt, 4)
    n = nbytes // esz
    a = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
    b = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
    if dt in (10, 11):  # finite fp8 codes
        a &= 0x77
        b &= 0x77
    d = torch.empty_like(a)
    s = torch.cuda.current_stream()
    variants = [None]
    for block, unroll, per in itertools.product((256, 512, 1024), (1, 2, 4, 8), (1, 2)):
        hunk = block * unroll * 16
        grid = max(1, (nbytes + hunk - 1) // hunk // per)
        variants.append({"blockSize": block, "unroll": unroll, "gridBlocks": grid,
                         "ntLoads": 1, "ntStores": 2, "order": 0})
    times = {i: [] for i in range(len(variants))}
    ref = None
    for r in range(rounds):
        order = list(range(len(variants)))
        np.random.default_rng(r).shuffle(order)
        for i in order:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(reps)]
            for e0, e1 in ev:
                e0.record(s)
                nccl.reduce_copy(0, dt, 0, [a.data_ptr(), b.data_ptr()], [d.data_ptr()], n, s.cuda_stream,
                                 config=variants[i])
                e1.record(s)
            torch.cuda.synchronize()
            times[i] += [e0.elapsed_time(e1) for e0, e1 in ev]
            if ref is None:
                ref = d.clone()
            elif r == 0:
                assert torch.equal(d, ref), variants[i]
    rows = []
    for i, cfg in enumerate(variants):
        t = np.array(times[i][reps:])
        gbs = 3 * nbytes / (t / 1e3) / 1e9
        rows.append({"dtype": dt, "cfg": cfg or "default", "median_gbs": round(float(np.median(gbs)), 1),
                     "median_us": round(float(np.median(t)) * 1e3, 2)})
    rows.sort(key=lambda x: -x["median_gbs"])
    for row in rows:
        print(json.dumps(row))


if __name__ == "__main__":
    main()
