"""Deterministic multi-rank collective cases shared by the single-process and
multi-process GPU tests (inputs regenerated from seeds on both sides)."""
import numpy as np

from oracle import oracle as O
from tests import _ring

# (name, coll, op, dtype, count) — count = AR count, RS recvcount, AG sendcount
CASES = [
    ("ar_f32_sum_ragged", "ar", 0, 7, (1 << 20) + 17),
    ("ar_f32_sum_tiny", "ar", 0, 7, 3),
    ("ar_bf16_sum", "ar", 0, 9, 100_003),
    ("ar_f16_avg", "ar", 4, 6, 65_536 + 8),
    ("ar_i32_max", "ar", 2, 2, 77_777),
    ("ar_i64_min", "ar", 3, 4, 5_001),
    ("ar_u8_prod", "ar", 1, 1, 33_333),
    ("ar_i32_avg", "ar", 4, 2, 40_000),
    ("ar_f64_sum", "ar", 0, 8, 30_001),
    ("ar_f32_sum_inplace", "ar_inplace", 0, 7, 1 << 21),
    ("ar_f16_sum_inplace_small", "ar_inplace", 0, 6, 4097),
    ("ar_bf16_sum_ll_edge", "ar", 0, 9, (1 << 19) - 3),
    # two-shot direct range under the test geometry (1 MiB < bytes <= 4 MiB)
    ("ar_f32_sum_direct", "ar", 0, 7, 786_433),
    ("ar_bf16_avg_direct", "ar", 4, 9, 1_200_001),
    ("ar_i8_max_direct", "ar", 2, 0, 3_000_001),
    ("ar_f16_sum_inplace_direct", "ar_inplace", 0, 6, 1_000_003),
    ("ar_i64_sum_direct", "ar", 0, 4, 300_001),
    ("ar_u32_avg_direct", "ar", 4, 3, 500_007),
    ("rs_f32_sum", "rs", 0, 7, 65_537),
    ("rs_bf16_avg", "rs", 4, 9, 20_000),
    ("rs_u32_min", "rs", 3, 3, 9_999),
    # per-rank blocks off 16-byte alignment: slot offsets + shifted sources
    ("rs_bf16_sum_odd", "rs", 0, 9, 20_001),
    ("rs_i8_max_odd", "rs", 2, 0, 1_003),
    ("ag_f16_odd", "ag", 0, 6, 3_001),
    ("ag_f32", "ag", 0, 7, 4_099),
    ("ag_u8_odd", "ag", 0, 1, 1_001),
    # fp8 (OCP e4m3 / e5m2 through half, reduce_kernel.h:309-321): LL, direct, ring
    ("ar_f8e4m3_sum", "ar", 0, 10, 100_003),
    ("ar_f8e5m2_avg_direct", "ar", 4, 11, 2_000_001),
    ("ar_f8e4m3_max_direct", "ar", 2, 10, 1_500_007),
    ("rs_f8e4m3_sum_odd", "rs", 0, 10, 20_001),
    ("rs_f8e5m2_prod", "rs", 1, 11, 9_999),
    # user buffers off 16-byte alignment (send and receive by different
    # amounts, MIS_OFFSETS): LL, direct (engine realignment + staged output)
    ("ar_f32_sum_mis_direct", "ar_mis", 0, 7, 786_433),
    ("ar_bf16_avg_mis_direct", "ar_mis", 4, 9, 1_200_001),
    ("ar_u8_max_mis_direct", "ar_mis", 2, 1, 3_000_001),
    ("ar_f64_sum_mis_direct", "ar_mis", 0, 8, 300_001),
    ("ar_f16_sum_mis_ll", "ar_mis", 0, 6, 20_001),
    # fp sum / prod per path, checked bit-exactly against the path's own fold
    # and within the §8c tolerance of VCCL's (exact value; VCCL's ring
    # schedule on a reference geometry) — the north-star fp parity claim
    ("ar_f32_prod_ll", "ar", 1, 7, 200_003),
    ("ar_f16_prod_direct", "ar", 1, 6, 1_000_001),
    ("ar_bf16_prod_ring", "ar", 1, 9, 3_000_001),
    ("ar_f16_sum_ring", "ar", 0, 6, 2_600_001),
    ("ar_bf16_sum_direct", "ar", 0, 9, 1_500_001),
    ("rs_f16_prod", "rs", 1, 6, 30_001),
    ("rs_bf16_sum", "rs", 0, 9, 70_001),
    # one-hop direct reduce-scatter / all-gather (a block above the test
    # geometry's 1 MiB LL slot; several inbox chunks), odd counts = blocks
    # off 16-byte alignment
    ("rs_f32_sum_direct", "rs", 0, 7, 300_001),
    ("rs_bf16_avg_direct_odd", "rs", 4, 9, 700_001),
    ("rs_i8_min_direct_odd", "rs", 3, 0, 1_500_003),
    ("rs_f16_prod_direct", "rs", 1, 6, 600_001),
    ("ag_f32_direct", "ag", 0, 7, 300_001),
    ("ag_u8_direct_odd", "ag", 0, 1, 1_500_007),
] + [
    # BASELINE config 5: fp16 sum at every power of two from 8 B to 128 KiB
    # (the one-hop LL all-reduce wherever the geometry's LL threshold admits
    # it — 8 ranks included — checked bit-exactly against the oracle's chain
    # fold, and within tolerance of VCCL's ring result)
    (f"ar_f16_sum_ll_{1 << p}B", "ar", 0, 6, (1 << p) // 2) for p in range(3, 18)
]

# VCCL's ring schedule on the geometry its own tuner would pick on an 8-GPU
# NVLink node (one ring order on every channel, 16 channels, NCCL_BUFFSIZE
# 4 MiB): the "VCCL result" fp outputs are held to within tolerance.
VCCL_REF_CHANNELS = 16
VCCL_REF_SLOT = 512 << 10
TOLERANCE_OPS = (0, 1)  # sum, prod


def mis_offsets(dt):
    """(send, recv) byte offsets of the "ar_mis" buffers: element-aligned,
    off 16-byte alignment, different from each other where possible."""
    esz = np.dtype(O.NP_DTYPE[dt]).itemsize
    return esz % 16, (3 * esz) % 16


def _fp8_codes(dt, x):
    """Vectorised RN-even f32 -> fp8 for |x| < 2 (no saturation or NaN in
    range): the code whose value is nearest, ties to the even code."""
    vals = O.fp8_bits_to_f32(dt, np.arange(128, dtype=np.uint8))
    vals = np.where(np.isnan(vals), np.inf, vals)
    a = np.abs(x)
    hi = np.searchsorted(vals, a)  # vals[hi-1] < a <= vals[hi]
    hi = np.clip(hi, 1, 127)
    lo = hi - 1
    dlo, dhi = a - vals[lo], vals[hi] - a
    pick = np.where((dhi < dlo) | ((dhi == dlo) & (hi % 2 == 0)), hi, lo)
    return (pick | np.where(np.signbit(x), 0x80, 0)).astype(np.uint8)


def gen_input(case_idx, rank, n_ranks):
    name, coll, op, dt, count = CASES[case_idx]
    total = count * n_ranks if coll == "rs" else count
    return _gen_values(np.random.default_rng(1000 * case_idx + rank), op, dt, total)


# ncclReduce cases (name, op, dtype, count, inplace): every root of each is
# run; ragged counts, every op family, PreMulSum (avg), and one bucket of
# several chunks per channel
REDUCE_CASES = [
    ("red_f32_sum_ragged", 0, 7, 300_001, False),
    ("red_f32_sum_one", 0, 7, 1, False),
    ("red_f16_sum", 0, 6, 70_001, False),
    ("red_bf16_sum", 0, 9, (1 << 20) + 3, False),
    ("red_f32_avg", 4, 7, 123_457, False),
    ("red_i32_max", 2, 2, 5_000, False),
    ("red_u8_prod", 1, 1, 4_099, False),
    ("red_f64_min", 3, 8, 1_000, False),
    ("red_bf16_prod", 1, 9, 33_333, False),
    ("red_i64_sum_multichunk", 0, 4, 1 << 21, False),
    ("red_f32_sum_inplace", 0, 7, 200_003, True),
]


def gen_reduce_input(ri, rank):
    name, op, dt, count, _ = REDUCE_CASES[ri]
    return _gen_values(np.random.default_rng(7000 + 100 * ri + rank), op, dt, count)


def _gen_values(rng, op, dt, total):
    if dt in (0, 1, 2, 3, 4, 5):
        npdt = O.NP_DTYPE[dt]
        if op == 1:  # keep products interesting
            return rng.integers(1, 4, total).astype(npdt)
        return rng.integers(0, 2**62, total, dtype=np.int64).astype(np.uint64).view(np.int64).astype(npdt)
    if op == 1 and dt in (6, 7, 8, 9):  # products of n values stay normal
        x = (rng.uniform(0.5, 2.0, total) * rng.choice([-1.0, 1.0], total)).astype(np.float32)
        return O.f32_to_bf16_bits(x) if dt == 9 else x.astype(O.NP_DTYPE[dt])
    if dt == 9:
        return O.f32_to_bf16_bits(rng.uniform(-1, 1, total).astype(np.float32))
    if dt in (10, 11):  # fp8 codes of uniform values (every code of the range)
        return _fp8_codes(dt, rng.uniform(-2, 2, total).astype(np.float32))
    return rng.uniform(-1, 1, total).astype(O.NP_DTYPE[dt])


# One ncclGroupStart/End of all-reduces (name, op, dtype, count): runs of
# small ones with one type and op are fused into one LL launch (up to 16 per
# launch); a different type, a bucket above the LL threshold or the 16-part
# cap starts a new launch.  Inputs are seeded per (group index, rank).
GROUP_CASES = (
    [("g_f32_sum_a", 0, 7, 1000), ("g_f32_sum_tiny", 0, 7, 3), ("g_f32_sum_b", 0, 7, 20_001),
     ("g_f16_sum_a", 0, 6, 777), ("g_f16_sum_b", 0, 6, 4096),
     ("g_f32_sum_big", 0, 7, 300_001),
     ("g_f32_sum_c", 0, 7, 513), ("g_bf16_avg_a", 4, 9, 1001), ("g_bf16_avg_b", 4, 9, 2003),
     ("g_i32_max_a", 2, 2, 999), ("g_u8_prod_a", 1, 1, 4097)]
    + [(f"g_f32_min_{i}", 3, 7, 64 + 37 * i) for i in range(20)])


def gen_group_input(gi, rank):
    name, op, dt, count = GROUP_CASES[gi]
    rng = np.random.default_rng(777_000 + 100 * gi + rank)
    if dt in (0, 1, 2, 3, 4, 5):
        if op == 1:
            return rng.integers(1, 4, count).astype(O.NP_DTYPE[dt])
        return rng.integers(-1000, 1000, count).astype(O.NP_DTYPE[dt])
    if dt == 9:
        return O.f32_to_bf16_bits(rng.uniform(-1, 1, count).astype(np.float32))
    return rng.uniform(-1, 1, count).astype(O.NP_DTYPE[dt])


GROUP_CALLS = [("ar", op, dt, count) for name, op, dt, count in GROUP_CASES]


def group_algos(coll_algo, n_ranks):
    """Every GROUP_CASES call's path as the comm lays the group out (the path
    of its 4x aggregate, _ring.group_algos; coll_algo = Comm.coll_algo)."""
    return _ring.group_algos(GROUP_CALLS, n_ranks, coll_algo)


def group_plan_works(n_ranks, nch, slot_bytes, nthreads=512, algos=None):
    """[CbdWork per GROUP_CASES call]: the group's VCCL plan
    (host/enqueue.cc launch_planned) with every call on its aggregate's path
    (`algos`, group_algos; None = every call RING / SIMPLE)."""
    return _ring.group_works(GROUP_CALLS, n_ranks, nch, slot_bytes, nthreads, algos=algos)


def expected_group(gi, n_ranks, nch, slot_bytes, nthreads=512, plan=None, algos=None, chain=None):
    """`plan`: group_plan_works(...) of the group (VCCL's grouped partition),
    `algos`: the calls' paths (LL: the chain fold; ring / LL128 ring / direct:
    the ring's fold on the call's place in the plan)."""
    name, op, dt, count = GROUP_CASES[gi]
    ins = [gen_group_input(gi, r) for r in range(n_ranks)]
    path = "ll" if algos[gi] == "ll" else "ring"
    return expected_ar(op, dt, ins, n_ranks, nch, slot_bytes, 0, 0, 0, nthreads, plan[gi].proto,
                       work=plan[gi], chain=chain, path=path)


def expected_ar(op, dt, ins, n_ranks, nch, slot_bytes, ll_max, direct_max, direct_chunk,
                nthreads=512, proto=2, work=None, chain=None, path=None):
    """All-reduce result: LL chain fold up to ll_max bytes, the ring's
    owner-map fold (VCCL's ring schedule on these channels) above — for the
    two-shot direct path too, which folds every element in the ring's order
    (direct.hpp phase 2), so neither direct_max nor the inbox chunk
    (direct_chunk) changes the expected bits.  `work`: the call's place in
    its group's plan; `chain`: the LL fold chain, root first (VCCL_LL_CHAIN;
    None = the identity); `path`: "ll" | "ring" when known (a grouped call
    takes its aggregate's path), else from ll_max."""
    del direct_max, direct_chunk
    count = len(ins[0])
    if path == "ll" or (path is None and count * ins[0].dtype.itemsize <= ll_max):
        dev_op, arg = O.host_to_dev_redop(op, dt, n_ranks)
        order = chain if chain is not None else range(n_ranks)
        return O.chain_fold(dev_op, dt, arg, dev_op == O.DEV_PREMULSUM, [ins[r] for r in order])
    return _ring.expected_allreduce(op, dt, ins, nch, slot_bytes, nthreads=nthreads, proto=proto,
                                    work=work)


def expected(case_idx, n_ranks, nch, slot_bytes, ll_max=0, direct_max=0, direct_chunk=16 << 20,
             nthreads=512, proto=2, chain=None, ll_rs_max=None):
    """proto: the ring's protocol (2 SIMPLE, 1 LL128 — VCCL's LL128 partition)."""
    """Per-rank expected outputs.  All-reduce buckets of at most `ll_max`
    bytes take the one-shot LL path, whose fold is the chain-tree order
    (oracle ref_chain_fold); larger ones the two-shot direct path (up to
    `direct_max`) or the ring, both in the ring's owner-map fold."""
    name, coll, op, dt, count = CASES[case_idx]
    ins = [gen_input(case_idx, r, n_ranks) for r in range(n_ranks)]
    if coll in ("ar", "ar_inplace", "ar_mis"):
        e = expected_ar(op, dt, ins, n_ranks, nch, slot_bytes, ll_max, direct_max, direct_chunk,
                        nthreads, proto, chain=chain)
        return [e] * n_ranks
    if coll == "rs":
        # the one-hop LL reduce-scatter (one rank's block within the LL
        # threshold, n <= 8; n x the threshold is the RS / AG default) folds
        # per channel of VCCL's LL ring partition
        # (ll_rs_max: that threshold when it differs from the all-reduce's —
        # NCCL_ALGO=Ring keeps ring LL for RS / AG but no LL all-reduce)
        ll = n_ranks <= 8 and count * ins[0].dtype.itemsize <= (ll_max if ll_rs_max is None else ll_rs_max)
        return _ring.expected_reducescatter(op, dt, ins, nch, nthreads=nthreads,
                                            proto=_ring.S.PROTO_LL if ll else proto)
    full = np.concatenate(ins)
    return [full] * n_ranks


def inputs(case_idx, n_ranks):
    return [gen_input(case_idx, r, n_ranks) for r in range(n_ranks)]


def vccl_reference(case_idx, n_ranks):
    """VCCL's own result for a float sum/prod case: its ring schedule (cbd
    partition, chunking, runRing fold) on VCCL_REF_CHANNELS identity-ring
    channels; None for cases outside the tolerance check."""
    name, coll, op, dt, count = CASES[case_idx]
    if dt not in (6, 7, 8, 9) or op not in TOLERANCE_OPS or coll == "ag":
        return None
    ins = inputs(case_idx, n_ranks)
    ring = [list(range(n_ranks))]
    if coll == "rs":
        return _ring.expected_reducescatter(op, dt, ins, VCCL_REF_CHANNELS, VCCL_REF_SLOT, rings=ring)
    e = _ring.expected_allreduce(op, dt, ins, VCCL_REF_CHANNELS, VCCL_REF_SLOT, rings=ring)
    return [e] * n_ranks


def vccl_group_reference(gi, n_ranks, vplan):
    """VCCL's own result for a float sum/prod GROUP_CASES call: its grouped
    ring schedule (vplan = group_plan_works on VCCL_REF_CHANNELS, every call
    taken as RING / SIMPLE) folded on identity rings; None outside the
    tolerance check."""
    name, op, dt, count = GROUP_CASES[gi]
    if dt not in (6, 7, 8, 9) or op not in TOLERANCE_OPS:
        return None
    ins = [gen_group_input(gi, r) for r in range(n_ranks)]
    return _ring.expected_allreduce(op, dt, ins, VCCL_REF_CHANNELS, VCCL_REF_SLOT,
                                    rings=[list(range(n_ranks))], work=vplan[gi])


def out_count(case_idx, n_ranks):
    name, coll, op, dt, count = CASES[case_idx]
    return count * n_ranks if coll == "ag" else count


def run_group(comm_streams, rank_of, n_ranks):
    """Enqueue GROUP_CASES inside one ncclGroupStart/End for each (comm, streams)
    pair (streams alternate per call, so the fused launch joins two streams).
    Returns {comm index: {name: output tensor}} once the device is idle."""
    import torch
    from vccl_amd import nccl
    bufs = []
    for ci, (comm, streams) in enumerate(comm_streams):
        per = {}
        for gi, (name, op, dt, count) in enumerate(GROUP_CASES):
            x = gen_group_input(gi, rank_of[ci])
            xb = torch.from_numpy(x.view(np.uint8).copy()).cuda()
            yb = torch.empty_like(xb)
            per[name] = (xb, yb, x.dtype)
        bufs.append(per)
    torch.cuda.synchronize()
    nccl.group_start()
    for ci, (comm, streams) in enumerate(comm_streams):
        for gi, (name, op, dt, count) in enumerate(GROUP_CASES):
            xb, yb, _ = bufs[ci][name]
            comm.all_reduce(xb.data_ptr(), yb.data_ptr(), count, dt, op,
                            streams[gi % len(streams)].cuda_stream)
    nccl.group_end()
    torch.cuda.synchronize()
    return {ci: {name: yb.cpu().numpy().view(npdt) for name, (xb, yb, npdt) in bufs[ci].items()}
            for ci in range(len(comm_streams))}
