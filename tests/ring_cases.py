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
    ("ag_f32", "ag", 0, 7, 4_099),
    ("ag_u8_odd", "ag", 0, 1, 1_001),
]


def gen_input(case_idx, rank, n_ranks):
    name, coll, op, dt, count = CASES[case_idx]
    total = count * n_ranks if coll == "rs" else count
    rng = np.random.default_rng(1000 * case_idx + rank)
    if dt in (0, 1, 2, 3, 4, 5):
        npdt = O.NP_DTYPE[dt]
        if op == 1:  # keep products interesting
            return rng.integers(1, 4, total).astype(npdt)
        return rng.integers(0, 2**62, total, dtype=np.int64).astype(np.uint64).view(np.int64).astype(npdt)
    if dt == 9:
        return O.f32_to_bf16_bits(rng.uniform(-1, 1, total).astype(np.float32))
    return rng.uniform(-1, 1, total).astype(O.NP_DTYPE[dt])


def expected(case_idx, n_ranks, nch, slot_bytes, ll_max=0, direct_max=0, direct_chunk=16 << 20):
    """Per-rank expected outputs.  All-reduce buckets of at most `ll_max`
    bytes take the one-shot LL path, whose fold is the chain-tree order
    (oracle ref_chain_fold); up to `direct_max` the two-shot direct path
    (identity-ring fold per shard of each `direct_chunk`-byte chunk); larger
    ones the ring (owner-map ring fold)."""
    name, coll, op, dt, count = CASES[case_idx]
    ins = [gen_input(case_idx, r, n_ranks) for r in range(n_ranks)]
    if coll in ("ar", "ar_inplace"):
        if count * ins[0].dtype.itemsize <= ll_max:
            dev_op, arg = O.host_to_dev_redop(op, dt, n_ranks)
            e = O.chain_fold(dev_op, dt, arg, dev_op == O.DEV_PREMULSUM, ins)
        elif count * ins[0].dtype.itemsize <= direct_max:
            e = _ring.expected_direct(op, dt, ins, direct_chunk)
        else:
            e = _ring.expected_allreduce(op, dt, ins, nch, slot_bytes)
        return [e] * n_ranks
    if coll == "rs":
        return _ring.expected_reducescatter(op, dt, ins, nch)
    full = np.concatenate(ins)
    return [full] * n_ranks


def out_count(case_idx, n_ranks):
    name, coll, op, dt, count = CASES[case_idx]
    return count * n_ranks if coll == "ag" else count
