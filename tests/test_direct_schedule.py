"""CPU simulation of the two-shot direct all-reduce's data movement
(vccl_amd/csrc/device/direct.hpp, host/enqueue.cc launch_direct).

Replays phases 1-3 with numpy over the same shard / block partition and inbox
region layout the kernel uses, and checks that (a) every write stays inside
its inbox region, (b) every output element is produced exactly once per rank,
and (c) the result equals the ring all-reduce's (VCCL's ring schedule on the same
channels and rings, tests/_ring.py expected_allreduce): phase 2 folds every
element in the order of its ring chunk (direct.hpp, ar_chunk_of), for ragged
counts, every element size and n = 2..8.  No GPU needed.
"""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import vccl_sched as S
from tests import _ring

MIN_BLK_BYTES = 16 << 10


def _geometry(count, n, esz, max_blocks, chunk_bytes):
    """host/enqueue.cc launch_direct: chunk, block length (fixed per launch),
    block count, inbox region bytes."""
    align = max(1, 16 // esz)
    region = (chunk_bytes + n - 1) // n // 256 * 256 + 256
    chunk = _ring.direct_chunk_elts(count, n, esz, chunk_bytes)
    shard0 = _ring.direct_shard_elts(chunk, n, esz)
    min_blk = MIN_BLK_BYTES // esz
    nb = max(1, min(-(-shard0 // min_blk), max_blocks))
    blk = -(-(-(-shard0 // nb)) // align) * align
    n_blocks = -(-shard0 // blk)
    return chunk, blk, n_blocks, region


def _simulate(op, dtype, inputs, nch, slot, max_blocks=64, chunk_bytes=16 << 20):
    n = len(inputs)
    dev_op, arg = O.host_to_dev_redop(op, dtype, n)
    pre = dev_op == O.DEV_PREMULSUM
    count = inputs[0].size
    esz = inputs[0].dtype.itemsize
    chunk, blk, n_blocks, region = _geometry(count, n, esz, max_blocks, chunk_bytes)
    # the ring's partition of the bucket: channel and finishing ring position
    # of every element (what ar_chunk_of looks up on the device)
    work = S.cbd_schedule("ar", count, esz, n, nch, buff_size=slot * S.NCCL_STEPS)
    chan, fin = S.allreduce_owner(work, count, n)
    rings = _ring.ring_orders(n)
    assert n_blocks <= 128
    n_chunks = -(-count // chunk)
    outs = [np.zeros_like(inputs[0]) for _ in range(n)]
    written = [np.zeros(count, np.int32) for _ in range(n)]
    for c in range(n_chunks):
        c0 = c * chunk
        cc = min(chunk, count - c0)
        shard = _ring.direct_shard_elts(cc, n, esz)
        inbox = {}  # (rank, phase, src, b) -> array

        def block_of(o, b):
            end = min((o + 1) * shard, cc)
            lo = o * shard + b * blk
            hi = min(lo + blk, end)
            return c0 + lo, max(0, hi - lo)

        for b in range(n_blocks):
            in_off = b * blk * esz
            for me in range(n):  # phase 1
                for k in range(1, n):
                    p = (me + k) % n
                    off, ln = block_of(p, b)
                    assert in_off + ln * esz <= region, "inbox region overflow"
                    inbox[p, 0, me, b] = inputs[me][off:off + ln].copy()
            for me in range(n):  # phase 2: every element in its ring chunk's order
                off, ln = block_of(me, b)
                res = inputs[me][off:off + ln].copy()
                src = {q: inbox[me, 0, q, b] for q in range(n) if q != me}
                src[me] = inputs[me][off:off + ln]
                ch = chan[off:off + ln]
                for c in np.unique(ch):
                    sel = np.nonzero(ch == c)[0]
                    ring = rings[c % len(rings)]
                    res[sel] = O.ring_fold(dev_op, dtype, arg, pre, [src[q][sel] for q in ring],
                                           fin[off + sel])
                outs[me][off:off + ln] = res
                written[me][off:off + ln] += 1
                for j in range(1, n):
                    inbox[(me + j) % n, 1, me, b] = res.copy()
            for me in range(n):  # phase 3
                for k in range(1, n):
                    o = (me + k) % n
                    off, ln = block_of(o, b)
                    outs[me][off:off + ln] = inbox[me, 1, o, b]
                    written[me][off:off + ln] += 1
    for r in range(n):
        assert (written[r] == 1).all(), "every element produced exactly once"
    return outs


@pytest.mark.parametrize("chunk_bytes", [16 << 20, 256 << 10])
@pytest.mark.parametrize("n", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("dtype,count", [(7, 786_433), (9, 100_003), (0, 3_001), (4, 5), (6, 70_001)])
def test_direct_simulation_matches_expected(n, dtype, count, chunk_bytes):
    rng = np.random.default_rng(n * 100 + dtype)
    if dtype in (0, 4):
        ins = [rng.integers(-100, 100, count).astype(O.NP_DTYPE[dtype]) for _ in range(n)]
        op = 2  # max
    elif dtype == 9:
        ins = [O.f32_to_bf16_bits(rng.uniform(-1, 1, count).astype(np.float32)) for _ in range(n)]
        op = 0
    else:
        ins = [rng.uniform(-1, 1, count).astype(O.NP_DTYPE[dtype]) for _ in range(n)]
        op = 4 if dtype == 6 else 0  # f16 avg exercises preOp on every input
    nch, slot = _ring.n_channels(n), 512 << 10
    outs = _simulate(op, dtype, ins, nch, slot, chunk_bytes=chunk_bytes)
    exp = _ring.expected_allreduce(op, dtype, ins, nch, slot)
    for r in range(n):
        assert np.array_equal(outs[r].view(np.uint8), exp.view(np.uint8)), f"rank {r}"


def test_direct_geometry_small_block_cap():
    # 16 blocks (the shared-GPU test cap) over an 8-rank 16 MiB bucket
    chunk, blk, nb, region = _geometry((16 << 20) // 4, 8, 4, 16, 16 << 20)
    assert nb == 16 and blk * nb * 4 <= region and blk % 4 == 0 and chunk == (16 << 20) // 4


def test_direct_chunks_cover_large_bucket():
    # a 1 GiB f32 bucket through the default 16 MiB inbox: 64+ chunks, each
    # shard within its region
    count, n, esz = (1 << 30) // 4, 8, 4
    chunk, blk, nb, region = _geometry(count, n, esz, 64, 16 << 20)
    assert _ring.direct_shard_elts(chunk, n, esz) * esz <= region
    assert -(-count // chunk) >= 64
