"""VCCL's ring channel partition (cbd split + chunking) — CPU checks.

* the library's host planner (vcclRingPartition, host/enqueue.cc
  cbd_schedule) equals the oracle's independent restatement
  (oracle/vccl_sched.py) over a sweep of collectives, sizes, types, rank and
  channel counts and slot sizes;
* properties the reference's code implies: parts tile [0, count) exactly, all
  boundaries are 16-byte multiples (cells are, enqueue.cc:600; so the 16 B
  fast path survives, common_kernel.h:237-241), at most nChannels channels,
  every channel but the last carries at least the 16 KiB traffic floor
  (enqueue.cc:528), and the SIMPLE ring chunk is 4 FIFO steps (2 MiB at the
  default 4 MiB NCCL_BUFFSIZE, collectives.h:16-22, enqueue.cc:2027-2030).
* hand-derived cases (worked through from enqueue.cc:598-644 in comments).
"""
import numpy as np
import pytest

from oracle import vccl_sched as S
from vccl_amd import nccl

COLLS = {"ar": 0, "rs": 1, "ag": 2}
ESZ = {0: 1, 9: 2, 6: 2, 7: 4, 8: 8, 4: 8}


def _sizes():
    rng = np.random.default_rng(5)
    fixed = [1, 3, 7, 16, 100, 2047, 2048, 2049, 4096, 65_536, 1 << 20, (1 << 20) + 17,
             (1 << 24) + 5, 1 << 28]
    return fixed + [int(x) for x in rng.integers(1, 1 << 26, 24)]


@pytest.mark.parametrize("coll", ["ar", "rs", "ag"])
@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_library_partition_equals_oracle(coll, n):
    for nch in (1, 2, 7, 14, 32, 56, 64):
        for dt in (7, 9, 0, 8):
            # NCCL_NTHREADS: 256 changes the channel tuning
            # (enqueue.cc:1921-1924) and with it every part boundary
            for slot, nt in ((4096, 512), (256 << 10, 512), (512 << 10, 512), (512 << 10, 256)):
                for count in _sizes():
                    lib = nccl.ring_partition(COLLS[coll], count, dt, n, nch, slot, nt)
                    w = S.cbd_schedule(coll, count, ESZ[dt], n, nch,
                                       buff_size=slot * S.NCCL_STEPS, nthreads=nt)
                    per = S.grain_size(w.proto) // w.elt_size
                    ref = (w.channel_lo, w.channel_hi, w.count_lo, w.count_mid, w.count_hi,
                           w.chunk_grains_lo * per, w.chunk_grains_mid * per, w.chunk_grains_hi * per)
                    # chunk sizes of absent parts are unused on the device
                    assert lib[:5] == ref[:5], (coll, n, nch, dt, slot, nt, count, lib, ref)
                    for i, cnt in ((5, w.count_lo), (6, w.count_mid), (7, w.count_hi)):
                        if cnt:
                            assert lib[i] == ref[i], (coll, n, nch, dt, slot, count, i)


@pytest.mark.parametrize("coll", ["ar", "rs", "ag"])
def test_partition_properties(coll):
    for n in (2, 4, 8):
        for nch in (1, 8, 56, 64):
            for dt in (7, 9, 0):
                for count in _sizes():
                    esz = ESZ[dt]
                    w = S.cbd_schedule(coll, count, esz, n, nch)
                    total = count * esz if coll == "ag" else count
                    e = w.elt_size
                    assert 0 <= w.channel_lo <= w.channel_hi < nch
                    ends = []
                    cover = 0
                    for c in range(w.channel_lo, w.channel_hi + 1):
                        off, ln, chunk = w.part(c)
                        assert off == cover and ln >= 0
                        assert (off * e) % 16 == 0
                        assert chunk * e == 2 << 20
                        cover += ln
                        ends.append(ln)
                    assert cover == total
                    if w.channel_hi > w.channel_lo:
                        tpb = 2 if coll == "ar" else n
                        assert all(ln * e * tpb >= S.MIN_TRAFFIC_PER_CHANNEL for ln in ends[:-1])


@pytest.mark.parametrize("coll", ["ar", "rs", "ag"])
def test_library_ll128_partition_equals_oracle(coll):
    """The LL128 ring's partition (VCCL's LL128 cells, 1,920 B grain, 576,000 B
    chunk of the 614,400 B step, 640-thread channel tuning, enqueue.cc:
    1902-1925, 2027-2032) from the library vs the oracle."""
    for n in (2, 4, 8):
        for nch in (1, 14, 56):
            for dt in (7, 9, 0):
                for count in _sizes():
                    lib = nccl.ring_partition(COLLS[coll], count, dt, n, nch, 614_400, 640,
                                              proto=nccl.PROTO_LL128)
                    w = S.cbd_schedule(coll, count, ESZ[dt], n, nch, proto=S.PROTO_LL128)
                    per = S.grain_size(w.proto) // w.elt_size
                    ref = (w.channel_lo, w.channel_hi, w.count_lo, w.count_mid, w.count_hi,
                           w.chunk_grains_lo * per, w.chunk_grains_mid * per, w.chunk_grains_hi * per)
                    assert lib[:5] == ref[:5], (coll, n, nch, dt, count, lib, ref)
                    for i, cnt in ((5, w.count_lo), (6, w.count_mid), (7, w.count_hi)):
                        if cnt:
                            assert lib[i] == ref[i] == 576_000 // w.elt_size, (coll, n, nch, dt, count, i)


def test_hand_derived_cases():
    # 1 GiB f32 all-reduce, 56 channels (8 GPUs x 7 rings x 8): traffic 2 GiB,
    # 38,347,922 B per channel; 8 KiB cells (16 KiB traffic), 131,072 cells;
    # cellsPerChannel = cellsLo = 2341, nMid = 54, cellsHi = 2317.
    w = S.cbd_schedule("ar", 1 << 28, 4, 8, 56)
    assert (w.channel_lo, w.channel_hi) == (0, 55)
    assert (w.count_lo, w.count_mid, w.count_hi) == (2341 * 2048, 2341 * 2048, 2317 * 2048)
    # 64 KiB f32 all-reduce: the channel tuning keeps nc = 2 (65,536 B is not
    # < 2 x 512 x 64), so 64 KiB of traffic per channel = 4 cells: lo 4, no
    # mid, hi 4 -> 2 channels of 8192 elements.
    w = S.cbd_schedule("ar", 16384, 4, 8, 56)
    assert (w.channel_lo, w.channel_hi, w.count_lo, w.count_mid, w.count_hi) == (0, 1, 8192, 0, 8192)
    # 256 KiB: nc = 8, 64 KiB per channel; cellsHi = 0 borrows the last mid
    # (enqueue.cc:620-623): lo, 6 mids, hi of 4 cells each.
    w = S.cbd_schedule("ar", 65536, 4, 8, 56)
    assert (w.channel_lo, w.channel_hi, w.count_lo, w.count_mid, w.count_hi) == (0, 7, 8192, 8192, 8192)
    # 3 elements: one channel, countLo = cell - excess
    w = S.cbd_schedule("ar", 3, 4, 8, 56)
    assert (w.channel_lo, w.channel_hi, w.count_lo) == (0, 0, 3)
    # one comm channel: everything goes to "lo" (enqueue.cc:607-608)
    w = S.cbd_schedule("rs", 1 << 20, 2, 8, 1)
    assert (w.channel_lo, w.channel_hi, w.count_lo) == (0, 0, 1 << 20)
    # the per-call channel tuning: 1 MiB all-reduce < nc * 512 thr * 64 B for
    # nc > 32, so at most 32 channels carry it (enqueue.cc:1921-1924)
    assert S.ring_n_max_channels("ar", 1 << 18, 4, 8, 56) == 32
    # NCCL_NTHREADS=256 halves the per-channel threshold: 64 channels' worth
    assert S.ring_n_max_channels("ar", 1 << 18, 4, 8, 56, nthreads=256) == 56
    assert nccl.ring_partition(0, 1 << 18, 7, 8, 56, 512 << 10, 256)[1] > \
        nccl.ring_partition(0, 1 << 18, 7, 8, 56, 512 << 10, 512)[1]


@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_library_chunk_lookup_equals_oracle(n):
    """vcclRingChunkOf (ring_types.hpp ar_chunk_of, the lookup the direct
    all-reduce folds by) vs the oracle's owner map of VCCL's ring all-reduce
    (channel and finishing ring position of every element): at every chunk
    boundary (both sides) and at random elements."""
    rng = np.random.default_rng(n)
    for nch in (1, 7, 14, 56):
        for dt in (7, 9, 0, 8):
            for count in (3, 1000, 65_536 + 8, (1 << 20) + 17, 3_000_001):
                w = S.cbd_schedule("ar", count, ESZ[dt], n, nch, buff_size=(256 << 10) * S.NCCL_STEPS)
                chan, owner = S.allreduce_owner(w, count, n)
                key = chan.astype(np.int64) * 64 + owner
                starts = np.concatenate([[0], np.nonzero(np.diff(key))[0] + 1])
                ends = np.concatenate([starts[1:], [count]])
                pick = set(starts[:200].tolist()) | set((ends[:200] - 1).tolist())
                pick |= set(rng.integers(0, count, 100).tolist())
                for i in sorted(pick):
                    ch, k, end = nccl.ring_chunk_of(count, dt, n, nch, 256 << 10, i)
                    j = np.searchsorted(starts, i, side="right") - 1
                    assert (ch, k, end) == (chan[i], owner[i], ends[j]), (n, nch, dt, count, i)
