"""VCCL's multi-task plan for a group of ring calls — CPU checks.

* the library's group planner (vcclGroupPlan, host/enqueue.cc group_plan)
  equals the oracle's independent restatement (oracle/vccl_sched.py
  plan_schedule) over random groups of mixed collectives, types, ops and
  sizes, and a group of one call equals the one-call partition;
* hand-derived cases worked through from enqueue.cc:352-437 (sorter, bins,
  4x aggregation) and :549-681 (shared trafficPerChannel, running channelId /
  currentTraffic);
* a group too large for one kernel's argument budget splits into plans whose
  channel assignment restarts at channel 0 (enqueue.cc:535, :636);
* the path per aggregate (vcclGroupPlanEx): every member of a 4x aggregate
  takes the path of the summed count (enqueue.cc:387-427), an LL member's
  traffic counts 4x (:418, :599) and LL calls move the channel cursor the
  ring calls after them start from — library == oracle over random groups
  and random path policies, plus hand-derived cases;
* NCCL_ALGO / NCCL_PROTO list parsing (vcclAlgoSelection, graph/tuning.cc:
  53-116 parseList semantics).
"""
import numpy as np
import pytest

from oracle import vccl_sched as S
from tests import _ring
from vccl_amd import nccl

COLL = {0: "ar", 1: "rs", 2: "ag", 3: "bc", 4: "red"}
ESZ = {0: 1, 1: 1, 2: 4, 3: 4, 4: 8, 5: 8, 6: 2, 7: 4, 8: 8, 9: 2, 10: 1, 11: 1}


def _oracle_calls(calls, n):
    """GroupCall list for the oracle: bins by (func, devOp, type) — AG as
    int8 copies — and device functions with the signed -> unsigned kernel
    equivalence (generate.py:129-137)."""
    out = []
    for coll, count, dt, op in calls:
        if coll in (2, 3):  # byte copies (AG, broadcast)
            key = func = (coll, 0, 0)
        else:
            dev_op, _ = nccl.host_to_dev_redop(op, dt, n)
            key = (coll, dev_op, dt)
            func = (coll, dev_op, nccl.kernel_type_of(dev_op, dt))
        out.append(S.GroupCall(COLL[coll], count, ESZ[dt], key, func))
    return out


def _as_tuple(w):
    per = S.grain_size(w.proto) // w.elt_size
    return (w.channel_lo, w.channel_hi, w.count_lo, w.count_mid, w.count_hi,
            w.chunk_grains_lo * per, w.chunk_grains_mid * per, w.chunk_grains_hi * per)


def _check_equal(calls, n, nch, slot=512 << 10, nthreads=512):
    order, plan_of, parts = nccl.group_plan(calls, n, nch, slot, nthreads)
    o_order, o_plan, o_works = S.plan_schedule(_oracle_calls(calls, n), n, nch,
                                               buff_size=slot * S.NCCL_STEPS, nthreads=nthreads)
    assert order == o_order, (calls, order, o_order)
    assert plan_of == o_plan, (calls, plan_of, o_plan)
    for i, (lib, w) in enumerate(zip(parts, o_works)):
        ref = _as_tuple(w)
        assert lib[:5] == ref[:5], (i, calls[i], lib, ref)
        for k, cnt in ((5, w.count_lo), (6, w.count_mid), (7, w.count_hi)):
            if cnt:
                assert lib[k] == ref[k], (i, calls[i], k)
    return order, plan_of, parts


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8])
def test_library_group_plan_equals_oracle(n):
    rng = np.random.default_rng(100 + n)
    for trial in range(40):
        k = int(rng.integers(1, 17))
        calls = []
        for _ in range(k):
            coll = int(rng.integers(0, 3))
            dt = int(rng.choice([7, 9, 6, 2, 3, 0, 8]))
            op = int(rng.choice([0, 1, 2, 3]))
            count = int(rng.choice([1, 100, 4096, 65_536, 1 << 20, (1 << 20) + 37, 3 << 20, 1 << 24])) \
                + int(rng.integers(0, 64))
            calls.append((coll, count, dt, op))
        nch = int(rng.choice([1, 2, 16, 32, 48, 56, 60, 63, 64]))  # incl. the defaults at 2-8 ranks
        nt = int(rng.choice([256, 512]))
        _check_equal(calls, n, nch, nthreads=nt)


def test_single_call_group_is_the_call_partition():
    for n in (2, 4, 8):
        for nch in (1, 16, 56):
            for coll, count, dt in ((0, 1 << 20, 7), (1, 12345, 9), (2, 1 << 22, 6), (0, 3, 7)):
                _, _, parts = nccl.group_plan([(coll, count, dt, 0)], n, nch)
                assert parts[0] == nccl.ring_partition(coll, count, dt, n, nch, 512 << 10), \
                    (n, nch, coll, count)


def test_hand_derived_four_allreduces():
    """4 fp32 all-reduces of 4 MiB at 8 ranks on 56 channels (enqueue.cc:
    549-681 by hand): traffic 8 MiB each, all in one aggregate (nc stays 56),
    trafficPerChannel = 32 MiB / 56 = 599,186 B; 8 KiB cells (16 KiB traffic),
    512 cells per call, cellsPerChannel = 37.
      call 0 at (ch 0, 0 B):        lo 37, 12 mid, hi 31 -> ch 0..13, next (13, 507,904)
      call 1 at (13, 507,904):      lo 6,  13 mid, hi 25 -> ch 13..27, next (27, 409,600)
      call 2 at (27, 409,600):      lo 12, 13 mid, hi 19 -> ch 27..41, next (41, 311,296)
      call 3 at (41, 311,296):      lo 18, 13 mid, hi 13 -> ch 41..55
    """
    calls = [(0, 1 << 20, 7, 0)] * 4
    order, plan_of, parts = _check_equal(calls, 8, 56)
    assert order == [0, 1, 2, 3] and plan_of == [0, 0, 0, 0]
    e = 2048  # elements per 8 KiB cell
    want = [(0, 13, 37 * e, 37 * e, 31 * e), (13, 27, 6 * e, 37 * e, 25 * e),
            (27, 41, 12 * e, 37 * e, 19 * e), (41, 55, 18 * e, 37 * e, 13 * e)]
    assert [p[:5] for p in parts] == want


def test_hand_derived_order_and_aggregation():
    """The plan order (enqueue.cc:352-437): sorter bins by trafficBytes
    descending (newest first within a bin), then one LIFO per (func, op,
    type) -> size-ascending lists in order of first appearance.  Calls at 4
    ranks: 0 = AR f32 2^18 (2 MiB traffic), 1 = RS bf16 recvcount 2^20
    (8 MiB), 2 = AR f32 2^22 (32 MiB), 3 = AR f32 2^20 (8 MiB).  Sorted:
    [2, 3, 1, 0] (3 and 1 share a bin, 3 is newer); AR list [0, 3, 2], RS
    list [1]; AR first -> order [0, 3, 2, 1].  No two AR calls aggregate
    (8 MiB is not < 4 x 2 MiB, 32 MiB is not < 4 x 8 MiB)."""
    calls = [(0, 1 << 18, 7, 0), (1, 1 << 20, 9, 0), (0, 1 << 22, 7, 0), (0, 1 << 20, 7, 0)]
    order, plan_of, parts = _check_equal(calls, 4, 48)
    assert order == [0, 3, 2, 1]
    assert set(plan_of) == {0}
    # channels are handed out in plan order: each call starts where the
    # previous one stopped
    assert parts[0][0] == 0
    for a, b in zip(order, order[1:]):
        assert parts[b][0] in (parts[a][1], parts[a][1] + 1), (a, b, parts[a], parts[b])
    # a min and a max reduction share ncclPrepareTasks' bin (one devOp,
    # MinMax): calls 0 (min), 1 (max), 2 (sum), equal sizes -> one sorter
    # bin, newest first [2, 1, 0]; the sum bin appears first; the MinMax LIFO
    # gives [0, 1] -> order [2, 0, 1]
    o, _, _ = _check_equal([(0, 1 << 20, 7, 3), (0, 1 << 20, 7, 2), (0, 1 << 20, 7, 0)], 4, 48)
    assert o == [2, 0, 1]


def test_aggregation_lowers_channel_tuning():
    """Four 64 KiB f32 all-reduces aggregate (each within 4x of the first):
    nMaxChannels is tuned on the aggregate's 256 KiB, not on 64 KiB."""
    calls = [(0, 16384, 7, 0)] * 4
    o_works = S.plan_schedule(_oracle_calls(calls, 8), 8, 56)[2]
    # alone, a 64 KiB all-reduce keeps 2 channels (S.ring_n_max_channels); the
    # aggregate's 256 KiB gives 8, so the plan spreads the four calls further
    assert S.ring_n_max_channels("ar", 16384, 4, 8, 56) == 2
    assert S.ring_n_max_channels("ar", 4 * 16384, 4, 8, 56) == 8
    assert max(w.channel_hi for w in o_works) >= 4
    _check_equal(calls, 8, 56)


def test_budget_splits_plans():
    """A group too large for one kernel's arguments is cut into several plans
    (enqueue.cc:533-545: the estimate admits calls while divUp(calls, 4)
    16-byte batches fit 4 KiB - 32 B of arguments: call k is admitted while
    16 * divUp(k, 4) <= 4,064, so 1,017 calls); each
    plan hands out channels from 0 again."""
    calls = [(0, 1024 + 4 * (i % 7), 7, 0) for i in range(1100)]
    order, plan_of, parts = _check_equal(calls, 8, 64)
    assert plan_of.count(0) == 1017
    assert max(plan_of) >= 1, plan_of
    for p in set(plan_of):
        first = [i for i in order if plan_of[i] == p][0]
        assert parts[first][0] == 0


def test_algo_selection():
    LL, LL128, SIMPLE, DIRECT, LLRS = 1, 2, 4, 8, 16  # LL: the LL all-reduce; LLRS: LL RS / AG
    cases = {
        (None, None): (0, LL | LLRS | LL128 | SIMPLE | DIRECT),
        (None, "LL128"): (4, LL128),
        (None, "^LL128"): (0, LL | LLRS | SIMPLE | DIRECT),  # excludes LL128
        (None, "LL,LL128"): (0, LL | LLRS | LL128),         # no longer "LL128 everywhere"
        (None, "ll"): (2, LL | LLRS),
        (None, "Simple"): (0, SIMPLE | DIRECT),
        ("Ring", None): (0, LLRS | LL128 | SIMPLE),         # ring LL for RS / AG
        ("Ring", "Simple"): (1, SIMPLE),
        ("Ring", "LL"): (2, LLRS),                          # ring + LL is a valid pair
        ("Tree", None): (2, LL | LLRS),
        ("Tree", "Simple"): (1, SIMPLE),                    # no SIMPLE tree here: the SIMPLE ring, WARNed
        ("Tree", "LL128"): (4, LL128),                      # Simple excluded -> the LL128 ring
        ("Direct", "LL128"): (4, LL128),
        ("NVLS", "Simple"): (1, SIMPLE),                    # no NVLS here: the SIMPLE ring, WARNed
        ("NVLS", "^Simple"): (4, LL128),
        ("Direct", None): (3, DIRECT),
        ("^Direct", None): (0, LL | LLRS | LL128 | SIMPLE),
        ("ring;allreduce:tree", None): (0, LLRS | LL128 | SIMPLE),  # per-collective entries ignored
    }
    for (algo, proto), want in cases.items():
        assert nccl.algo_selection(algo, proto) == want, (algo, proto)
    # unknown names, or lists that leave no protocol / no algorithm at all
    for algo, proto in ((None, "bogus"), ("Ring,Foo", None), (None, "^LL,LL128,Simple"),
                        ("Direct", "LL"), ("NVLS,PAT", "LL"),  # only LL allowed, no LL path for them
                        ("^Tree,Ring,CollnetDirect,CollnetChain,NVLS,NVLSTree,PAT,Direct", None)):
        with pytest.raises(nccl.VcclError) as e:
            nccl.algo_selection(algo, proto)
        assert e.value.code == nccl.ncclInvalidUsage


def _random_policy(rng, n):
    ll_max = int(rng.choice([0, 64 << 10, 128 << 10, 1 << 20]))
    return dict(force=int(rng.choice([0, 0, 0, 0, 1, 2, 3, 4])),
                ll_slot=int(rng.choice([0, 1 << 20, 1 << 20, 2 << 20])),
                ll_max=ll_max, ll_rsag_max=int(rng.choice([n * ll_max, 0, 1 << 20])),
                ll128=int(rng.integers(0, 2)), ll128_min=64 << 10,
                ll128_max=int(rng.choice([0, 1 << 20, 8 << 20])),
                direct=int(rng.integers(0, 2)), direct_max=int(rng.choice([0, 4 << 20, 8 << 20])),
                direct_rsag_max=int(rng.choice([0, 8 << 20, 64 << 20])))


def _check_equal_ex(calls, n, nch, policy, slot=512 << 10, nthreads=512):
    """vcclGroupPlanEx == the oracle's plan with the same path per aggregate
    (_ring.select_algo on the aggregate's count)."""
    algos, order, plan_of, parts = nccl.group_plan_ex(calls, n, nch, policy, slot, nthreads)

    def algo_of(i, agg):
        coll, _, dt, _ = calls[i]
        return _ring.select_algo(policy, COLL[coll], 1 if coll in (2, 3) else ESZ[dt], agg, n)
    o_algos = []
    o_order, o_plan, o_works = S.plan_schedule(_oracle_calls(calls, n), n, nch, buff_size=slot * S.NCCL_STEPS,
                                               nthreads=nthreads, algo_of=algo_of, algos_out=o_algos)
    assert algos == o_algos, (calls, policy, algos, o_algos)
    assert order == o_order and plan_of == o_plan, (calls, policy)
    for i, (lib, w) in enumerate(zip(parts, o_works)):
        ref = _as_tuple(w)
        assert lib[:5] == ref[:5], (i, calls[i], algos[i], lib, ref)
        for k, cnt in ((5, w.count_lo), (6, w.count_mid), (7, w.count_hi)):
            if cnt:
                assert lib[k] == ref[k], (i, calls[i], algos[i], k)
    return algos, order, plan_of, parts


@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_library_group_plan_ex_equals_oracle(n):
    rng = np.random.default_rng(900 + n)
    for trial in range(60):
        k = int(rng.integers(1, 21))
        calls = []
        for _ in range(k):
            coll = int(rng.integers(0, 5))  # incl. broadcast and reduce
            dt = int(rng.choice([7, 9, 6, 2, 0, 8]))
            op = int(rng.choice([0, 1, 2, 3]))
            count = int(rng.choice([1, 100, 4096, 16384, 40_000, 65_536, 300_000, 1 << 20, 3 << 20])) \
                + int(rng.integers(0, 64))
            calls.append((coll, count, dt, op))
        nch = int(rng.choice([1, 2, 14, 16, 32, 56, 63, 64]))
        _check_equal_ex(calls, n, nch, _random_policy(rng, n), nthreads=int(rng.choice([256, 512])))


def test_group_plan_ex_without_policy_is_group_plan():
    calls = [(0, 1 << 20, 7, 0), (1, 12_345, 9, 0), (2, 4096, 6, 0), (0, 3, 7, 2)]
    algos, order, plan_of, parts = nccl.group_plan_ex(calls, 4, 56, None)
    assert algos == ["ring"] * 4
    assert (order, plan_of, parts) == nccl.group_plan(calls, 4, 56)


DEFAULTS_8 = dict(force=0, ll_slot=1 << 20, ll_max=128 << 10, ll_rsag_max=8 * (128 << 10), ll128=0,
                  ll128_min=64 << 10, ll128_max=0, direct=0, direct_max=0, direct_rsag_max=0)


def test_hand_derived_ll_call_moves_the_cursor():
    """A 64 KiB fp32 all-reduce (LL: VCCL's tree LL) planned with three 8 MiB
    ones (ring) at 8 ranks on 56 channels, worked through enqueue.cc:387-427,
    :549-681 by hand.  LL trafficBytes = 64 KiB x 2 x 4 = 512 KiB; nMaxChannels
    LL (tree: threshold 8, 512 threads): 16; ring: 56.  trafficPerChannel =
    (512 KiB + 3 x 16 MiB) / 56 = 908,141 B.  The LL call (first: its bin is
    size-ascending) at (ch 0, 0): cells of 2 KiB (16 KiB traffic each, x4),
    32 cells, all on ch 0 (lo = min(32, divUp(908,141, 16,384))), cursor (0,
    524,288).  Ring call 1 at (0, 524,288): 8 KiB cells, 1024 cells,
    cellsPerChannel 56, lo = divUp(908,141 - 524,288, 16,384) = 24, 17 mid,
    hi 48 -> ch 0..18."""
    calls = [(0, 16384, 7, 0)] + [(0, 2 << 20, 7, 0)] * 3
    algos, order, plan_of, parts = _check_equal_ex(calls, 8, 56, DEFAULTS_8)
    assert algos == ["ll", "ring", "ring", "ring"] and order == [0, 1, 2, 3]
    assert parts[0][:5] == (0, 0, 16384, 0, 0)
    assert parts[1][:5] == (0, 18, 24 * 2048, 56 * 2048, 48 * 2048)
    # planned as a SIMPLE ring call the small bucket would leave call 1 on
    # another partition: the LL protocol's 4x traffic is what moves it
    _, _, _, ring_parts = nccl.group_plan_ex(calls, 8, 56, None)
    assert ring_parts[1][:5] != parts[1][:5]


def test_hand_derived_ll_split_then_ring_at_four_ranks():
    """another plan worked through enqueue.cc:352-437, :518-681 by
    hand and asserted on the library directly (not only through the Python
    restatement).  4 ranks, 48 channels: fp32 all-reduces of 32 KiB (LL) and
    4 MiB (ring) in one group.  Sorter + LIFO bin: [32 KiB, 4 MiB]; 4 MiB is
    not within 4x of 32 KiB, so two aggregates.  trafficBytes: LL 32 KiB x 2
    x 4 = 256 KiB, ring 4 MiB x 2 = 8 MiB; nMaxChannels: LL (threshold 8, 512
    threads) 8, ring 48 -> min(56, 48) = 48; trafficPerChannel = 8,650,752 /
    48 = 180,224 B.
      LL call at (0, 0): cell 2 KiB (traffic x 8), 16 cells, cellsPerChannel
        = cellsLo = divUp(180,224, 16,384) = 11, hi 5 -> ch 0..1, counts
        (5,632, 0, 2,560); cursor -> (1, 2,560 x 32 = 81,920)
      ring call at (1, 81,920): cell 8 KiB, 512 cells, lo = divUp(98,304,
        16,384) = 6, 46 mid x 11 with no remainder -> 45 mid + hi 11
        -> ch 1..47, counts (12,288, 22,528, 22,528)."""
    pol = dict(DEFAULTS_8, ll_rsag_max=4 * (128 << 10))
    calls = [(0, 8192, 7, 0), (0, 1 << 20, 7, 0)]
    algos, order, plan_of, parts = _check_equal_ex(calls, 4, 48, pol)
    assert algos == ["ll", "ring"] and order == [0, 1] and plan_of == [0, 0]
    assert parts[0][:5] == (0, 1, 5632, 0, 2560)
    assert parts[1][:5] == (1, 47, 12288, 22528, 22528)


def test_aggregate_takes_one_path():
    """Two fp32 all-reduces of 48 KiB and 100 KiB at 8 ranks: each alone is
    on the LL path (<= 128 KiB), but the second is within 4x of the first, so
    they aggregate and the 148 KiB aggregate takes the ring — for both
    (enqueue.cc:392-424: getAlgoInfo on the aggregate, its choice given to
    every member).  A third call 4x larger starts its own aggregate (ring by
    its own size); 16 KiB and 64 KiB calls stay apart and both on LL."""
    calls = [(0, 12 * 1024, 7, 0), (0, 25 * 1024, 7, 0), (0, 100 * 1024, 7, 0)]
    for coll, count, dt, _ in calls[:2]:
        assert _ring.select_algo(DEFAULTS_8, "ar", 4, count, 8) == "ll"
    algos, order, _, _ = _check_equal_ex(calls, 8, 56, DEFAULTS_8)
    assert algos == ["ring", "ring", "ring"], algos
    calls = [(0, 4096, 7, 0), (0, 16384, 7, 0)]  # 64 KiB is not < 4 x 16 KiB: two aggregates
    algos, _, _, _ = _check_equal_ex(calls, 8, 56, DEFAULTS_8)
    assert algos == ["ll", "ll"], algos


def test_single_call_ll_partition():
    """The one-hop LL reduce-scatter folds per channel of VCCL's LL ring
    partition (LL cells: traffic x4; LL threshold x nRanks): library ==
    oracle (vcclRingPartition with proto 0)."""
    for n in (2, 4, 8):
        for nch in (1, 14, 56):
            for count, dt in ((1000, 7), (20_001, 9), (65_537, 7), (1_003, 0), (30_001, 6)):
                for nt in (256, 512):
                    lib = nccl.ring_partition(1, count, dt, n, nch, 8 * 512 * 16, nt, proto=0)
                    w = S.cbd_schedule("rs", count, ESZ[dt], n, nch, proto=S.PROTO_LL, nthreads=nt)
                    ref = _as_tuple(w)
                    assert lib[:5] == ref[:5], (n, nch, count, dt, nt, lib, ref)
                    assert lib[5] == ref[5] == 32768 // ESZ[dt]  # half a VCCL LL step



def test_broadcast_partition():
    """The ring broadcast's partition (traffic 1 per byte, one FIFO step per
    chunk, BROADCAST_CHUNKSTEPS, collectives.h:23-24; bytes on the wire):
    library (vcclRingPartition coll 3) == oracle."""
    for n in (2, 4, 8):
        for nch in (1, 14, 56, 64):
            for count, dt in ((1, 7), (1000, 7), (300_001, 9), (1 << 22, 0), ((1 << 24) + 3, 6)):
                for nt in (256, 512):
                    lib = nccl.ring_partition(3, count, dt, n, nch, 512 << 10, nt)
                    w = S.cbd_schedule("bc", count, ESZ[dt], n, nch, buff_size=(512 << 10) * 8, nthreads=nt)
                    ref = _as_tuple(w)
                    assert lib[:5] == ref[:5] and lib[5] == ref[5] == 512 << 10, (n, nch, count, dt, lib, ref)


def test_reduce_partition():
    """The ring reduce's partition (traffic 1 per byte, REDUCE_CHUNKSTEPS 1,
    collectives.h:25-26; typed elements, not bytes): library
    (vcclRingPartition coll 4) == oracle, SIMPLE and LL128."""
    for n in (2, 3, 4, 8):
        for nch in (1, 14, 56, 64):
            for count, dt in ((1, 7), (1000, 7), (300_001, 9), (1 << 22, 0), ((1 << 24) + 3, 6), (77_777, 4)):
                for nt in (256, 512):
                    lib = nccl.ring_partition(4, count, dt, n, nch, 512 << 10, nt)
                    w = S.cbd_schedule("red", count, ESZ[dt], n, nch, buff_size=(512 << 10) * 8, nthreads=nt)
                    ref = _as_tuple(w)
                    assert lib[:5] == ref[:5] and lib[5] == ref[5] == (512 << 10) // ESZ[dt], \
                        (n, nch, count, dt, lib, ref)
                lib = nccl.ring_partition(4, count, dt, n, nch, S.DEFAULT_BUFFSIZE[S.PROTO_LL128] // 8, 640,
                                          proto=S.PROTO_LL128)
                ref = _as_tuple(S.cbd_schedule("red", count, ESZ[dt], n, nch, proto=S.PROTO_LL128))
                assert lib[:5] == ref[:5] and lib[5] == ref[5], (n, nch, count, dt, lib, ref)
