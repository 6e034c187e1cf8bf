"""CPU step-simulation of the device ring schedules (ring.hpp: cbd part per
channel, chunk steps sliced into FIFO slots) against the owner-map
restatement of VCCL's runRing (oracle/vccl_sched.py via tests/_ring.py).  Two independent derivations of the
same fold order must agree bit-exactly, at n = 2..8, ragged counts and tiny
slots (many rounds, empty chunks in the last round).  Also checks the ring
sets: arc-disjoint for 8, every arc twice for 4."""
from collections import deque
from itertools import permutations

import numpy as np
import pytest

from oracle import oracle as O
from oracle import vccl_sched as S
from tests import _ring
from tests._util import assert_bitexact

K_STEPS = 8


def _align_up(x, a):
    return (x + a - 1) // a * a


def _prims_allreduce(n, pos, work, c, slot_elems, elt_align):
    """Yield (recv, send, src_off, dst_off, nelem, post) slot transfers for one
    rank/channel, exactly as ring_allreduce() / ring_step() in ring.hpp: the
    channel's cbd part and chunk (VCCL's partition), each chunk step cut into
    slot-sized slices (an empty step still moves one empty slot)."""
    if not work.channel_lo <= c <= work.channel_hi:
        return
    goff, chcount, chunk = work.part(c)
    loop = n * chunk
    eo = 0
    while eo < chcount:
        rem = chcount - eo
        if rem < loop:
            chunk = _align_up(-(-rem // n), elt_align)
        off = lambda k: goff + eo + k * chunk  # noqa: E731
        ln = lambda k: max(0, min(chunk, rem - k * chunk))  # noqa: E731

        def step(recv, send, k, src, dst, post):
            total = ln(k)
            nsl = max(1, -(-total // slot_elems))
            for s_ in range(nsl):
                o = s_ * slot_elems
                ne = max(0, min(slot_elems, total - o))
                yield (recv, send, off(k) + o if src else None, off(k) + o if dst else None, ne, post)
        yield from step(False, True, (pos + n - 1) % n, True, False, False)
        for j in range(2, n):
            yield from step(True, True, (pos + n - j) % n, True, False, False)
        yield from step(True, True, pos, True, True, True)
        for j in range(1, n - 1):
            yield from step(True, True, (pos + n - j) % n, False, True, False)
        yield from step(True, False, (pos + 1) % n, False, True, False)
        eo += loop


def _simulate_allreduce(op, dt, inputs, nch, slot_bytes):
    n = len(inputs)
    dev_op, arg = O.host_to_dev_redop(op, dt, n)
    esz = inputs[0].dtype.itemsize
    elt_align = max(1, 16 // esz)
    rings = _ring.ring_orders(n)
    outs = [np.zeros_like(inputs[0]) for _ in range(n)]
    work = S.cbd_schedule("ar", inputs[0].size, esz, n, nch, buff_size=slot_bytes * S.NCCL_STEPS)
    for c in range(nch):
        ring = rings[c % len(rings)]
        progs = {r: list(_prims_allreduce(n, ring.index(r), work, c,
                                          slot_bytes // esz, elt_align)) for r in range(n)}
        fifo = {r: deque() for r in range(n)}  # fifo[r]: slots arriving at r
        pc = {r: 0 for r in range(n)}
        while any(pc[r] < len(progs[r]) for r in range(n)):
            moved = False
            for r in range(n):
                if pc[r] >= len(progs[r]):
                    continue
                recv, send, so, do, ne, post = progs[r][pc[r]]
                nxt = ring[(ring.index(r) + 1) % n]
                if recv and not fifo[r]:
                    continue
                if send and len(fifo[nxt]) >= K_STEPS:
                    continue
                srcs, pre = [], 0
                if so is not None:
                    srcs.append(inputs[r][so:so + ne])
                    pre = 1 if dev_op == O.DEV_PREMULSUM else 0
                if recv:
                    srcs.append(fifo[r].popleft()[:ne])
                if ne > 0:
                    val = O.reduce_copy(dev_op, dt, arg, srcs, pre_op_args=[arg] * pre,
                                        post_op=post)[0]
                else:
                    val = inputs[r][:0].copy()
                if send:
                    fifo[nxt].append(val)
                if do is not None and ne > 0:
                    outs[r][do:do + ne] = val
                pc[r] += 1
                moved = True
            assert moved, "deadlock in simulated schedule"
    return outs


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 8])
@pytest.mark.parametrize("dt,op", [(7, 0), (9, 0), (6, 4), (2, 4), (7, 1)])
def test_simulated_schedule_matches_owner_map(n, dt, op):
    rng = np.random.default_rng(n * 10 + dt)
    count = 150_000 + 37 * n  # several loops per channel, a short last loop
    if dt == 9:
        ins = [O.f32_to_bf16_bits(rng.uniform(-1, 1, count).astype(np.float32)) for _ in range(n)]
    elif dt == 2:
        ins = [rng.integers(-1000, 1000, count).astype(np.int32) for _ in range(n)]
    else:
        ins = [rng.uniform(-1, 1, count).astype(O.NP_DTYPE[dt]) for _ in range(n)]
    slot = 4096  # bytes: chunk = 4 slots = 16 KiB, sliced back into slots
    nch = 3
    sim = _simulate_allreduce(op, dt, ins, nch, slot)
    exp = _ring.expected_allreduce(op, dt, ins, nch, slot)
    for r in range(n):
        assert_bitexact(dt, sim[r], exp, what=f"n{n} rank{r}")


def test_ring_sets_are_arc_balanced():
    # every n-1 rings arc-disjoint (8; odd n by Walecki's construction) or every
    # arc in exactly 2 rings (4)
    for n, mult in ((8, 1), (4, 2), (3, 1), (5, 1), (7, 1)):
        arcs = {}
        for ring in _ring.ring_orders(n):
            assert sorted(ring) == list(range(n))
            for i in range(n):
                a = (ring[i], ring[(i + 1) % n])
                arcs[a] = arcs.get(a, 0) + 1
        assert len(arcs) == n * (n - 1)
        assert set(arcs.values()) == {mult}
    # 4 GPUs: no 3 arc-disjoint Hamiltonian cycles exist (why all 6 are used)
    cyc = [(0,) + p for p in permutations((1, 2, 3))]
    arcsets = [{(c[i], c[(i + 1) % 4]) for i in range(4)} for c in cyc]
    disjoint3 = [(a, b, d) for a in range(6) for b in range(a + 1, 6) for d in range(b + 1, 6)
                 if not (arcsets[a] & arcsets[b] or arcsets[a] & arcsets[d] or arcsets[b] & arcsets[d])]
    assert disjoint3 == []


def test_six_rank_rings_edge_disjoint():
    """6 GPUs (no directed Hamiltonian decomposition of K6 exists): two
    edge-disjoint Hamiltonian cycles in both directions — every used arc
    once, 4 of each rank's 5 outgoing links."""
    arcs = {}
    for ring in _ring.ring_orders(6):
        assert sorted(ring) == list(range(6))
        for i in range(6):
            a = (ring[i], ring[(i + 1) % 6])
            arcs[a] = arcs.get(a, 0) + 1
    assert set(arcs.values()) == {1} and len(arcs) == 24
    assert all(sum(1 for a in arcs if a[0] == r) == 4 for r in range(6))


def test_library_ring_sets_equal_restatement():
    """vcclRingOrders (host/init.cc) == tests/_ring.py for every n."""
    from vccl_amd import nccl
    for n in range(1, 9):
        assert nccl.ring_orders(n) == _ring.ring_orders(n), n
