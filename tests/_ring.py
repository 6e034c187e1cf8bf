"""Test-side restatement of the ring data partition, to compute the exact
expected result of a ring collective with the CPU oracle.

The ring's element -> (channel, chunk) partition is VCCL's own (the device
follows it, host/enqueue.cc cbd_schedule; the tests take it from the oracle's
independent restatement, oracle/vccl_sched.py); the ring set per channel and
the channel count mirror vccl_amd/csrc/host/init.cc.  The oracle's ring_fold
then reproduces the fold order element by element, so ring results are
checked bit-exactly against VCCL's schedule on the same rings and channels —
the two-shot direct all-reduce folds in that same order — and the one-shot
LL all-reduce (VCCL's chain-tree order) bit-exactly against its own order
and within the §8c tolerance of VCCL's ring result.
"""
import numpy as np

from oracle import oracle as O
from oracle import vccl_sched as S

RINGS = {
    8: [[0, 1, 2, 3, 4, 5, 6, 7], [0, 2, 1, 3, 5, 4, 7, 6], [0, 3, 1, 4, 6, 2, 7, 5],
        [0, 4, 1, 5, 7, 2, 6, 3], [0, 5, 3, 6, 1, 7, 4, 2], [0, 6, 5, 2, 4, 3, 7, 1],
        [0, 7, 3, 2, 5, 1, 6, 4]],
    4: [[0, 1, 2, 3], [0, 1, 3, 2], [0, 2, 1, 3], [0, 2, 3, 1], [0, 3, 1, 2], [0, 3, 2, 1]],
}


# 6 GPUs: two edge-disjoint Hamiltonian cycles of K6, both directions.
RINGS[6] = [[0, 1, 2, 3, 4, 5], [0, 5, 4, 3, 2, 1], [0, 2, 4, 1, 5, 3], [0, 3, 5, 1, 4, 2]]


def walecki(n):
    """Odd n = 2m+1: Walecki's m edge-disjoint Hamiltonian cycles of K_n (hub
    n-1, then k, k+1, k-1, k+2, ... mod 2m), each in both directions, rotated
    to start at 0 — an independent restatement of host/init.cc."""
    m, h = (n - 1) // 2, n - 1
    out = []
    for k in range(m):
        cyc = [n - 1, k]
        j = 1
        while len(cyc) < n:
            cyc.append((k + j) % h)
            if len(cyc) < n:
                cyc.append((k - j) % h)
            j += 1
        for c in (cyc, [cyc[0]] + cyc[1:][::-1]):
            i = c.index(0)
            out.append(c[i:] + c[:i])
    return out


def ring_orders(n):
    if n in RINGS:
        return RINGS[n]
    if n >= 3 and n % 2 == 1 and n - 1 <= 8:
        return walecki(n)
    return [list(range(n))]


def default_per_ring(n):
    """The library's link-bound channel model (host/init.cc):
    ceil(8 x 76.8 GB/s / (k x 40 GB/s)) channels per ring, k = rings per arc
    (2 for the 4-GPU set), within VCCL's MAXCHANNELS of 64 in total."""
    k = 2 if n == 4 else 1
    model = -(-8 * 768 // (10 * 40 * k))
    return max(1, min(model, 64 // len(ring_orders(n))))


def n_channels(n, per_ring=None, nch=None):
    """Library default channel count (host/init.cc) unless overridden."""
    rings = ring_orders(n)
    if per_ring is None:
        per_ring = default_per_ring(n)
    c = nch if nch is not None else per_ring * len(rings)
    return max(1, min(c, 128))  # kMaxChannels


def _align_up(x, a):
    return (x + a - 1) // a * a


def _div_up(x, a):
    return (x + a - 1) // a


def _sched(coll, count, esz, n, nch, slot_bytes, nthreads, proto):
    """The ring's partition: SIMPLE with the comm's slot and NCCL_NTHREADS,
    LL128 with VCCL's default LL128 buffer and NCCL_LL128_NTHREADS (640), or
    LL (the one-hop LL reduce-scatter's per-channel fold) with NCCL_NTHREADS."""
    if proto == S.PROTO_LL128:
        return S.cbd_schedule(coll, count, esz, n, nch, proto=S.PROTO_LL128)
    if proto == S.PROTO_LL:
        return S.cbd_schedule(coll, count, esz, n, nch, proto=S.PROTO_LL, nthreads=nthreads)
    return S.cbd_schedule(coll, count, esz, n, nch, buff_size=slot_bytes * S.NCCL_STEPS,
                          nthreads=nthreads)


_KERNEL_KEY = {0: 1, 1: 1, 2: 3, 3: 3, 4: 5, 5: 5}  # signed ints run the unsigned kernel


def _group_calls(calls, n):
    gc = []
    for coll, op, dt, count in calls:
        esz = np.dtype(O.NP_DTYPE[dt]).itemsize
        if coll in ("ag", "bc"):  # byte copies
            key = func = (coll, 0, 0)
        else:
            dev_op, _ = O.host_to_dev_redop(op, dt, n)
            key = (coll, dev_op, dt)
            func = (coll, dev_op, _KERNEL_KEY.get(dt, dt))
        gc.append(S.GroupCall(coll, count, esz, key, func))
    return gc


def group_works(calls, n, nch, slot_bytes=512 << 10, nthreads=512, algos=None):
    """VCCL's group plan (oracle/vccl_sched.py plan_schedule) for a group's
    calls of one comm, in call order: calls = [(coll "ar" | "rs" | "ag", op,
    dtype, count)], algos = every call's path (group_algos; None = every call
    "ring"); returns every call's CbdWork (under its path's protocol)."""
    algo_of = None if algos is None else (lambda i, agg: algos[i])
    return S.plan_schedule(_group_calls(calls, n), n, nch, buff_size=slot_bytes * S.NCCL_STEPS,
                           nthreads=nthreads, algo_of=algo_of)[2]


_COLL_CODE = {"ar": 0, "rs": 1, "ag": 2, "bc": 3, "red": 4}


def group_algos(calls, n, coll_algo):
    """The path of every call of a group, as the library lays the group out:
    each (func, op, type) aggregate of VCCL's ncclPrepareTasks (the oracle's
    restatement) takes the path coll_algo(coll code, aggregate count, dtype)
    — the comm's single-call selection (vcclCommCollAlgo) on the summed count
    (all-gathers: bytes, as int8) — and every member takes it."""
    out = []
    def algo_of(i, agg):
        coll, op, dt, count = calls[i]
        return coll_algo(_COLL_CODE[coll], agg, 0 if coll in ("ag", "bc") else dt)
    S.plan_schedule(_group_calls(calls, n), n, 1, nthreads=512, algo_of=algo_of, algos_out=out)
    return out


def select_algo(policy, coll, esz, count, n):
    """The library's path of one bucket (host/enqueue.cc select_algo) on an
    explicit policy dict (vcclGroupPlanEx's policy fields); coll "ar" | "rs" |
    "ag", count in elements of esz."""
    if n < 2 or policy["force"] == 1:
        return "ring"
    if policy["force"] == 4:
        return "ll128" if policy["ll128"] else "ring"
    if coll in ("bc", "red"):  # the broadcast / reduce rings: SIMPLE, or the LL128 window
        nb = count * esz
        return "ll128" if policy["ll128"] and policy["ll128_max"] and policy["ll128_min"] <= nb <= policy["ll128_max"] \
            else "ring"
    block = count * esz
    nbytes = block if coll == "ar" else block * n
    if coll == "ar":
        ll_fits = policy["ll_slot"] > 0 and nbytes <= policy["ll_max"]
        direct_fits = policy["direct"] and nbytes <= policy["direct_max"]
    else:
        ll_fits = (policy["ll_slot"] > 0 and n <= 8 and block <= policy["ll_slot"]
                   and nbytes <= policy["ll_rsag_max"])
        direct_fits = policy["direct"] and nbytes <= policy["direct_rsag_max"]
    if policy["force"] == 2:
        return "ll" if ll_fits else "ring"
    if policy["force"] == 3:
        return "direct" if policy["direct"] and n <= 8 else "ring"
    if ll_fits:
        return "ll"
    if policy["ll128"] and policy["ll128_max"] and policy["ll128_min"] <= nbytes <= policy["ll128_max"]:
        return "ll128"
    return "direct" if direct_fits else "ring"


def expected_allreduce(op, dtype, inputs, nch, slot_bytes, rings=None, nthreads=512,
                       proto=S.PROTO_SIMPLE, work=None):
    """Exact expected ring all-reduce output (identical on every rank): the
    oracle's restatement of VCCL's channel partition and chunking
    (oracle/vccl_sched.py) decides channel and finishing ring index per
    element, channel c runs on rings[c % len(rings)], the C oracle folds.
    `work`: the call's partition inside its group's plan (group_works), else
    the call planned alone."""
    n = len(inputs)
    rings = rings or ring_orders(n)
    dev_op, arg = O.host_to_dev_redop(op, dtype, n)
    pre = dev_op == O.DEV_PREMULSUM
    count = inputs[0].size
    esz = inputs[0].dtype.itemsize
    if work is None:
        work = _sched("ar", count, esz, n, nch, slot_bytes, nthreads, proto)
    chan, owner = S.allreduce_owner(work, count, n)
    out = np.empty_like(inputs[0])
    for c in range(work.channel_lo, work.channel_hi + 1):
        idx = np.nonzero(chan == c)[0]
        if idx.size == 0:
            continue
        ring = rings[c % len(rings)]
        ins = [inputs[r][idx] for r in ring]
        out[idx] = O.ring_fold(dev_op, dtype, arg, pre, ins, owner[idx])
    return out


def expected_reducescatter(op, dtype, inputs, nch, slot_bytes=512 << 10, rings=None, nthreads=512,
                           proto=S.PROTO_SIMPLE, work=None):
    """Per-rank expected outputs; inputs[r] has n*recvcount elements.  Rank
    r's block is folded on the ring of each element's channel (VCCL's cbd
    partition of the recvcount block), finishing at r."""
    n = len(inputs)
    rings = rings or ring_orders(n)
    dev_op, arg = O.host_to_dev_redop(op, dtype, n)
    pre = dev_op == O.DEV_PREMULSUM
    count = inputs[0].size // n
    if work is None:
        work = _sched("rs", count, inputs[0].dtype.itemsize, n, nch, slot_bytes, nthreads, proto)
    chan = S.channel_of(work, count)
    outs = [np.empty(count, inputs[0].dtype) for _ in range(n)]
    for c in range(work.channel_lo, work.channel_hi + 1):
        idx = np.nonzero(chan == c)[0]
        if idx.size == 0:
            continue
        ring = rings[c % len(rings)]
        for r in range(n):
            ins = [inputs[q][r * count + idx] for q in ring]
            own = np.full(idx.size, ring.index(r), np.int32)
            outs[r][idx] = O.ring_fold(dev_op, dtype, arg, pre, ins, own)
    return outs


def expected_reduce(op, dtype, inputs, root, nch, slot_bytes=512 << 10, rings=None, nthreads=512,
                    proto=S.PROTO_SIMPLE, work=None):
    """Expected output of the ring reduce on `root` (reduce.h:12-55): each
    element's channel (VCCL's cbd partition of the call, REDUCE_CHUNKSTEPS 1)
    picks its ring; the fold starts at root's successor and ends at root with
    postOp — the reduce-scatter fold of the block root owns."""
    n = len(inputs)
    rings = rings or ring_orders(n)
    dev_op, arg = O.host_to_dev_redop(op, dtype, n)
    pre = dev_op == O.DEV_PREMULSUM
    count = inputs[0].size
    if work is None:
        work = _sched("red", count, inputs[0].dtype.itemsize, n, nch, slot_bytes, nthreads, proto)
    chan = S.channel_of(work, count)
    out = np.empty(count, inputs[0].dtype)
    for c in range(work.channel_lo, work.channel_hi + 1):
        idx = np.nonzero(chan == c)[0]
        if idx.size == 0:
            continue
        ring = rings[c % len(rings)]
        ins = [inputs[q][idx] for q in ring]
        out[idx] = O.ring_fold(dev_op, dtype, arg, pre, ins, np.full(idx.size, ring.index(root), np.int32))
    return out


def direct_shard_elts(count, n, elt_size):
    """Shard length of one chunk of the two-shot direct all-reduce
    (direct.hpp direct_shard_elts): ceil(count / n) rounded up to 16 bytes."""
    return _align_up(_div_up(count, n), max(1, 16 // elt_size))


def direct_chunk_elts(count, n, elt_size, chunk_bytes=16 << 20):
    """Elements per chunk (host/init.cc inbox region, host/enqueue.cc launch_direct)."""
    region = (chunk_bytes + n - 1) // n // 256 * 256 + 256
    unit = n * max(1, 16 // elt_size)
    return min(count, (region - 16) // elt_size * n // unit * unit)
