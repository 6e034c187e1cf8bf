"""ORACLE — test infrastructure only (tests/ may import it; the product never does).

Restatement of VCCL's channel partition and chunking for the RING collectives,
i.e. which channel (hence which ring) and which chunk of which loop every
element of an all-reduce / reduce-scatter / all-gather lands in.  With the
per-channel ring, that fixes the fp fold order of every element, so together
with the C oracle's ring_fold (oracle/reduce_ref.c) it gives VCCL's exact
result for a given (ring set, channel count, buffer size).

Followed, for a plan holding one collective (the ncclAllReduce /
ncclReduceScatter / ncclAllGather call outside a group; plan_schedule below
restates the multi-task plan of a group):
  * taskAppend: AG counted in bytes as int8 (enqueue.cc:2398-2404);
    trafficBytes = count * eltSize * trafficPerByte (enqueue.cc:2405,
    ncclFuncTrafficPerByte enqueue.cc:67-74: AR 2, RS/AG nRanks)
  * topoGetAlgoInfo ring channel tuning: nc = comm nChannels, decreased while
    nBytes < nc * nt * threadThreshold (enqueue.cc:1902-1925), nBytes =
    eltSize * ncclFuncMaxSendRecvCount (enqueue.cc:1955, enqueue.h:36-38),
    nt = maxThreads[RING][proto] (tuning.cc:198-211: SIMPLE 512 unless the ring
    is PCI-bound, LL 512, LL128 640), threadThreshold SIMPLE 64 / LL 8 * nRanks
    / LL128 8 (comm.h:38-40, tuning.cc:489-493)
  * scheduleCollTasksToPlan, the cbd cell split (enqueue.cc:518-565, 597-644)
  * calcCollChunking for RING (enqueue.cc:1983-2093): chunkSize = stepSize *
    chunkSteps (SIMPLE ring: 4 steps of buffSize/8, collectives.h:16-22), LL
    halves it, LL128 keeps 15/16, rounded down to the protocol grain
    (device.h:290-295: SIMPLE 512 B, LL 16 B, LL128 1920 B)
  * ncclCollCbdPart (device.h:297-323) and the per-loop chunk layout of
    runRing all-reduce with the short last loop's alignUp(divUp(rem, nranks),
    16/sizeof(T)) (all_reduce.h:32-47), reduce-scatter (reduce_scatter.h:33-36)
    and all-gather (all_gather.h:43-46).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

PROTO_LL, PROTO_LL128, PROTO_SIMPLE = 0, 1, 2   # nccl_common.h protocol ids
NCCL_STEPS = 8                                   # device.h:24
MIN_TRAFFIC_PER_CHANNEL = 16 << 10               # enqueue.cc:528
DEFAULT_BUFFSIZE = {PROTO_LL: 8 * 512 * NCCL_STEPS * 16,        # init.cc:617
                    PROTO_LL128: 120 * 640 * NCCL_STEPS * 8,    # init.cc:618
                    PROTO_SIMPLE: 1 << 22}                      # init.cc:619
MAX_THREADS = {PROTO_LL: 512, PROTO_LL128: 640, PROTO_SIMPLE: 512}
THREAD_THRESHOLD = {PROTO_LL: 8, PROTO_LL128: 8, PROTO_SIMPLE: 64}
CHUNK_STEPS = 4                                  # ALLREDUCE/REDUCESCATTER/ALLGATHER_CHUNKSTEPS
LL128_LINEELEMS, LL128_DATAELEMS = 16, 15        # device.h:81-83


def grain_size(proto):
    """ncclProtoGrainSize (device.h:290-295); LL128 = 32 * 16 / 16 * 15 * 8."""
    return {PROTO_LL: 16, PROTO_LL128: 1920, PROTO_SIMPLE: 512}[proto]


def _div_up(x, y):
    return (x + y - 1) // y


def _align_up(x, a):
    return _div_up(x, a) * a


@dataclass
class CbdWork:
    """ncclDevWorkColl.cbd + channel range (device.h:258-287)."""
    channel_lo: int
    channel_hi: int
    count_lo: int
    count_mid: int
    count_hi: int
    chunk_grains_lo: int
    chunk_grains_mid: int
    chunk_grains_hi: int
    proto: int
    elt_size: int

    def part(self, channel):
        """ncclCollCbdPart: (partOffset, partCount, chunkCount) in elements."""
        per_grain = grain_size(self.proto) // self.elt_size
        n_mid = self.channel_hi - self.channel_lo - 1
        if channel == self.channel_lo:
            return 0, self.count_lo, self.chunk_grains_lo * per_grain
        if channel == self.channel_hi:
            return (self.count_lo + n_mid * self.count_mid, self.count_hi,
                    self.chunk_grains_hi * per_grain)
        mid = channel - self.channel_lo - 1
        return self.count_lo + mid * self.count_mid, self.count_mid, self.chunk_grains_mid * per_grain


def traffic_per_byte(coll, nranks):
    """ncclFuncTrafficPerByte (enqueue.cc:67-74): AR 2, RS / AG nRanks, else
    (broadcast "bc", reduce "red") 1."""
    return 2 if coll == "ar" else 1 if coll in ("bc", "red") else nranks


def max_send_recv_count(coll, nranks, count):
    return nranks * count if coll in ("ag", "rs") else count  # AR / broadcast / reduce: count


def chunk_size(proto, buff_size=None, coll="ar"):
    """calcCollChunking for the RING algorithm (enqueue.cc:2027-2032, 2093);
    broadcast / reduce: BROADCAST_CHUNKSTEPS / REDUCE_CHUNKSTEPS 1
    (collectives.h:23-26)."""
    buff = DEFAULT_BUFFSIZE[proto] if buff_size is None else buff_size
    step = buff // NCCL_STEPS
    cs = step * (CHUNK_STEPS if proto == PROTO_SIMPLE and coll not in ("bc", "red") else 1)
    if proto == PROTO_LL:
        cs //= 2
    if proto == PROTO_LL128:
        cs = cs // LL128_LINEELEMS * LL128_DATAELEMS
    g = grain_size(proto)
    return cs // g * g


def ring_n_max_channels(coll, count, elt_size, nranks, comm_channels, proto=PROTO_SIMPLE,
                        nthreads=None):
    """topoGetAlgoInfo's ring / tree channel count for this call
    (enqueue.cc:1902-1925); LL's threshold is times nRanks on the ring
    (tuning.cc:493) — reduce-scatter / all-gather — not on the tree that
    carries VCCL's LL all-reduce."""
    nbytes = elt_size * max_send_recv_count(coll, nranks, count)
    nt = MAX_THREADS[proto] if nthreads is None else nthreads
    thr = THREAD_THRESHOLD[proto] * (nranks if proto == PROTO_LL and coll != "ar" else 1)
    nc = comm_channels
    while nbytes < nc * nt * thr:
        if nc >= 2:
            nc -= 1
        else:
            break
    return nc


def cbd_schedule(coll, count, elt_size, nranks, comm_channels, proto=PROTO_SIMPLE,
                 buff_size=None, nthreads=None) -> CbdWork:
    """scheduleCollTasksToPlan for a plan of one ring collective.

    coll: "ar" | "rs" | "ag" | "bc" | "red"; count: AR count, RS recvcount, AG
    sendcount, broadcast / reduce count (in elements of elt_size; AG and broadcast are
    rewritten to bytes here as taskAppend does)."""
    if coll in ("ag", "bc"):
        count, elt_size = count * elt_size, 1
    tpb = traffic_per_byte(coll, nranks)
    task_traffic = count * elt_size * tpb * (4 if proto == PROTO_LL else 1)   # enqueue.cc:418
    n_task_ch = ring_n_max_channels(coll, count, elt_size, nranks, comm_channels, proto, nthreads)
    traffic = max(MIN_TRAFFIC_PER_CHANNEL, task_traffic)
    n_ch = min(n_task_ch, comm_channels)
    n_max = comm_channels
    traffic_per_channel = max(MIN_TRAFFIC_PER_CHANNEL, traffic // n_ch)
    channel_id, current_traffic = 0, 0
    if proto == PROTO_LL:
        tpb *= 4
    cell_size = _div_up(_div_up(MIN_TRAFFIC_PER_CHANNEL, tpb), 16) * 16
    elements_per_cell = cell_size // elt_size
    cells = _div_up(count * elt_size, cell_size)
    traffic_per_cell = cell_size * tpb
    cells_per_channel = min(cells, _div_up(traffic_per_channel, traffic_per_cell))
    if channel_id + 1 == n_max:
        cells_lo = cells
    else:
        cells_lo = min(cells, _div_up(traffic_per_channel - current_traffic, traffic_per_cell))
    n_mid = (cells - cells_lo) // cells_per_channel
    cells_hi = (cells - cells_lo) % cells_per_channel
    n_channels = (1 if cells_lo else 0) + n_mid + (1 if cells_hi else 0)
    if n_max < channel_id + n_channels:
        n_mid = n_max - channel_id - 2
        cells_per_channel = (cells - cells_lo) // (n_mid + 1)
        cells_hi = cells_per_channel + (cells - cells_lo) % (n_mid + 1)
    if cells_hi == 0 and n_mid != 0:
        cells_hi = cells_per_channel
        n_mid -= 1
    if cells_lo == 0:
        channel_id += 1
        if n_mid == 0:
            cells_lo, cells_hi = cells_hi, 0
        else:
            cells_lo = cells_per_channel
            n_mid -= 1
    count_mid = cells_per_channel * elements_per_cell if n_mid != 0 else 0
    count_lo = cells_lo * elements_per_cell
    count_hi = cells_hi * elements_per_cell
    excess = cells * elements_per_cell - count
    if count_hi != 0:
        count_hi -= excess
    else:
        count_lo -= excess
    n_channels = (1 if count_lo else 0) + n_mid + (1 if cells_hi else 0)
    g = grain_size(proto)
    cs = chunk_size(proto, buff_size, coll)  # ring: independent of nBytes (enqueue.cc:2034-2082)
    grains = cs // g
    return CbdWork(channel_id, channel_id + n_channels - 1, count_lo, count_mid, count_hi,
                   grains if count_lo else 0, grains if n_mid else 0, grains if count_hi else 0,
                   proto, elt_size)


# ------------------------------------------------------------------ group plan
# VCCL's plan for a GROUP of collectives of one communicator (every call RING
# / SIMPLE unless `algo_of` gives each aggregate its path):
#   * taskAppend (enqueue.cc:2398-2413): AG as int8 bytes, trafficBytes =
#     count * eltSize * trafficPerByte, inserted into ncclTaskCollSorter;
#   * the sorter (comm.h:294-343): bin = BinCount-1 - u32fpEncode(min(size,
#     1 GiB) >> 10, 2) (bitops.h:252-262), bins walked in ascending index
#     (descending size), each bin's tasks newest first;
#   * ncclPrepareTasks (enqueue.cc:352-437): pushed onto one LIFO per
#     (func, devOp, type) -> each list size-ascending, lists in order of first
#     appearance; runs within 4x of the run's first trafficBytes aggregated,
#     the aggregate's path (getAlgoInfo, :398 — here `algo_of`, the library's
#     selection standing in for VCCL's tuner) and nMaxChannels from the
#     channel tuning on the aggregate's count, both given to every member;
#     an LL member's trafficBytes x4 (:418);
#   * scheduleCollTasksToPlan (enqueue.cc:518-769): per plan, the tasks that
#     pass the work-budget estimate give trafficPerChannel = sum(max(16K,
#     traffic)) / min(sum nMaxChannels, comm channels); every task is split
#     into cells at the running (channelId, currentTraffic); a task whose
#     channels would exceed the argument budget (testBudget :278-286, work
#     batches counted as addWorkBatchToPlan :91-156) ends the plan.
U32FP_BITS, SORTER_UNIT_LOG2, SORTER_MAX_LOG2 = 2, 10, 30
SORTER_BINS = 1 + (SORTER_MAX_LOG2 - SORTER_UNIT_LOG2) * (1 << U32FP_BITS)
WORK_COLL_BYTES, WORK_BATCH_BYTES = 96, 16           # sizeof(ncclDevWorkColl / ncclDevWorkBatch)
IN_ARGS_BYTES = (4 << 10) - 32                        # workArgsBytes - sizeof(ncclDevKernelArgs)
OUT_ARGS_BYTES = (1 << 20) // 2                       # NCCL_WORK_FIFO_BYTES default / 2
MAX_BATCH_BYTES = 1024                                # NCCL_MAX_DEV_WORK_BATCH_BYTES


def u32fp_encode(x, bits):
    """bitops.h:252-262."""
    log2x = (x | 1).bit_length() - 1
    mant = (x >> (log2x - bits if log2x >= bits else 0)) & ((1 << bits) - 1)
    expo = log2x - (bits - 1) if log2x >= bits else 0
    return (expo << bits) | mant


@dataclass
class GroupCall:
    """One queued collective: coll "ar"|"rs"|"ag"|"bc"|"red", count (AR /
    broadcast / reduce count, RS recvcount, AG sendcount) in elements of elt_size; key = (func, devOp,
    type) of ncclPrepareTasks' bins; func = the device function (batches of a
    channel merge while it is the same)."""
    coll: str
    count: int
    elt_size: int
    key: tuple
    func: tuple


def _place(cur, coll, count, elt_size, nranks, proto, buff_size):
    """One task's cbd split at the plan cursor (enqueue.cc:597-644; LL traffic
    x4, :599) and the cursor advanced (:667-681).  cur = dict(tpc, ch, cur,
    nmax)."""
    tpb = traffic_per_byte(coll, nranks) * (4 if proto == PROTO_LL else 1)
    cell = _div_up(_div_up(MIN_TRAFFIC_PER_CHANNEL, tpb), 16) * 16
    epc = cell // elt_size
    cells = _div_up(count * elt_size, cell)
    tpe = elt_size * tpb
    tpcell = cell * tpb
    tpc, ch, used, nmax = cur["tpc"], cur["ch"], cur["cur"], cur["nmax"]
    per_ch = min(cells, _div_up(tpc, tpcell))
    lo = cells if ch + 1 == nmax else min(cells, _div_up(tpc - used, tpcell))
    n_mid = (cells - lo) // per_ch
    hi = (cells - lo) % per_ch
    n_ch = (1 if lo else 0) + n_mid + (1 if hi else 0)
    if nmax < ch + n_ch:
        n_mid = nmax - ch - 2
        per_ch = (cells - lo) // (n_mid + 1)
        hi = per_ch + (cells - lo) % (n_mid + 1)
    if hi == 0 and n_mid != 0:
        hi, n_mid = per_ch, n_mid - 1
    if lo == 0:
        ch += 1
        if n_mid == 0:
            lo, hi = hi, 0
        else:
            lo, n_mid = per_ch, n_mid - 1
    c_mid = per_ch * epc if n_mid else 0
    c_lo, c_hi = lo * epc, hi * epc
    excess = cells * epc - count
    if c_hi:
        c_hi -= excess
    else:
        c_lo -= excess
    n_ch = (1 if c_lo else 0) + n_mid + (1 if hi else 0)
    grains = chunk_size(proto, buff_size, coll) // grain_size(proto)
    work = CbdWork(ch, ch + n_ch - 1, c_lo, c_mid, c_hi, grains if c_lo else 0, grains if n_mid else 0,
                   grains if c_hi else 0, proto, elt_size)
    if c_hi:
        ch, used = ch + n_ch - 1, hi * epc * tpe
    elif n_mid:
        ch, used = ch + n_ch, 0
    else:
        used += lo * epc * tpe
    if used >= tpc and ch + 1 != nmax:
        ch, used = ch + 1, 0
    return work, dict(tpc=tpc, ch=ch, cur=used, nmax=nmax)


ALGO_PROTO = {"ring": PROTO_SIMPLE, "direct": PROTO_SIMPLE, "ll": PROTO_LL, "ll128": PROTO_LL128}


def plan_schedule(calls, nranks, comm_channels, buff_size=None, nthreads=None, algo_of=None,
                  ll128_buff=None, ll128_threads=None, algos_out=None):
    """VCCL's plans for a group of calls.  Returns (order, plan_of, works):
    the calls in execution order, the plan (kernel) index of every call, and
    every call's CbdWork (indexed like `calls`).

    algo_of(i, agg_count) -> "ring" | "direct" | "ll" | "ll128": the path of
    the aggregate headed by call i with agg_count elements in total (AG in
    bytes); None = every call "ring".  The direct path is placed as a SIMPLE
    ring call, "ll" as VCCL's LL (tree for the all-reduce, ring otherwise),
    "ll128" as the LL128 ring (ll128_buff / ll128_threads: VCCL's defaults).
    algos_out (a list) receives every call's path."""
    calls = [GroupCall(c.coll, c.count * c.elt_size, 1, c.key, c.func) if c.coll in ("ag", "bc") else c
             for c in calls]
    traffic = [c.count * c.elt_size * traffic_per_byte(c.coll, nranks) for c in calls]
    bins = [[] for _ in range(SORTER_BINS)]
    for i, t in enumerate(traffic):
        x = min(t, 1 << SORTER_MAX_LOG2) >> SORTER_UNIT_LOG2
        bins[SORTER_BINS - 1 - u32fp_encode(x, U32FP_BITS)].append(i)
    sorted_ = [i for b in bins for i in reversed(b)]
    by_key = {}
    for i in sorted_:
        by_key.setdefault(calls[i].key, []).insert(0, i)   # dicts keep first-appearance order
    nmax, proto, algo, queue = {}, {}, {}, []
    for lst in by_key.values():
        a = 0
        while a < len(lst):
            e, agg = a + 1, calls[lst[a]].count
            while e < len(lst) and traffic[lst[e]] < 4 * traffic[lst[a]]:
                agg += calls[lst[e]].count
                e += 1
            c0 = calls[lst[a]]
            path = algo_of(lst[a], agg) if algo_of is not None else "ring"
            pr = ALGO_PROTO[path]
            nt = (ll128_threads or MAX_THREADS[PROTO_LL128]) if pr == PROTO_LL128 else nthreads
            nc = ring_n_max_channels(c0.coll, agg, c0.elt_size, nranks, comm_channels, pr, nt)
            for j in lst[a:e]:
                nmax[j], proto[j], algo[j] = nc, pr, path
                if pr == PROTO_LL:
                    traffic[j] *= 4
            a = e
        queue += lst
    if algos_out is not None:
        algos_out[:] = [algo[i] for i in range(len(calls))]
    buffs = {PROTO_SIMPLE: buff_size, PROTO_LL: None, PROTO_LL128: ll128_buff}

    def budget_ok(n_batches, work_bytes):
        bb = n_batches * WORK_BATCH_BYTES
        return bb + work_bytes <= IN_ARGS_BYTES or (bb <= IN_ARGS_BYTES and work_bytes <= OUT_ARGS_BYTES)

    plan_of, works = [None] * len(calls), [None] * len(calls)
    head, plan = 0, 0
    while head < len(queue):
        n_plan, tb, nch, wb = 0, 0, 0, 0
        for i in queue[head:]:
            if not budget_ok(_div_up(n_plan, 4), wb + WORK_COLL_BYTES):
                break
            n_plan += 1
            wb += WORK_COLL_BYTES
            tb += max(MIN_TRAFFIC_PER_CHANNEL, traffic[i])
            nch = min(nch + nmax[i], comm_channels)
        cur = dict(tpc=max(MIN_TRAFFIC_PER_CHANNEL, tb // nch), ch=0, cur=0, nmax=comm_channels)
        batch = {}                        # channel -> [func, offsetBase, wipBytes]
        n_batches = work_bytes = 0
        while n_plan and head < len(queue):
            i = queue[head]
            c = calls[i]
            w, nxt = _place(cur, c.coll, c.count, c.elt_size, nranks, proto[i], buffs[proto[i]])
            if not budget_ok(n_batches + w.channel_hi - w.channel_lo + 1, work_bytes + WORK_COLL_BYTES):
                break
            cur = nxt
            for ch in range(w.channel_lo, w.channel_hi + 1):
                b = batch.get(ch)
                fn = (c.func, proto[i])   # devFuncId: (func, op, type, algo, proto)
                new = b is None or b[0] != fn or b[2] + WORK_COLL_BYTES > MAX_BATCH_BYTES
                off = 0 if new else work_bytes - b[1]
                if new or 63 * WORK_COLL_BYTES < off:
                    b = [fn, work_bytes, 0 if new else b[2]]
                    n_batches += 1
                b[0] = fn
                b[2] += WORK_COLL_BYTES
                batch[ch] = b
            work_bytes += WORK_COLL_BYTES
            plan_of[i], works[i] = plan, w
            head += 1
            n_plan -= 1
        plan += 1
    return queue, plan_of, works


def allreduce_owner(work: CbdWork, count, nranks):
    """Per element: (channel, ring index of the rank that finishes it) for the
    ring all-reduce (all_reduce.h:32-64: chunk k of every loop finishes at
    ring index k)."""
    chan = np.full(count, -1, np.int32)
    owner = np.full(count, -1, np.int32)
    elt_align = max(1, 16 // work.elt_size)
    for c in range(work.channel_lo, work.channel_hi + 1):
        off, length, chunk = work.part(c)
        loop = nranks * chunk
        eo = 0
        while eo < length:
            rem = length - eo
            if rem < loop:
                chunk = _align_up(_div_up(rem, nranks), elt_align)
            for k in range(nranks):
                lo = eo + k * chunk
                hi = min(eo + (k + 1) * chunk, length)
                if hi > lo:
                    chan[off + lo:off + hi] = c
                    owner[off + lo:off + hi] = k
            eo += loop
    assert (chan >= 0).all(), "partition does not cover the buffer"
    return chan, owner


def channel_of(work: CbdWork, count):
    """Per element of a reduce-scatter block / all-gather block: its channel."""
    chan = np.full(count, -1, np.int32)
    for c in range(work.channel_lo, work.channel_hi + 1):
        off, length, _ = work.part(c)
        chan[off:off + length] = c
    assert (chan >= 0).all(), "partition does not cover the block"
    return chan


def allreduce_owner_at(work: CbdWork, count, nranks, idx):
    """allreduce_owner for selected elements only (sampled windows of
    buffers too large for the full map): (channel, finishing ring index) of
    every index in `idx`."""
    idx = np.asarray(idx, dtype=np.int64)
    chan = np.full(idx.size, -1, np.int32)
    owner = np.full(idx.size, -1, np.int32)
    elt_align = max(1, 16 // work.elt_size)
    for c in range(work.channel_lo, work.channel_hi + 1):
        off, length, chunk = work.part(c)
        sel = (idx >= off) & (idx < off + length)
        if not sel.any():
            continue
        local = idx[sel] - off
        loop = nranks * chunk
        n_full = length // loop
        tail0 = n_full * loop            # start of the short last loop (if any)
        k = (local % loop) // chunk
        rem = length - tail0
        if rem > 0:
            short = _align_up(_div_up(rem, nranks), elt_align)
            in_tail = local >= tail0
            k = np.where(in_tail, (local - tail0) // short, k)
        chan[sel] = c
        owner[sel] = k
    assert (chan >= 0).all(), "index outside the partition"
    return chan, owner
