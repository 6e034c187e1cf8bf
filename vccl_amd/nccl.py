"""ctypes binding of libvccl.so's C ABI (include/nccl.h, include/vccl_device.h).

This is the binding a Python caller of the reference would write against
libnccl (same function names, enum values, argument order and error codes —
see INTEGRATION.md).  It loads the in-tree ``vccl_amd/lib/libvccl.so`` and
raises ``VcclError`` if the library is missing: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import time
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VCCL_LIB") or os.path.join(_HERE, "lib", "libvccl.so")

# ncclResult_t (nccl.h.in:40-48)
ncclSuccess, ncclUnhandledCudaError, ncclSystemError, ncclInternalError = 0, 1, 2, 3
ncclInvalidArgument, ncclInvalidUsage, ncclRemoteError, ncclInProgress = 4, 5, 6, 7
# ncclRedOp_t (nccl.h.in:221-236)
ncclSum, ncclProd, ncclMax, ncclMin, ncclAvg = 0, 1, 2, 3, 4
# ncclDataType_t (nccl.h.in:239-252)
ncclInt8, ncclUint8, ncclInt32, ncclUint32, ncclInt64, ncclUint64 = 0, 1, 2, 3, 4, 5
ncclFloat16, ncclFloat32, ncclFloat64, ncclBfloat16 = 6, 7, 8, 9
ncclFloat8e4m3, ncclFloat8e5m2, ncclNumTypes = 10, 11, 12
# ncclScalarResidence_t
ncclScalarDevice, ncclScalarHostImmediate = 0, 1
# vcclDevRedOp_t (include/vccl_device.h)
vcclDevSum, vcclDevProd, vcclDevMinMax, vcclDevPreMulSum, vcclDevSumPostDiv = 0, 1, 2, 3, 4
vcclDevCopy = 15

TYPE_SIZE = {0: 1, 1: 1, 2: 4, 3: 4, 4: 8, 5: 8, 6: 2, 7: 4, 8: 8, 9: 2, 10: 1, 11: 1}

# Every symbol include/*.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "ncclGetVersion", "ncclGetUniqueId", "ncclCommInitRankConfig", "ncclCommInitRank",
    "ncclCommInitAll", "ncclCommFinalize", "ncclCommDestroy", "ncclCommAbort",
    "ncclGetErrorString", "ncclGetLastError", "ncclCommGetAsyncError", "ncclCommCount",
    "ncclCommCuDevice", "ncclCommUserRank", "ncclRedOpCreatePreMulSum", "ncclRedOpDestroy",
    "ncclAllReduce", "ncclReduceScatter", "ncclAllGather", "ncclGroupStart", "ncclGroupEnd",
    "vcclReduceCopy", "vcclReduceCopyEx", "vcclHostToDevRedOp", "vcclKernelTypeOf",
    "vcclBuildInfo", "vcclBootstrapAllGather", "vcclCommCollAlgo", "vcclCommSetAlgo",
    "vcclCommLaunchStats", "vcclCommNetStats", "vcclCommSetFences", "vcclCommDebugSetEpochs",
    "vcclCommSetRingWave", "vcclCommRingTrace", "vcclCommGroupAlgos",
    "vcclRingPartition", "vcclRingChunkOf", "vcclRingOrders", "vcclGroupPlan", "vcclGroupPlanEx", "vcclAlgoSelection",
    # rooted rings, split and debug reload
    "ncclReduce", "ncclBcast", "ncclBroadcast", "ncclCommSplit", "ncclResetDebugInit",
    # out of scope, exported so libnccl-linked binaries load: WARN + ncclInvalidUsage
    "ncclSend", "ncclRecv", "ncclGroupSimulateEnd", "ncclAllToAll", "ncclAllToAllv",
    # memory / registration / scalable init (what a libnccl caller such as
    # PyTorch's nccl backend imports)
    "ncclMemAlloc", "ncclMemFree", "ncclCommInitRankScalable", "ncclCommRegister", "ncclCommDeregister",
]
ALGO_NAMES = {0: "ring", 1: "ll", 2: "direct", 3: "one_rank", 4: "ll128"}


class VcclError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = lib().ncclGetErrorString(code).decode() if _lib is not None else str(code)
        super().__init__(f"{what}: {msg} (ncclResult_t={code})")


class ncclUniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


class vcclLaunchConfig(ctypes.Structure):
    _fields_ = [("blockSize", ctypes.c_int), ("unroll", ctypes.c_int),
                ("gridBlocks", ctypes.c_int), ("ntLoads", ctypes.c_int),
                ("ntStores", ctypes.c_int), ("order", ctypes.c_int)]


class ncclConfig_t(ctypes.Structure):
    """nccl.h.in:57-85 (include/nccl.h), filled as NCCL_CONFIG_INITIALIZER."""
    _fields_ = [("size", ctypes.c_size_t), ("magic", ctypes.c_uint), ("version", ctypes.c_uint),
                ("blocking", ctypes.c_int), ("cgaClusterSize", ctypes.c_int), ("minCTAs", ctypes.c_int),
                ("maxCTAs", ctypes.c_int), ("netName", ctypes.c_void_p), ("splitShare", ctypes.c_int),
                ("trafficClass", ctypes.c_int)]

    @classmethod
    def initializer(cls, **kw) -> "ncclConfig_t":
        undef = -2147483648  # NCCL_CONFIG_UNDEF_INT
        c = cls(ctypes.sizeof(cls), 0xcafebeef, get_version(), undef, undef, undef, undef, None, undef, undef)
        for k, v in kw.items():
            setattr(c, k, v)
        return c


_lib = None


def last_error(comm=None) -> str:
    """ncclGetLastError: the last WARN's text (comm unused, may be None)."""
    return (lib().ncclGetLastError(comm) or b"").decode(errors="replace")


def lib() -> ctypes.CDLL:
    """Load libvccl.so (fails loudly if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `make -j8` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    c_int, c_size, vp, u64 = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint64
    pcomm = ctypes.POINTER(vp)
    sig = {
        "ncclGetVersion": [ctypes.POINTER(c_int)],
        "ncclGetUniqueId": [ctypes.POINTER(ncclUniqueId)],
        "ncclCommInitRank": [pcomm, c_int, ncclUniqueId, c_int],
        "ncclCommInitAll": [pcomm, c_int, ctypes.POINTER(c_int)],
        "ncclCommInitRankConfig": [pcomm, c_int, ncclUniqueId, c_int, ctypes.POINTER(ncclConfig_t)],
        "ncclCommFinalize": [vp],
        "ncclCommDestroy": [vp],
        "ncclCommAbort": [vp],
        "ncclCommGetAsyncError": [vp, ctypes.POINTER(c_int)],
        "ncclCommCount": [vp, ctypes.POINTER(c_int)],
        "ncclCommCuDevice": [vp, ctypes.POINTER(c_int)],
        "ncclCommUserRank": [vp, ctypes.POINTER(c_int)],
        "ncclRedOpCreatePreMulSum": [ctypes.POINTER(c_int), vp, c_int, c_int, vp],
        "ncclRedOpDestroy": [c_int, vp],
        "ncclAllReduce": [vp, vp, c_size, c_int, c_int, vp, vp],
        "ncclReduceScatter": [vp, vp, c_size, c_int, c_int, vp, vp],
        "ncclAllGather": [vp, vp, c_size, c_int, vp, vp],
        "ncclBroadcast": [vp, vp, c_size, c_int, c_int, vp, vp],
        "ncclReduce": [vp, vp, c_size, c_int, c_int, c_int, vp, vp],
        "ncclGroupStart": [],
        "ncclGroupEnd": [],
        "vcclReduceCopy": [c_int, c_int, u64, c_int, c_int, c_int, ctypes.POINTER(vp), c_int,
                           ctypes.POINTER(vp), c_size, vp],
        "vcclReduceCopyEx": [c_int, c_int, u64, c_int, c_int, c_int, ctypes.POINTER(vp), c_int,
                             ctypes.POINTER(vp), c_size, vp, ctypes.POINTER(vcclLaunchConfig)],
        "vcclHostToDevRedOp": [c_int, c_int, c_int, ctypes.POINTER(c_int), ctypes.POINTER(u64)],
        "vcclKernelTypeOf": [c_int, c_int],
        "vcclBootstrapAllGather": [ctypes.POINTER(ncclUniqueId), c_int, c_int, vp, c_size],
        "vcclCommSetFences": [vp, c_int],
        "vcclCommSetRingWave": [vp, c_int, ctypes.POINTER(ctypes.c_ulonglong)],
        "vcclRingPartition": [c_int, c_size, c_int, c_int, c_int, c_int, c_size, c_int,
                              ctypes.POINTER(ctypes.c_int64)],
        "vcclCommDebugSetEpochs": [vp, ctypes.c_uint32, ctypes.c_uint32],
        "vcclRingChunkOf": [c_size, c_int, c_int, c_int, c_size, c_int, c_size,
                            ctypes.POINTER(ctypes.c_int64)],
        "vcclRingOrders": [c_int, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int)],
        "vcclGroupPlan": [c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_size), ctypes.POINTER(c_int),
                          ctypes.POINTER(c_int), c_int, c_int, c_size, c_int, ctypes.POINTER(c_int),
                          ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_int64)],
        "vcclGroupPlanEx": [c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_size), ctypes.POINTER(c_int),
                            ctypes.POINTER(c_int), c_int, c_int, ctypes.POINTER(ctypes.c_int64),
                            ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                            ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_int64)],
        "vcclCommGroupAlgos": [vp, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_size), ctypes.POINTER(c_int),
                               ctypes.POINTER(c_int), ctypes.POINTER(c_int)],
        "vcclAlgoSelection": [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(c_int),
                              ctypes.POINTER(c_int)],
    }
    for name, args in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = c_int
    L.ncclGetErrorString.argtypes = [c_int]
    L.ncclGetErrorString.restype = ctypes.c_char_p
    for name in ("ncclGetLastError", "pncclGetLastError"):
        getattr(L, name).argtypes = [vp]
        getattr(L, name).restype = ctypes.c_char_p
    L.vcclBuildInfo.argtypes = []
    L.vcclBuildInfo.restype = ctypes.c_char_p
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc != ncclSuccess:
        raise VcclError(rc, what)


def get_version() -> int:
    v = ctypes.c_int()
    check(lib().ncclGetVersion(ctypes.byref(v)), "ncclGetVersion")
    return v.value


def get_unique_id() -> ncclUniqueId:
    uid = ncclUniqueId()
    check(lib().ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
    return uid


def unique_id_to_bytes(uid: ncclUniqueId) -> bytes:
    return ctypes.string_at(ctypes.addressof(uid), 128)  # .internal stops at the first NUL


def unique_id_from_bytes(b: bytes) -> ncclUniqueId:
    uid = ncclUniqueId()
    ctypes.memmove(ctypes.byref(uid), b, 128)
    return uid


def bootstrap_allgather(uid: ncclUniqueId, rank: int, nranks: int, mine: bytes) -> list[bytes]:
    """One all-gather round over the TCP rendezvous (host only)."""
    n = len(mine)
    buf = ctypes.create_string_buffer(n * nranks)
    ctypes.memmove(ctypes.addressof(buf) + rank * n, mine, n)
    check(lib().vcclBootstrapAllGather(ctypes.byref(uid), rank, nranks, buf, n),
          "vcclBootstrapAllGather")
    raw = buf.raw
    return [raw[i * n:(i + 1) * n] for i in range(nranks)]


def host_to_dev_redop(op: int, dtype: int, nranks: int) -> tuple[int, int]:
    d, a = ctypes.c_int(), ctypes.c_uint64()
    check(lib().vcclHostToDevRedOp(op, dtype, nranks, ctypes.byref(d), ctypes.byref(a)),
          "vcclHostToDevRedOp")
    return d.value, a.value


def kernel_type_of(dev_op: int, dtype: int) -> int:
    return lib().vcclKernelTypeOf(dev_op, dtype)


PROTO_LL128, PROTO_SIMPLE = 1, 2


def ring_partition(coll: int, count: int, dtype: int, nranks: int, nchannels: int,
                   slot_bytes: int, nthreads: int = 512, proto: int = PROTO_SIMPLE) -> tuple[int, ...]:
    """vcclRingPartition: (channelLo, channelHi, countLo, countMid, countHi,
    chunkLo, chunkMid, chunkHi) of the ring's cbd partition (host only);
    slot_bytes = the protocol's FIFO step, nthreads = NCCL_NTHREADS (SIMPLE)
    or NCCL_LL128_NTHREADS (LL128)."""
    out = (ctypes.c_int64 * 8)()
    check(lib().vcclRingPartition(coll, count, dtype, nranks, nchannels, proto, slot_bytes, nthreads,
                                  out),
          "vcclRingPartition")
    return tuple(out)


def ring_orders(nranks: int) -> list[list[int]]:
    """vcclRingOrders: the library's ring set for nranks ranks."""
    out = (ctypes.c_int * (16 * nranks))()
    nr = ctypes.c_int()
    check(lib().vcclRingOrders(nranks, 16, out, ctypes.byref(nr)), "vcclRingOrders")
    return [list(out[k * nranks:(k + 1) * nranks]) for k in range(nr.value)]


def ring_chunk_of(count: int, dtype: int, nranks: int, nchannels: int, slot_bytes: int,
                  i: int, nthreads: int = 512) -> tuple[int, int, int]:
    """vcclRingChunkOf: (channel, ring chunk c, chunk end) of all-reduce
    element i on the ring's partition (the direct all-reduce's fold lookup)."""
    out = (ctypes.c_int64 * 3)()
    check(lib().vcclRingChunkOf(count, dtype, nranks, nchannels, slot_bytes, nthreads, i, out),
          "vcclRingChunkOf")
    return tuple(out)


def group_plan(calls, nranks: int, nchannels: int, slot_bytes: int = 512 << 10,
               nthreads: int = 512):
    """vcclGroupPlan: VCCL's multi-task plan of a group of ring / direct calls.
    calls = [(coll, count, dtype, op)]; returns (order, plan_of, parts) with
    parts[i] = (channelLo, channelHi, countLo, countMid, countHi, chunkLo,
    chunkMid, chunkHi) as ring_partition gives it."""
    n = len(calls)
    ci = ctypes.c_int * n
    colls, dts, ops = ci(*[c[0] for c in calls]), ci(*[c[2] for c in calls]), ci(*[c[3] for c in calls])
    counts = (ctypes.c_size_t * n)(*[c[1] for c in calls])
    order, plan_of = ci(), ci()
    cbd = (ctypes.c_int64 * (8 * n))()
    check(lib().vcclGroupPlan(n, colls, counts, dts, ops, nranks, nchannels, slot_bytes, nthreads, order,
                              plan_of, cbd), "vcclGroupPlan")
    return list(order), list(plan_of), [tuple(cbd[8 * i:8 * i + 8]) for i in range(n)]


POLICY_FIELDS = ("force", "ll_slot", "ll_max", "ll_rsag_max", "ll128", "ll128_min", "ll128_max", "direct",
                 "direct_max", "direct_rsag_max")


def group_plan_ex(calls, nranks: int, nchannels: int, policy: dict | None, slot_bytes: int = 512 << 10,
                  nthreads: int = 512, ll128_step: int = 120 * 640 * 8, ll128_threads: int = 640):
    """vcclGroupPlanEx: the plan a comm lays a group out on — a path per
    aggregate from `policy` (POLICY_FIELDS; None = every call on the SIMPLE
    ring).  Returns (algos, order, plan_of, parts), algos as ALGO_NAMES."""
    n = len(calls)
    ci = ctypes.c_int * n
    colls, dts, ops = ci(*[c[0] for c in calls]), ci(*[c[2] for c in calls]), ci(*[c[3] for c in calls])
    counts = (ctypes.c_size_t * n)(*[c[1] for c in calls])
    geo = (ctypes.c_int64 * 4)(slot_bytes, nthreads, ll128_step, ll128_threads)
    pol = None if policy is None else (ctypes.c_int64 * 10)(*[int(policy[k]) for k in POLICY_FIELDS])
    algos, order, plan_of = ci(), ci(), ci()
    cbd = (ctypes.c_int64 * (8 * n))()
    check(lib().vcclGroupPlanEx(n, colls, counts, dts, ops, nranks, nchannels, geo, pol, algos, order, plan_of,
                                cbd), "vcclGroupPlanEx")
    return ([ALGO_NAMES[a] for a in algos], list(order), list(plan_of),
            [tuple(cbd[8 * i:8 * i + 8]) for i in range(n)])


def algo_selection(algo: str | None, proto: str | None) -> tuple[int, int]:
    """vcclAlgoSelection: (force, allowed mask) for NCCL_ALGO / NCCL_PROTO strings."""
    f, a = ctypes.c_int(), ctypes.c_int()
    check(lib().vcclAlgoSelection(algo.encode() if algo is not None else None,
                                  proto.encode() if proto is not None else None, ctypes.byref(f),
                                  ctypes.byref(a)), "vcclAlgoSelection")
    return f.value, a.value


def reduce_copy(dev_op: int, dtype: int, red_arg: int, srcs, dsts, n_elts: int, stream: int = 0,
                pre_op_srcs: int = 0, post_op: bool = False, config: dict | None = None) -> None:
    """vcclReduceCopy on raw device pointers (ints)."""
    s = (ctypes.c_void_p * len(srcs))(*srcs)
    d = (ctypes.c_void_p * len(dsts))(*dsts)
    if config:
        cfg = vcclLaunchConfig(**config)
        rc = lib().vcclReduceCopyEx(dev_op, dtype, red_arg, pre_op_srcs, int(post_op), len(srcs),
                                    s, len(dsts), d, n_elts, stream, ctypes.byref(cfg))
    else:
        rc = lib().vcclReduceCopy(dev_op, dtype, red_arg, pre_op_srcs, int(post_op), len(srcs), s,
                                  len(dsts), d, n_elts, stream)
    check(rc, "vcclReduceCopy")


class Comm:
    """Owning wrapper over ncclComm_t."""

    def __init__(self, handle: int):
        self.handle = ctypes.c_void_p(handle)

    @classmethod
    def init_rank(cls, nranks: int, uid: ncclUniqueId, rank: int, config: "ncclConfig_t | None" = None) -> "Comm":
        h = ctypes.c_void_p()
        if config is None:
            rc = lib().ncclCommInitRank(ctypes.byref(h), nranks, uid, rank)
        else:
            rc = lib().ncclCommInitRankConfig(ctypes.byref(h), nranks, uid, rank, ctypes.byref(config))
        if rc == ncclInProgress:  # a non-blocking comm: poll its state, as a caller must
            st = ctypes.c_int(ncclInProgress)
            while st.value == ncclInProgress:
                check(lib().ncclCommGetAsyncError(h, ctypes.byref(st)), "ncclCommGetAsyncError")
                if st.value == ncclInProgress:
                    time.sleep(1e-3)
            rc = st.value
        check(rc, "ncclCommInitRankConfig" if config is not None else "ncclCommInitRank")
        return cls(h.value)

    @classmethod
    def init_all(cls, devices: list[int]) -> list["Comm"]:
        n = len(devices)
        hs = (ctypes.c_void_p * n)()
        dl = (ctypes.c_int * n)(*devices)
        check(lib().ncclCommInitAll(hs, n, dl), "ncclCommInitAll")
        return [cls(hs[i]) for i in range(n)]

    def _q(self, fn, what):
        v = ctypes.c_int()
        check(fn(self.handle, ctypes.byref(v)), what)
        return v.value

    @property
    def count(self) -> int:
        return self._q(lib().ncclCommCount, "ncclCommCount")

    @property
    def rank(self) -> int:
        return self._q(lib().ncclCommUserRank, "ncclCommUserRank")

    @property
    def device(self) -> int:
        return self._q(lib().ncclCommCuDevice, "ncclCommCuDevice")

    def async_error(self) -> int:
        return self._q(lib().ncclCommGetAsyncError, "ncclCommGetAsyncError")

    def all_reduce(self, send: int, recv: int, count: int, dtype: int, op: int, stream: int = 0):
        check(lib().ncclAllReduce(send, recv, count, dtype, op, self.handle, stream), "ncclAllReduce")

    def reduce_scatter(self, send: int, recv: int, recvcount: int, dtype: int, op: int,
                       stream: int = 0):
        check(lib().ncclReduceScatter(send, recv, recvcount, dtype, op, self.handle, stream),
              "ncclReduceScatter")

    def all_gather(self, send: int, recv: int, sendcount: int, dtype: int, stream: int = 0):
        check(lib().ncclAllGather(send, recv, sendcount, dtype, self.handle, stream), "ncclAllGather")

    def broadcast(self, send: int, recv: int, count: int, dtype: int, root: int, stream: int = 0):
        check(lib().ncclBroadcast(send, recv, count, dtype, root, self.handle, stream), "ncclBroadcast")

    def reduce(self, send: int, recv: int, count: int, dtype: int, op: int, root: int, stream: int = 0):
        """ncclReduce (reduce.h ring): `count` elements reduced into root's `recv`."""
        check(lib().ncclReduce(send, recv, count, dtype, op, root, self.handle, stream), "ncclReduce")

    def coll_algo(self, coll: int, count: int, dtype: int) -> str:
        """vcclCommCollAlgo: "ring" | "ll" | "direct" | "ll128" | "one_rank" (coll 0 AR, 1 RS, 2 AG, 3 broadcast, 4 reduce)."""
        a = ctypes.c_int()
        check(lib().vcclCommCollAlgo(self.handle, coll, ctypes.c_size_t(count), dtype,
                                     ctypes.byref(a)), "vcclCommCollAlgo")
        return ALGO_NAMES[a.value]

    def group_algos(self, calls) -> list[str]:
        """vcclCommGroupAlgos: the path of every call of a group on this comm
        (its aggregate's); calls = [(coll 0 AR / 1 RS / 2 AG, count, dtype, op)]."""
        n = len(calls)
        ci = ctypes.c_int * n
        out = ci()
        check(lib().vcclCommGroupAlgos(self.handle, n, ci(*[c[0] for c in calls]),
                                       (ctypes.c_size_t * n)(*[c[1] for c in calls]), ci(*[c[2] for c in calls]),
                                       ci(*[c[3] for c in calls]), out), "vcclCommGroupAlgos")
        return [ALGO_NAMES[a] for a in out]

    def split(self, color: int, key: int):
        """ncclCommSplit: the new communicator of this rank's color (None for
        NCCL_SPLIT_NOCOLOR = -1).  Collective over this comm."""
        h = ctypes.c_void_p()
        check(lib().ncclCommSplit(self.handle, color, key, ctypes.byref(h), None), "ncclCommSplit")
        return Comm(h.value) if h.value else None

    def set_algo(self, algo: str | None):
        """vcclCommSetAlgo: force "ring" | "ll" | "direct" | "ll128" for later calls; None = automatic."""
        code = -1 if algo is None else {v: k for k, v in ALGO_NAMES.items()}[algo]
        check(lib().vcclCommSetAlgo(self.handle, code), "vcclCommSetAlgo")

    def launch_stats(self) -> tuple[int, int]:
        """vcclCommLaunchStats: (collectives enqueued, fused group launches)."""
        a, b = ctypes.c_ulonglong(), ctypes.c_ulonglong()
        check(lib().vcclCommLaunchStats(self.handle, ctypes.byref(a), ctypes.byref(b)),
              "vcclCommLaunchStats")
        return a.value, b.value

    def n_channels(self) -> int:
        """The ring channel count of this communicator (vcclCommRingTrace's
        size query, which needs no trace buffer)."""
        nch = ctypes.c_int()
        lib().vcclCommRingTrace(self.handle, None, 0, ctypes.byref(nch), None)
        return nch.value

    def ring_trace(self):
        """vcclCommRingTrace: the SIMPLE ring's slot timeline of the last launch
        as a numpy structured array [nChannels, cap] (VCCL_RING_TRACE at init)."""
        import numpy as np
        nch, cap = ctypes.c_int(), ctypes.c_int()
        lib().vcclCommRingTrace(self.handle, None, 0, ctypes.byref(nch), ctypes.byref(cap))
        dt = np.dtype([("t0", "<u8"), ("t1", "<u8"), ("t2", "<u8"), ("t3", "<u8"), ("t4", "<u8"),
                       ("shape", "<u4"), ("bytes", "<u4"), ("step", "<u8"), ("tc", "<u8")])
        out = np.zeros((nch.value, cap.value), dtype=dt)
        check(lib().vcclCommRingTrace(self.handle, out.ctypes.data_as(ctypes.c_void_p),
                                      ctypes.c_size_t(out.nbytes), None, None), "vcclCommRingTrace")
        return out

    def net_stats(self) -> tuple[int, int, int]:
        """vcclCommNetStats: (bytes sent, bytes received, connections) of the net proxy."""
        a, b, n = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
        check(lib().vcclCommNetStats(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(n)),
              "vcclCommNetStats")
        return a.value, b.value, n.value

    def set_fences(self, on: bool):
        """vcclCommSetFences: system-scope fences around every slot hand-off (VCCL_FENCES)."""
        check(lib().vcclCommSetFences(self.handle, int(bool(on))), "vcclCommSetFences")

    def set_ring_wave(self, on: bool | None) -> int:
        """vcclCommSetRingWave: the SIMPLE ring's per-wave slot hand-off for
        later launches (VCCL_RING_WAVE; None leaves it); returns the ring
        launches that ran the per-wave kernel so far."""
        n = ctypes.c_ulonglong(0)
        check(lib().vcclCommSetRingWave(self.handle, -1 if on is None else int(bool(on)), ctypes.byref(n)),
              "vcclCommSetRingWave")
        return int(n.value)

    def debug_set_epochs(self, ll_epoch: int, direct_epoch: int):
        """vcclCommDebugSetEpochs: overwrite the LL / direct call epochs (wrap tests)."""
        check(lib().vcclCommDebugSetEpochs(self.handle, ll_epoch, direct_epoch),
              "vcclCommDebugSetEpochs")

    def create_premulsum(self, scalar_ptr: int, dtype: int, residence: int) -> int:
        op = ctypes.c_int()
        check(lib().ncclRedOpCreatePreMulSum(ctypes.byref(op), scalar_ptr, dtype, residence,
                                             self.handle), "ncclRedOpCreatePreMulSum")
        return op.value

    def destroy_op(self, op: int):
        check(lib().ncclRedOpDestroy(op, self.handle), "ncclRedOpDestroy")

    def destroy(self):
        if self.handle:
            check(lib().ncclCommDestroy(self.handle), "ncclCommDestroy")
            self.handle = ctypes.c_void_p()

    def abort(self):
        if self.handle:
            check(lib().ncclCommAbort(self.handle), "ncclCommAbort")
            self.handle = ctypes.c_void_p()


def group_start():
    check(lib().ncclGroupStart(), "ncclGroupStart")


def group_end():
    check(lib().ncclGroupEnd(), "ncclGroupEnd")
