/*
 * vccl-mi355x communicator extensions (host only, no GPU work).
 *
 *   vcclCommCollAlgo  which algorithm ncclAllReduce / ncclReduceScatter /
 *                     ncclAllGather would run for (count, datatype) on this
 *                     communicator — the outcome of the tuner step
 *                     topoGetAlgoInfo (src/enqueue.cc:1805-1945) that VCCL
 *                     only reports through NCCL_DEBUG=INFO logs.  For
 *                     benchmarks and tests; enqueues nothing.
 *   vcclCommSetAlgo   per-communicator override of that choice (the
 *                     NCCL_ALGO / NCCL_PROTO environment, graph/tuning.cc:
 *                     354-373, read once at init): -1 = automatic, otherwise
 *                     a vcclAlgo_t; an algorithm that cannot carry a call
 *                     (bucket above its buffer, not an all-reduce) falls
 *                     through to the ring, as with the environment.
 *   vcclCommLaunchStats  collectives enqueued on this communicator so far and
 *                     how many launches carried more than one of them (group
 *                     aggregation of small all-reduces into one LL launch).
 *   vcclCommRingTrace the SIMPLE ring's slot timeline of the last launch
 *                     (VCCL_RING_TRACE=<records per channel> at init, else
 *                     ncclInvalidUsage): per channel `cap` records of 56 bytes
 *                     {t0 entry, t1 credits seen, t2 released, t3 payload
 *                     drained, t4 flags stored (s_memrealtime, 100 MHz);
 *                     uint32 shape = RECV | SEND<<1 | SRC<<2 | DST<<3; uint32
 *                     payload bytes; uint64 step}, unused records zero.  A
 *                     measurement hook (no reference counterpart).
 *   vcclCommNetStats  payload bytes this rank's net proxy has sent / received
 *                     and its connection count (0 when every peer is reached
 *                     over xGMI).  The net transport carries ring connections
 *                     to peers on other nodes (or every connection with
 *                     VCCL_NET_FORCE=1) through host-pinned staging buffers
 *                     and TCP, as the reference's proxy + net transport
 *                     (src/proxy.cc:914-971, src/transport/net.cc:1293-1482).
 *   vcclCommSetFences  switch the system-scope acquire/release fences around
 *                     every FIFO slot / inbox hand-off on (1) or off (0, the
 *                     default: write-through sc0 sc1 payload accesses need no
 *                     fence) — the VCCL_FENCES=1 safety valve at run time, so
 *                     one process can check a transport both ways.  Blocks
 *                     until the device is idle; call with no collective of
 *                     this communicator in flight.
 *   vcclCommSetRingWave  the SIMPLE ring's slot hand-off for this
 *                     communicator's later launches: 0 (the default, or
 *                     VCCL_RING_WAVE=0 at init) the workgroup hand-off — every
 *                     wave drains its stores, a barrier, one thread posts, as
 *                     the reference's postPeer after its barrier
 *                     (src/device/prims_simple.h:183-319); 1 the per-wave
 *                     hand-off, each wave draining its slot behind its next
 *                     slot's loads and the last one posting,
 *                     for the kernels built with it (sums over f32 / f16 /
 *                     bf16, the byte-copy all-gather and broadcast; other
 *                     calls keep the workgroup hand-off).  Same FIFOs,
 *                     partition and fold either way, so results are
 *                     identical and calls may switch between the two.
 *                     perWave -1 leaves the setting as it is; *waveLaunches
 *                     (may be NULL): ring launches that ran the per-wave
 *                     kernel so far.  Host only.
 *   vcclCommDebugSetEpochs  overwrite the device-resident call epochs of the
 *                     one-shot LL and two-shot direct paths (tests of the
 *                     32-bit wrap; the reference's TEST_LL_CLEANUP knob,
 *                     src/include/device.h:70-77, serves the same purpose).
 *                     Every rank must set the same values between calls.
 *   vcclRingPartition  the channel partition the ring algorithm uses for a
 *                     call (host only): VCCL's cbd split and chunking
 *                     (scheduleCollTasksToPlan, src/enqueue.cc:518-644, for a
 *                     plan of one collective) for `nChannels` channels,
 *                     protocol `proto` (2 SIMPLE, 1 LL128, 0 LL) with a FIFO step
 *                     of `stepBytes` (that protocol's buffer size / 8) and
 *                     `nThreads` ring threads (NCCL_NTHREADS: the channel
 *                     tuning's maxThreads[RING][SIMPLE], tuning.cc:198-200).
 *                     out[0..7]
 *                     = channelLo, channelHi, countLo, countMid, countHi,
 *                     chunkLo, chunkMid, chunkHi (elements; bytes for
 *                     all-gather, which the reference runs as int8).
 *   vcclRingOrders     the arc-balanced ring set for n ranks (SURVEY.md
 *                     Appendix D; Walecki's decomposition for odd n).
 *   vcclRingChunkOf    for element i of an all-reduce on that partition:
 *                     out[0] = its channel, out[1] = the ring chunk c of its
 *                     loop (the chunk that finishes at ring position c,
 *                     src/device/all_reduce.h:32-64), out[2] = the end of that
 *                     chunk — the lookup the direct all-reduce folds by.
 *   vcclGroupPlan      the partition a GROUP of calls of one
 *                     communicator gets (host only): VCCL's multi-task plan —
 *                     the size sorter and (func, op, type) bins with 4x
 *                     aggregation of ncclPrepareTasks (src/enqueue.cc:352-437)
 *                     and scheduleCollTasksToPlan's shared trafficPerChannel,
 *                     running channelId and currentTraffic, split into kernel
 *                     plans at the argument budget (:518-769).  Inputs per
 *                     call: colls[i], counts[i] (AR count, RS recvcount, AG
 *                     sendcount), datatypes[i], ops[i] (ncclRedOp_t built-in;
 *                     ignored for all-gather).  Outputs: order[0..n) the calls
 *                     in plan (execution) order, planOf[i] the kernel plan of
 *                     call i, cbd[8 i .. 8 i + 8) its partition as in
 *                     vcclRingPartition.  Every call is taken as RING /
 *                     SIMPLE (LL128 geometry: VCCL's defaults).
 *   vcclGroupPlanEx    the same plan with a path per aggregate, as a comm
 *                     lays out a group: each aggregate takes the path the
 *                     library's selection gives its summed count (VCCL gives
 *                     getAlgoInfo's choice to every member, enqueue.cc:
 *                     387-427) and is placed under that path's protocol (LL
 *                     traffic x4).  geometry[4] = SIMPLE step bytes,
 *                     NCCL_NTHREADS, LL128 step bytes, NCCL_LL128_NTHREADS;
 *                     policy[10] (NULL: every call RING / SIMPLE) =
 *                     algoForce (0 automatic, 1 ring, 2 LL, 3 direct,
 *                     4 LL128), LL slot bytes (0: no LL buffers), LL
 *                     all-reduce max bytes, LL RS / AG max bucket bytes,
 *                     LL128 FIFOs (0/1), LL128 window min, max (0: off),
 *                     direct inboxes (0/1), direct all-reduce max bytes,
 *                     direct RS / AG max bucket bytes; algos[i] (may be
 *                     NULL) = the vcclAlgo_t of call i.
 *   vcclAlgoSelection  how NCCL_ALGO / NCCL_PROTO strings select paths (the
 *                     reference's parseList, graph/tuning.cc:53-116: comma
 *                     lists, a leading '^' excludes): *force = 0 automatic,
 *                     1 SIMPLE ring, 2 LL, 3 direct, 4 LL128 ring; *allowed =
 *                     bit 0 LL, bit 1 LL128, bit 2 SIMPLE, bit 3 direct.
 *                     ncclInvalidUsage for an unknown name, as at init.
 */
#ifndef VCCL_EXT_H_
#define VCCL_EXT_H_
#include <stddef.h>
#include <stdint.h>

#include "nccl.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  vcclCollAllReduce = 0,
  vcclCollReduceScatter = 1,
  vcclCollAllGather = 2,
  vcclCollBroadcast = 3,
  vcclCollReduce = 4
} vcclColl_t;
typedef enum {
  vcclAlgoRing = 0,     /* SIMPLE ring over arc-balanced ring sets */
  vcclAlgoLL = 1,       /* one-shot LL all-reduce, chain-tree fold */
  vcclAlgoDirect = 2,   /* two-shot direct all-reduce over the full mesh */
  vcclAlgoOneRank = 3,  /* nRanks == 1: copy / PreMulSum kernel */
  vcclAlgoLL128 = 4     /* ring over LL128 FIFOs (64-byte lines by default, in-line flags) */
} vcclAlgo_t;

ncclResult_t vcclCommCollAlgo(ncclComm_t comm, int coll, size_t count, ncclDataType_t datatype,
                              int* algo);
ncclResult_t vcclCommSetAlgo(ncclComm_t comm, int algo);
/* The vcclAlgo_t every call of a group would take on this comm: the path of
 * its 4x aggregate in VCCL's plan (see vcclGroupPlanEx); nothing launched.
 * colls / counts / datatypes / ops as in vcclGroupPlan. */
ncclResult_t vcclCommGroupAlgos(ncclComm_t comm, int nCalls, const int* colls, const size_t* counts,
                                const int* datatypes, const int* ops, int* algos);
ncclResult_t vcclCommLaunchStats(ncclComm_t comm, unsigned long long* collectives,
                                 unsigned long long* fusedLaunches);
ncclResult_t vcclCommRingTrace(ncclComm_t comm, void* hostBuf, size_t bytes, int* nChannels, int* cap);
ncclResult_t vcclCommNetStats(ncclComm_t comm, uint64_t* bytesSent, uint64_t* bytesReceived,
                              int* connections);
ncclResult_t vcclCommSetFences(ncclComm_t comm, int useFences);
ncclResult_t vcclCommSetRingWave(ncclComm_t comm, int perWave, unsigned long long* waveLaunches);
ncclResult_t vcclCommDebugSetEpochs(ncclComm_t comm, uint32_t llEpoch, uint32_t directEpoch);
ncclResult_t vcclRingPartition(int coll, size_t count, ncclDataType_t datatype, int nRanks,
                               int nChannels, int proto, size_t stepBytes, int nThreads,
                               int64_t* out);
ncclResult_t vcclRingChunkOf(size_t count, ncclDataType_t datatype, int nRanks, int nChannels,
                             size_t slotBytes, int nThreads, size_t i, int64_t* out);
/* The ring set of an nRanks communicator: orders[k * nRanks + i] = the rank
 * at position i of ring k (channel c runs on ring c mod nRings). */
ncclResult_t vcclRingOrders(int nRanks, int maxRings, int* orders, int* nRings);
ncclResult_t vcclGroupPlan(int nCalls, const int* colls, const size_t* counts, const int* datatypes,
                           const int* ops, int nRanks, int nChannels, size_t stepBytes, int nThreads,
                           int* order, int* planOf, int64_t* cbd);
ncclResult_t vcclGroupPlanEx(int nCalls, const int* colls, const size_t* counts, const int* datatypes,
                             const int* ops, int nRanks, int nChannels, const int64_t* geometry,
                             const int64_t* policy, int* algos, int* order, int* planOf, int64_t* cbd);
ncclResult_t vcclAlgoSelection(const char* algo, const char* proto, int* force, int* allowed);

#ifdef __cplusplus
}
#endif
#endif /* VCCL_EXT_H_ */
