// Host/device-shared layout of the ring transport (POD, no HIP types).
//
// Replaces ncclDevChannel / ncclConnInfo (src/include/device.h) with the
// minimum the MI355X ring needs.  One channel = one workgroup = one ring
// position with its own FIFO pair (reference: one block per channel,
// enqueue.cc:1576-1666).  FIFOs follow the SIMPLE protocol of
// prims_simple.h:108-181: kSteps slots, the sender waits for a free slot
// (head + kSteps > step), the receiver waits for a posted slot (tail > step).
//
// Memory placement: every FIFO and flag lives in the
// RECEIVER's HBM, allocated uncached (hipDeviceMallocUncached) so peer writes
// over xGMI are never hidden behind a stale L2/L1 line; the sender writes the
// slot payload remotely ("P2P write", as NCCL on NVLink, transport/p2p.cc:484-503).
#pragma once
#include <stdint.h>

namespace vccl {

constexpr int kSteps = 8;            // NCCL_STEPS (device.h:24)
constexpr int kMaxRanks = 64;
// MAXCHANNELS (device.h:62) is 64 in the reference: the default channel
// counts stay within it (kVcclMaxChannels, host/init.cc), so VCCL can run the
// same geometry.  NCCL_NCHANNELS / VCCL_CHANNELS_PER_RING may go up to 128
// here: a channel is one workgroup on one CU, and on one GPU shared by
// several ranks (the rehearsals) the ring is bound by its channels' copy rate
// (2 ranks on one GPU: 64 -> 96 -> 128 channels, 512 MiB AR 1039 -> 868 ->
// 845 us, profiles/r03q).
constexpr int kVcclMaxChannels = 64;
#ifndef VCCL_MAX_CHANNELS
#define VCCL_MAX_CHANNELS 128
#endif
constexpr int kMaxChannels = VCCL_MAX_CHANNELS;
constexpr int kFlagStride = 128;     // bytes between flags (one line each)
constexpr int kOrderMaxRings = 8;    // ring sets of SURVEY.md Appendix D: 7 (n=8), 6 (n=4), 1
constexpr int kOrderMaxRanks = 8;
// Slot stride = slotBytes + kSlotPad: RS / AG place a chunk at byte offset
// (logical offset mod 16) inside its slot, so the slot shares the user
// block's misalignment and the copy stays on 16-byte packs (ring.hpp).
constexpr int kSlotPad = 64;
__host__ __device__ constexpr int64_t slot_stride(int slotBytes) { return (int64_t)slotBytes + kSlotPad; }

// Values of the comm's error word (DevComm::errorFlag): a spin without
// progress (a lost peer, ncclRemoteError), or a net slot whose landed byte
// count is not the step's slice length (ncclInternalError).
constexpr int kErrSpinTimeout = 1;
constexpr int kErrSlotSize = 2;
// Net slot size word before the GPU writes it / after the proxy shipped the
// slot (the reference's -1, src/transport/net.cc:1250-1255, 1365-1367).
constexpr uint32_t kNetSizeUnset = 0xffffffffu;

struct DevChannel {
  // ring order: ringRanks[k] = rank at ring position (myPos + k) mod n
  // (userRanks rotated to self, init.cc:599-615)
  int ringRanks[kMaxRanks];
  int ringPos;                       // my index in the ring (ring->index)
  int pad0;
  // receive side: data arrives in MY memory
  char* recvFifo;                    // kSteps * slotBytes, local
  uint64_t* recvTail;                // local flag, written by prev: slots posted
  uint64_t* prevSendHead;            // prev's flag (remote): slots I consumed
  // send side: data goes to NEXT's memory
  char* sendFifo;                    // next's recvFifo (remote)
  uint64_t* nextRecvTail;            // next's recvTail (remote)
  uint64_t* sendHead;                // local flag, written by next
  // Net connection only (null over xGMI): bytes of each posted slot, stored
  // before the tail so the proxy sends only what the step filled.
  uint32_t* sendSizes;
  // Net connection only: bytes the proxy landed in each slot (written before
  // recvTail); the ring kernel checks them against the slice length it
  // computes itself (ring.hpp recv_size_ok) and raises kErrSlotSize on a
  // mismatch instead of reducing a short or stale slot.
  const uint32_t* recvSizes;
  // LL128 FIFOs (ring.hpp prim_ll128): kSteps slots of 64-byte lines, local
  // (receive) and next's (send); null when the comm has no LL128 buffers.
  // Steps, credits (sendHead / prevSendHead) and the slot index are shared
  // with the SIMPLE FIFO: a step is one slot of either protocol.
  char* ll128Recv;
  char* ll128Send;
  // persistent step counters (kernel reads at start, writes at end)
  uint64_t recvStep;
  uint64_t sendStep;
};

struct DevComm {
  int rank, nRanks;
  int nChannels;
  int slotBytes;                     // bytes per FIFO slot
  volatile int* abortFlag;           // host-pinned, mapped (ncclCommAbort)
  int* errorFlag;                    // host-pinned, mapped: kErrSpinTimeout / kErrSlotSize
  uint64_t spinTimeoutTicks;         // s_memrealtime ticks (100 MHz)
  int useFences;                     // 1: system acquire/release around each slot
  int pollMode;                      // 0: system-scope load, 1: atomic RMW poll
  // LL call epoch, device-resident so captured graphs replay correctly:
  // every workgroup reads llEpoch at start; the last one to finish (llDone
  // ticket) advances it for the next call.
  uint32_t llEpoch;
  uint32_t llDone;
  // Same scheme for the two-shot direct all-reduce (direct.hpp).
  uint32_t dEpoch;
  uint32_t dDone;
  // This rank's reduce-scatter fold order on each ring of the comm's ring
  // set: rsOrder[k][j] = the rank at ring-k position (pos(me) + 1 + j) mod n,
  // the order VCCL's ring reduce-scatter folds my block in on a channel of
  // ring k (reduce_scatter.h:39-53: from my ring successor around to me).
  // Channel c runs on ring c mod nRings.  The one-hop LL / direct
  // reduce-scatters (n <= kOrderMaxRanks) fold in the same order.
  int nRings;
  int8_t rsOrder[kOrderMaxRings][kOrderMaxRanks];
  // ringAt[k][p] = the rank at position p of ring k (the ring's own order,
  // ring->index space): VCCL's ring all-reduce folds chunk c of a loop from
  // position c+1 around to c (all_reduce.h:42-64), whichever rank computes
  // it — the direct all-reduce folds in that order too.
  int8_t ringAt[kOrderMaxRings][kOrderMaxRanks];
  // The chain the one-hop LL all-reduce folds along, root first: VCCL's
  // intra-node tree is a chain in its topology's order (graph/connect.cc:
  // 64-65; the root at index 0 applies postOp), reduced from the leaf up,
  // each hop computing child (+) own (prims_ll.h:258-266).  The identity by
  // default; VCCL_LL_CHAIN pins another order (e.g. the one VCCL's topology
  // search picked) so the LL result matches VCCL's bit for bit.
  int8_t llChain[kOrderMaxRanks];
  // Opt-in slot timeline of the SIMPLE ring (VCCL_RING_TRACE=<records per
  // channel>, vcclCommRingTrace): per channel, the first traceCap slot
  // hand-offs of each launch as RingTraceRec; nullptr = off.
  uint64_t* trace;
  int traceCap;
  // SIMPLE ring slots of at least this many bytes hand over per wave
  // (ring.hpp prim_ws), smaller ones as a workgroup (VCCL_RING_WAVE_MIN)
  int64_t ringWaveMin;
};

// One SIMPLE-ring slot hand-off, s_memrealtime ticks (100 MHz), taken by
// thread 0: entry, credits seen, workgroup released, payload drained
// (every wave's stores complete, second barrier), flags stored; shape =
// RECV | SEND << 1 | SRC << 2 | DST << 3; bytes of payload; tc = thread 0's
// own loads and stores issued (before its drain), so t3 - tc is the drain of
// the memory pipeline plus the wait for the slowest wave.
struct RingTraceRec {
  uint64_t t0, t1, t2, t3, t4;
  uint32_t shape, bytes;
  uint64_t step;
  uint64_t tc;
};
static_assert(sizeof(RingTraceRec) == 64, "trace record layout");

// The part of VCCL's cbd partition a reduce-scatter needs to know which
// channel (hence ring, hence fold order) an element of the block is on.
struct CbdLite {
  int channelLo, channelHi;
  int64_t countLo, countMid, count;  // count = the whole block (recvcount)
};

// ncclCollCbdPart (device.h:297-323) inverted: the channel of element i and
// the end of that channel's part.
__host__ __device__ inline int cbd_channel_of(const CbdLite& p, int64_t i, int64_t* end) {
  if (p.channelHi == p.channelLo) {
    *end = p.count;
    return p.channelLo;
  }
  if (i < p.countLo) {
    *end = p.countLo;
    return p.channelLo;
  }
  const int64_t nMid = p.channelHi - p.channelLo - 1;
  const int64_t j = i - p.countLo;
  if (p.countMid > 0 && j < nMid * p.countMid) {
    const int64_t m = j / p.countMid;
    *end = p.countLo + (m + 1) * p.countMid;
    return p.channelLo + 1 + (int)m;
  }
  *end = p.count;
  return p.channelHi;
}

// The ring all-reduce's chunk of element i (all_reduce.h:32-47 inside the
// ncclCollCbdPart of its channel): channel, chunk index c within its loop
// (the chunk that finishes at ring position c) and the end of that chunk.
// `chunk` is the SIMPLE chunk of every part (cbd_schedule: one value),
// eltAlign = 16 / sizeof(T); the last loop's chunk is
// alignUp(divUp(rem, n), eltAlign), exactly as ring_allreduce steps it.
__host__ __device__ inline int ar_chunk_of(const CbdLite& p, int64_t chunk, int n, int64_t eltAlign,
                                           int64_t i, int* c, int64_t* end) {
  int64_t partEnd;
  const int ch = cbd_channel_of(p, i, &partEnd);
  const int64_t nMid = p.channelHi - p.channelLo - 1;
  const int64_t partStart = ch == p.channelLo ? 0
                            : ch == p.channelHi ? p.countLo + nMid * p.countMid
                                                : p.countLo + (int64_t)(ch - p.channelLo - 1) * p.countMid;
  const int64_t rel = i - partStart, loopCount = (int64_t)n * chunk;
  const int64_t eo = rel / loopCount * loopCount, rem = partEnd - partStart - eo;
  const int64_t ck = rem < loopCount ? ((rem + n - 1) / n + eltAlign - 1) / eltAlign * eltAlign : chunk;
  *c = (int)((rel - eo) / ck);
  const int64_t e = partStart + eo + (int64_t)(*c + 1) * ck;
  *end = e < partEnd ? e : partEnd;
  return ch;
}

// Per-launch work descriptor (kernel argument, by value).
struct RingWork {
  DevComm* comm;                     // device-resident
  DevChannel* channels;              // device-resident, nChannels entries
  const void* sendbuff;
  void* recvbuff;
  uint64_t count;                    // AR: count; RS: recvcount; AG: bytes per rank; BC: bytes
  uint64_t redArg;                   // device op argument (also the preOp scalar)
  const void* redArgPtr;             // ncclScalarDevice scalar (read on device)
  int redArgBytes;
  int preOp;                         // PreMulSum: scale own input
  int nChannels;                     // workgroups launched (= cbd.channelHi + 1)
  int slotBytes;
  int nRanks;
  // VCCL's channel partition of this call (ncclDevWorkColl.cbd, device.h:
  // 258-287, filled by the host's restatement of scheduleCollTasksToPlan,
  // enqueue.cc:597-644): channels [channelLo, channelHi] carry parts of
  // countLo / countMid... / countHi elements, moved in chunks of chunkLo /
  // chunkMid / chunkHi elements per ring step (calcCollChunking: 4 FIFO slots
  // for SIMPLE) — each chunk step crosses the FIFO as ceil(chunk / slot)
  // slices.  Same partition => the same fold order per element as VCCL.
  int channelLo, channelHi;
  int64_t countLo, countMid, countHi;
  int64_t chunkLo, chunkMid, chunkHi;
  // LL128 ring (proto = kProtoLL128): bytes per LL128 FIFO slot
  int64_t ll128SlotBytes;
  int root;                          // broadcast / reduce: the root's rank
};

// Protocols of the ring kernels (nccl_common.h ids).  kProtoSimpleWave is a
// device-side tag only: the SIMPLE protocol (same FIFOs, partition and fold)
// with the per-wave slot hand-off (ring.hpp prim_ws), built as its own
// kernels (ring_kernels.hip PART 4) and chosen per comm at run time.
enum : int { kProtoLL = 0, kProtoLL128 = 1, kProtoSimple = 2, kProtoSimpleWave = 3 };
// LL128 wire format on gfx950 (ring.hpp ll128_prim): lines of L bytes, one
// per L/16 lanes — every lane but the line's last carries a 16-byte data
// piece, the last an 8-byte data piece and the 8-byte flag — so one wave
// instruction moves 1 KiB ("a round") of 1024/L lines.
//   L = 64 (default): 16 lines, 896 data bytes per round (7/8), one flag per
//       64-byte write request — the unit a wave store reaches memory in
//       (every TCC_EA0 write request is 64 B, profiles/r04f), so a line lands
//       whole;
//   L = 128 (-DVCCL_LL128_LINE=128 -DVCCL_LL128_PROBE_BUILD, VCCL's 15/16 NVLink line, device.h:
//       82-83): 8 lines, 960 data bytes per round, 2-4 % faster at 1-8 MiB
//       (profiles/r04e) — but a line is TWO write requests with no order
//       between them, and r04l caught the tear: 16 fp32 (the first 64 bytes
//       of a line, data lanes 0-3) stale under a fresh flag in a 4-rank
//       LL128 all-reduce (profiles/r04l).  Not safe; kept only for probes.
#ifndef VCCL_LL128_LINE
#define VCCL_LL128_LINE 64
#endif
static_assert(VCCL_LL128_LINE == 64 || VCCL_LL128_LINE == 128, "LL128 line: 64 or 128 bytes");
// the 128-byte line tears (above), so a build with it is for the
// tearing probe only and must say so
#if VCCL_LL128_LINE == 128 && !defined(VCCL_LL128_PROBE_BUILD)
#error "VCCL_LL128_LINE=128 tears (profiles/r04l): probe builds only, add -DVCCL_LL128_PROBE_BUILD"
#endif
constexpr int kLL128LineBytes = VCCL_LL128_LINE;
constexpr int kLL128LaneSpan = kLL128LineBytes / 16;    // lanes per line
constexpr int kLL128LinesPerRound = 64 / kLL128LaneSpan;
constexpr int kLL128RoundWire = 1024;
constexpr int kLL128RoundData = kLL128RoundWire - 8 * kLL128LinesPerRound;

// Group aggregation (the reference's planner packing a group's collectives
// into one plan, enqueue.cc:352-508 / :518-769, run by one kernel over its
// work batch, common.h:260-293): one ring launch carries up to kRingMaxWorks
// calls of one comm with the same collective, type and op — part 0 in `w`,
// the others as RingPart (what differs per call).  Every channel workgroup
// runs the parts in order on its ring, so the FIFO step sequence is the same
// on every rank; a channel outside a part's [channelLo, channelHi] skips it.
constexpr int kRingMaxWorks = 16;
struct RingPart {
  const void* sendbuff;
  void* recvbuff;
  uint64_t count;
  int root;
  int channelLo, channelHi;
  int64_t countLo, countMid, countHi;
  int64_t chunkLo, chunkMid, chunkHi;
};
struct RingBatch {
  RingWork w;                        // part 0 and everything the parts share
  int nParts;                        // 1 .. kRingMaxWorks
  RingPart more[kRingMaxWorks - 1];  // parts 1 .. nParts-1
};
__host__ __device__ inline RingPart ring_part_of(const RingWork& w) {
  return RingPart{w.sendbuff, w.recvbuff, w.count, w.root, w.channelLo, w.channelHi, w.countLo,
                  w.countMid, w.countHi, w.chunkLo, w.chunkMid, w.chunkHi};
}
__host__ __device__ inline RingWork ring_work_with(RingWork w, const RingPart& p) {
  w.sendbuff = p.sendbuff;
  w.recvbuff = p.recvbuff;
  w.count = p.count;
  w.root = p.root;
  w.channelLo = p.channelLo;
  w.channelHi = p.channelHi;
  w.countLo = p.countLo;
  w.countMid = p.countMid;
  w.countHi = p.countHi;
  w.chunkLo = p.chunkLo;
  w.chunkMid = p.chunkMid;
  w.chunkHi = p.chunkHi;
  return w;
}

}  // namespace vccl
