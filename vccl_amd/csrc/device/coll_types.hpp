// Work descriptors and buffer layouts of the one-hop LL (ll.hpp) and direct
// (direct.hpp) collectives, shared by the host planner and the kernels.  Kept
// apart from the kernel code so host objects and the other kernel families do
// not recompile when a kernel body changes.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "ring_types.hpp"

namespace vccl {

// ------------------------------------------------------------------- LL
constexpr int kLLMaxParts = 16;

// One call of an LL launch.  All-reduce: nbytes = count * sizeof(T).
// Reduce-scatter / all-gather: nbytes = the bytes of ONE rank's block (send
// holds n blocks for a reduce-scatter, recv n blocks for an all-gather); the
// reduce-scatter folds each line on the ring of its channel (VCCL's cbd
// partition of the block, `cbd`, DevComm::rsOrder).
struct LLPart {
  const char* send;
  char* recv;
  int64_t nbytes;
  int64_t line0;           // first line of this part in the slot
  CbdLite cbd;             // reduce-scatter only
};

struct LLWork {
  DevComm* comm;
  uint64_t redArg;
  const void* redArgPtr;
  int redArgBytes;
  int preOp;
  int nRanks, rank;
  int linesPerSlot;        // capacity of one (parity, source) slot
  int nParts;              // 1 .. kLLMaxParts calls of one collective in this launch
  int64_t nLines;          // lines of all parts (<= linesPerSlot)
  char* localBuf;          // my LL buffer: [2 parities][nRanks sources][linesPerSlot] lines
  char* peerBuf[kMaxRanks];  // every rank's LL buffer mapped here (peerBuf[rank] = local)
  LLPart parts[kLLMaxParts];
};

// Byte offset of the (parity, source rank) slot inside an LL buffer.
__host__ __device__ __forceinline__ size_t ll_slot_off(int parity, int src, int nRanks,
                                                       int linesPerSlot) {
  return ((size_t)parity * nRanks + src) * (size_t)linesPerSlot * 16;
}

// --------------------------------------------------------------- direct
constexpr int kDirectMaxRanks = 8;     // phase 2 folds all n inputs in registers
constexpr int kDirectMaxBlocks = 128;
constexpr int kDirectFlagStride = 64;  // bytes between flags
constexpr int kDirectThreads = 512;
constexpr int kDirectUnroll = 2;

// Every rank's inbox and flag array, mapped into this process (device memory,
// so runtime peer indices never index a by-value kernel argument).
struct DirectPeers {
  char* buf[kDirectMaxRanks];
  char* flags[kDirectMaxRanks];
};

struct DirectWork {
  DevComm* comm;
  const DirectPeers* peers;
  const void* sendbuff;
  void* recvbuff;
  uint64_t count;        // elements
  uint64_t redArg;
  const void* redArgPtr;
  int redArgBytes;
  int preOp;
  int nRanks, rank;
  int nBlocks;           // workgroups (block b of every shard -> workgroup b)
  int nChunks;           // the bucket moves through the inbox in chunks
  int64_t chunkElts;     // elements per chunk (last one shorter)
  int64_t blkElts;       // elements per block, the same for every chunk
  int64_t regionBytes;   // bytes per (phase, rank) inbox region
  // VCCL's cbd channel partition (host/enqueue.cc cbd_schedule, the ring's
  // own) of the recvcount block (reduce-scatter) or of the whole bucket
  // (all-reduce, with the ring chunk arChunk): channel c of [channelLo,
  // channelHi] folds on ring c mod nRings (DevComm::rsOrder / ringAt), so
  // the direct path reproduces the ring's (= VCCL's) fold order exactly.
  CbdLite cbd;
  int64_t arChunk;
};

// Shard length of a chunk of `cc` elements: ceil(cc / n) in 16-byte units.
// The block length stays that of the first (largest) chunk, so block b sits
// at the same inbox offset in every chunk (a shorter last chunk only leaves
// high blocks empty) — the buffer-reuse argument (direct.hpp header) needs
// fixed offsets.
__host__ __device__ __forceinline__ int64_t direct_shard_elts(int64_t cc, int n, int64_t eltAlign) {
  return ((cc + n - 1) / n + eltAlign - 1) / eltAlign * eltAlign;
}

// Inbox: [2 phases][2 parities][nRanks sources][region]; flags likewise.
// The all-reduce double-buffers its chunks by parity (direct.hpp); the
// one-hop reduce-scatter / all-gather use parity 0.
constexpr int kDirectInboxRegions = 4;  // regions per source: phases x parities
__host__ __device__ __forceinline__ size_t direct_region_off(int phase, int parity, int src, int nRanks,
                                                             int64_t regionBytes) {
  return (((size_t)phase * 2 + parity) * nRanks + src) * (size_t)regionBytes;
}
__host__ __device__ __forceinline__ size_t direct_flag_off(int phase, int parity, int src, int b) {
  return ((((size_t)phase * 2 + parity) * kDirectMaxRanks + src) * kDirectMaxBlocks + b) *
         kDirectFlagStride;
}
constexpr size_t kDirectFlagBytes =
    (size_t)kDirectInboxRegions * kDirectMaxRanks * kDirectMaxBlocks * kDirectFlagStride;

// Group aggregation of direct calls (DirectBatch: part 0 in `w`, the others
// as DirectPart — what differs per call), run in order by one launch.
constexpr int kDirectMaxWorks = 16;
struct DirectPart {
  const void* sendbuff;
  void* recvbuff;
  uint64_t count;
  int nChunks;
  int pad;
  int64_t chunkElts, blkElts;
  CbdLite cbd;
  int64_t arChunk;
};
struct DirectBatch {
  DirectWork w;
  int nParts;
  DirectPart more[kDirectMaxWorks - 1];
};
__host__ __device__ inline DirectPart direct_part_of(const DirectWork& w) {
  return DirectPart{w.sendbuff, w.recvbuff, w.count, w.nChunks, 0, w.chunkElts, w.blkElts, w.cbd,
                    w.arChunk};
}
__host__ __device__ inline DirectWork direct_work_with(DirectWork w, const DirectPart& p) {
  w.sendbuff = p.sendbuff;
  w.recvbuff = p.recvbuff;
  w.count = p.count;
  w.nChunks = p.nChunks;
  w.chunkElts = p.chunkElts;
  w.blkElts = p.blkElts;
  w.cbd = p.cbd;
  w.arChunk = p.arChunk;
  return w;
}

}  // namespace vccl
