// Ring primitives and schedules (SIMPLE protocol) for gfx950.
//
// Protocol semantics follow prims_simple.h:108-319 (waitPeer / genericOp /
// postPeer) and the schedules all_reduce.h:12-83, reduce_scatter.h:12-55,
// all_gather.h:12-83.  The MI355X design differs where the hardware does:
//  * one workgroup per channel, no role warps or named barriers: lane 0 of
//    wave 0 polls both credits, one s_barrier releases the workgroup, every
//    thread copies/reduces, every wave drains its stores (s_waitcnt vmcnt(0)),
//    s_barrier, lane 0 publishes (system-scope release fence + relaxed
//    system-scope store of the step counter into the peer's flag);
//  * FIFOs are uncached receiver-side HBM reached over xGMI by the sender;
//  * every spin is bounded (abort flag + wall-clock timeout via s_memrealtime)
//    so a lost peer ends the kernel instead of hanging the GPU.
#pragma once
#include "reduce_copy.hpp"
#include "ring_types.hpp"

#ifndef VCCL_RING_SRC_POL
#define VCCL_RING_SRC_POL kNT  // load policy of the rank's own input in ring steps
#endif

namespace vccl {

__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void drain_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

struct RingCtx {
  DevChannel* ch;
  const DevComm* comm;
  uint64_t recvStep, sendStep;
  int tid, nthreads;
  int slotBytes;
  int* shAbort;  // LDS

  // Bounded spin on `flag` until pred(value); returns false on abort/timeout.
  // The timeout is per wait (no progress for spinTimeoutTicks), not per call.
  __device__ uint64_t poll(const uint64_t* flag) const {
    // pollMode 1: atomic RMW (resolved at the point of coherence, never a
    // cached copy); 0: relaxed system-scope load.
    if (comm->pollMode == 1)
      return __hip_atomic_fetch_add((uint64_t*)flag, (uint64_t)0, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_SYSTEM);
    return ld_sys(flag);
  }

  __device__ bool spin_ge(const uint64_t* flag, uint64_t target) {
    uint64_t spins = 0, start = 0;
    while (poll(flag) < target) {
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 255) == 0) {
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (start == 0) start = now;
        if (*comm->abortFlag) return false;
        if (now - start > comm->spinTimeoutTicks) {
          __hip_atomic_store(comm->errorFlag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          return false;
        }
        if (__hip_atomic_load(comm->errorFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
          return false;
      }
    }
    return true;
  }

  __device__ bool aborted() const { return *shAbort != 0; }

  // One primitive call: at most one slot of payload.
  //   srcs = [SRC ? own input] ++ [RECV ? recv slot]
  //   dsts = [SEND ? peer slot] ++ [DST ? own output]
  //   recvOff / sendOff: byte offset of the chunk inside its slot (< 16)
  template <class Fn, bool RECV, bool SEND, bool SRC, bool DST, int UNROLL>
  __device__ void prim(const Fn& fn, const void* src, void* dst, int64_t nelem, bool postOp,
                       int recvOff = 0, int sendOff = 0) {
    if (aborted()) return;
    if (tid == 0) {
      bool ok = true;
      if (RECV) ok = spin_ge(ch->recvTail, recvStep + 1);
      if (SEND && ok && sendStep + 1 > (uint64_t)kSteps) ok = spin_ge(ch->sendHead, sendStep + 1 - kSteps);
      if (!ok) *shAbort = 1;
      if (comm->useFences) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system-scope acquire
        drain_vmem();
      }
    }
    __syncthreads();
    if (aborted()) return;
    if (nelem > 0) {
      // Operand order and memory policy: own input streamed once (nt), FIFO
      // slots system-coherent write-through (sc0 sc1).  Own output: sc0 sc1
      // when it is the only destination, nt beside a FIFO slot — the
      // two-destination shape runs at 7.13 TB/s with one write-through and
      // one nt destination, 6.0 with both write-through, 5.5 with both plain
      // (tools/sweep_rc.py twodst, profiles/r03a; PMC traffic = algorithmic
      // in every case, so the policy mix, not the bytes, sets the rate).
      constexpr int NS = (SRC ? 1 : 0) + (RECV ? 1 : 0);
      constexpr int ND = (SEND ? 1 : 0) + (DST ? 1 : 0);
      constexpr int S0 = SRC ? VCCL_RING_SRC_POL : kSys, S1 = kSys;
      constexpr int D0 = kSys, D1 = kNT;
      constexpr int POLS = mkpol(S0, S1, S1, S1, D0, D1, D1, D1);
      RCArgs a;
      int s = 0, d = 0;
      if (SRC) a.srcs[s++] = (const char*)src;
      if (RECV) a.srcs[s++] = ch->recvFifo + (int64_t)(recvStep % kSteps) * slot_stride(slotBytes) + recvOff;
      if (SEND) a.dsts[d++] = ch->sendFifo + (int64_t)(sendStep % kSteps) * slot_stride(slotBytes) + sendOff;
      if (DST) a.dsts[d++] = (char*)dst;
      a.nSrcs = NS;
      a.nDsts = ND;
      a.preOpSrcs = SRC ? 1 : 0;
      a.postOp = postOp ? 1 : 0;
      reduce_copy<Fn, NS, ND, UNROLL, POLS, 0, true>(fn, a, nelem, 0, 1, tid, nthreads);
    }
    drain_vmem();  // every storing wave: its write-through payload stores are complete
    __syncthreads();
    if (tid == 0) {
      if (comm->useFences) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system-scope release (L2 writeback)
        drain_vmem();
      }
      if (SEND && ch->sendSizes)
        __hip_atomic_store(ch->sendSizes + sendStep % kSteps,
                           (uint32_t)(nelem > 0 ? sendOff + nelem * (int64_t)sizeof(typename Fn::EltType) : 0),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (SEND) st_sys(ch->nextRecvTail, sendStep + 1);
      if (RECV) st_sys(ch->prevSendHead, recvStep + 1);
    }
    if (SEND) sendStep++;
    if (RECV) recvStep++;
  }
};

__device__ __forceinline__ int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }
__device__ __forceinline__ int64_t div_up(int64_t x, int64_t a) { return (x + a - 1) / a; }

// ncclCollCbdPart (device.h:297-323): this channel's part of the call
// (element offset, element count) and its chunk size; false = idle channel.
__device__ __forceinline__ bool cbd_part(const RingWork& w, int c, int64_t* off, int64_t* len,
                                         int64_t* chunk) {
  if (c < w.channelLo || c > w.channelHi) return false;
  const int64_t nMid = w.channelHi - w.channelLo - 1;
  if (c == w.channelLo) {
    *off = 0;
    *len = w.countLo;
    *chunk = w.chunkLo;
  } else if (c == w.channelHi) {
    *off = w.countLo + nMid * w.countMid;
    *len = w.countHi;
    *chunk = w.chunkHi;
  } else {
    *off = w.countLo + (int64_t)(c - w.channelLo - 1) * w.countMid;
    *len = w.countMid;
    *chunk = w.chunkMid;
  }
  return true;
}

// One ring step of `nelem` elements (a VCCL chunk, up to 4 slots): the chunk
// crosses the FIFO slot by slot (the reference's slices, prims_simple.h:
// 193-194); an empty step still hands over one (empty) slot, as the
// reference's nelem <= 0 primitive calls do.  Sender and receiver of a chunk
// always agree on its length, so they agree on the slice count.
template <class Fn, bool RECV, bool SEND, bool SRC, bool DST, int UNROLL>
__device__ __forceinline__ void ring_step(RingCtx& r, const Fn& fn, const void* src, void* dst,
                                          int64_t nelem, bool postOp, int recvOff = 0,
                                          int sendOff = 0) {
  using T = typename Fn::EltType;
  const int64_t slotElts = (int64_t)r.slotBytes / (int64_t)sizeof(T);
  const int64_t nSlices = nelem > 0 ? div_up(nelem, slotElts) : 1;
  for (int64_t s = 0; s < nSlices; s++) {
    const int64_t o = s * slotElts;
    const int64_t len = nelem - o < slotElts ? nelem - o : slotElts;
    r.prim<Fn, RECV, SEND, SRC, DST, UNROLL>(fn, SRC ? (const void*)((const T*)src + o) : nullptr,
                                             DST ? (void*)((T*)dst + o) : nullptr,
                                             len > 0 ? len : 0, postOp, recvOff, sendOff);
  }
}

// ----------------------------------------------------------------- AllReduce
// all_reduce.h:12-83 (runRing): RS then AG within one kernel, chunk c of each
// round finishing at ring position c.
template <class Fn, int UNROLL>
__device__ void ring_allreduce(RingCtx& r, const Fn& fn, const RingWork& w, int c) {
  using T = typename Fn::EltType;
  const int n = w.nRanks;
  const int64_t eltAlign = 16 / sizeof(T) ? 16 / sizeof(T) : 1;
  int64_t gridOff, chCount, chunkCount;
  if (!cbd_part(w, c, &gridOff, &chCount, &chunkCount)) return;
  const T* in = (const T*)w.sendbuff;
  T* out = (T*)w.recvbuff;
  const int ringIx = r.ch->ringPos;
  const int64_t loopCount = (int64_t)n * chunkCount;
  auto modRanks = [n](int x) { return x >= n ? x - n : x; };
  for (int64_t eo = 0; eo < chCount; eo += loopCount) {
    const int64_t rem = chCount - eo;
    if (rem < loopCount) chunkCount = align_up(div_up(rem, n), eltAlign);  // all_reduce.h:36
    auto off_of = [&](int chunk) { return gridOff + eo + chunk * chunkCount; };
    auto len_of = [&](int chunk) {
      int64_t l = rem - (int64_t)chunk * chunkCount;
      return l < chunkCount ? (l < 0 ? 0 : l) : chunkCount;
    };
    int chunk = modRanks(ringIx + n - 1);  // step 0: send own chunk
    ring_step<Fn, false, true, true, false, UNROLL>(r, fn, in + off_of(chunk), nullptr, len_of(chunk), false);
    for (int j = 2; j < n; ++j) {          // n-2 recv-reduce-send
      chunk = modRanks(ringIx + n - j);
      ring_step<Fn, true, true, true, false, UNROLL>(r, fn, in + off_of(chunk), nullptr, len_of(chunk),
                                                     false);
    }
    chunk = ringIx;                         // final reduce: output + send
    ring_step<Fn, true, true, true, true, UNROLL>(r, fn, in + off_of(chunk), out + off_of(chunk),
                                                  len_of(chunk), true);
    for (int j = 1; j < n - 1; ++j) {      // n-2 recv-copy-send
      chunk = modRanks(ringIx + n - j);
      ring_step<Fn, true, true, false, true, UNROLL>(r, fn, nullptr, out + off_of(chunk), len_of(chunk),
                                                     false);
    }
    chunk = modRanks(ringIx + 1);          // final recv
    ring_step<Fn, true, false, false, true, UNROLL>(r, fn, nullptr, out + off_of(chunk), len_of(chunk),
                                                    false);
  }
}

// ------------------------------------------------------------- ReduceScatter
// reduce_scatter.h:12-55: the chunk owned by rank ringRanks[k] starts at its
// ring successor; the owner writes output[off] with postOp.
template <class Fn, int UNROLL>
__device__ void ring_reducescatter(RingCtx& r, const Fn& fn, const RingWork& w, int c) {
  using T = typename Fn::EltType;
  const int n = w.nRanks;
  const int64_t count = (int64_t)w.count;
  int64_t gridOff, chCount, chunkCount;
  if (!cbd_part(w, c, &gridOff, &chCount, &chunkCount)) return;
  const T* in = (const T*)w.sendbuff;
  T* out = (T*)w.recvbuff;
  const int* ringRanks = r.ch->ringRanks;
  // A chunk for rank k sits in its slots at k's block misalignment (the same
  // on every rank: dataOff is a 16-byte multiple), so the FIFO operand shares
  // the input block's alignment (reduce_copy_misaligned).
  auto mis = [&](int k) { return (int)(((int64_t)k * count * (int64_t)sizeof(T)) & 15); };
  for (int64_t eo = 0; eo < chCount; eo += chunkCount) {
    const int64_t nelem = chCount - eo < chunkCount ? chCount - eo : chunkCount;
    const int64_t dataOff = gridOff + eo;
    int rankDest = ringRanks[n - 1];
    ring_step<Fn, false, true, true, false, UNROLL>(r, fn, in + dataOff + rankDest * count, nullptr, nelem,
                                                    false, 0, mis(rankDest));
    for (int j = 2; j < n; ++j) {
      rankDest = ringRanks[n - j];
      ring_step<Fn, true, true, true, false, UNROLL>(r, fn, in + dataOff + rankDest * count, nullptr,
                                                     nelem, false, mis(rankDest), mis(rankDest));
    }
    rankDest = ringRanks[0];
    ring_step<Fn, true, false, true, true, UNROLL>(r, fn, in + dataOff + rankDest * count, out + dataOff,
                                                   nelem, true, mis(rankDest), 0);
  }
}

// ----------------------------------------------------------------- AllGather
// all_gather.h:12-83: byte copies (enqueue.cc:2400-2404 rewrites AG as int8).
template <int UNROLL>
__device__ void ring_allgather(RingCtx& r, const RingWork& w, int c) {
  using Fn = FnCopy<uint8_t>;
  const Fn fn(0);
  const int n = w.nRanks;
  const int64_t count = (int64_t)w.count;  // bytes per rank
  int64_t partOff, partCount, chunkCount;
  if (!cbd_part(w, c, &partOff, &partCount, &chunkCount)) return;
  const uint8_t* in = (const uint8_t*)w.sendbuff;
  uint8_t* out = (uint8_t*)w.recvbuff;
  const int* ringRanks = r.ch->ringRanks;
  // A block for rank k travels at k's output misalignment inside the slots
  // (same on every rank), so the slot and the output block share alignment.
  auto mis = [&](int k) { return (int)(((int64_t)k * count) & 15); };
  for (int64_t eo = 0; eo < partCount; eo += chunkCount) {
    const int64_t nelem = partCount - eo < chunkCount ? partCount - eo : chunkCount;
    const int64_t dataOff = partOff + eo;
    int rankDest = ringRanks[0];
    int64_t off = dataOff + rankDest * count;
    if (in + dataOff == out + off)
      ring_step<Fn, false, true, true, false, UNROLL>(r, fn, in + dataOff, nullptr, nelem, false, 0,
                                                      mis(rankDest));
    else
      ring_step<Fn, false, true, true, true, UNROLL>(r, fn, in + dataOff, out + off, nelem, false, 0,
                                                     mis(rankDest));
    for (int j = 1; j < n - 1; ++j) {
      rankDest = ringRanks[n - j];
      off = dataOff + rankDest * count;
      ring_step<Fn, true, true, false, true, UNROLL>(r, fn, nullptr, out + off, nelem, false, mis(rankDest),
                                                     mis(rankDest));
    }
    rankDest = ringRanks[1];
    off = dataOff + rankDest * count;
    ring_step<Fn, true, false, false, true, UNROLL>(r, fn, nullptr, out + off, nelem, false, mis(rankDest),
                                                    0);
  }
}

}  // namespace vccl
