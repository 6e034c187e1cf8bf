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
#ifndef VCCL_RING_OUT_POL
// Store policy of the own output when it is the only destination of a ring
// step (final reduce of a reduce-scatter, recv-copy of an all-gather):
// nontemporal, 2.6-3.3 % faster than sc0 sc1 write-through on RS / AG of a
// 512 MiB bucket (2 ranks, 3 interleaved reps, profiles/r03j).
#define VCCL_RING_OUT_POL kNT
#endif
#ifndef VCCL_RING_OUT2_POL
// Store policy of the own output beside a FIFO slot (the two-destination
// steps S+F->F+O, S->F+O, F->F+O): nontemporal (profiles/r03a twodst sweep).
#define VCCL_RING_OUT2_POL kNT
#endif

#ifndef VCCL_RING_SPOLL
// 1: prim_ws reads a missing credit once through the scalar unit before it
// drains its stores and polls (see sread_u64); 0: drain first, always.
#define VCCL_RING_SPOLL 0
#endif
#ifndef VCCL_RING_LAST_DRAINS
// 1: the wave that finishes issuing a slot last drains and posts at once
// (prim_ws); 0: every wave defers its drain past its next slot's first loads.
#define VCCL_RING_LAST_DRAINS 1
#endif

// LDS / global pointers are typed as such: through a generic pointer the
// compiler emits flat_* accesses, which vmcnt counts out of order (a wait on
// one drains every outstanding load and store, MI355X_MICROARCH.md) —
// exactly what the partial vmcnt of the per-wave hand-off must avoid.
#define VCCL_LDS __attribute__((address_space(3)))
#define VCCL_GLOBAL __attribute__((address_space(1)))

namespace vccl {

// Per-wave slot hand-off state of one channel workgroup, in LDS (prim_ws).
// done[i]: waves that completed prim p, cumulative over p = i, i + D, ...;
// tail / head: the highest credit values any wave has seen; abort: a wave's
// spin failed (abort word, peer error or timeout).
constexpr int kSyncDepth = 4;  // prims a wave may run ahead of the slowest (<= kSteps / 2)
struct WaveSync {
  uint32_t done[kSyncDepth];
  uint64_t tail, head;
  int abort;
  int poller;  // 1 while one wave polls the flags for the workgroup
};

// Flags through global-typed pointers: a generic pointer would make these
// flat_* accesses, which vmcnt retires out of order.
__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) {
  return __hip_atomic_load((const VCCL_GLOBAL uint64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint64_t* p, uint64_t v) {
  __hip_atomic_store((VCCL_GLOBAL uint64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void drain_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// A flag read through the scalar unit, globally coherent (glc: a scalar-cache
// miss, so the uncached flag is read from memory): it waits on lgkmcnt only,
// never behind the wave's outstanding vector stores — the credit check of
// the per-wave hand-off (prim_ws) reads a fresh flag without draining them.
__device__ __forceinline__ uint64_t sread_u64(const uint64_t* p) {
  uint64_t v;
  asm volatile("s_load_dwordx2 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}
template <class P>
__device__ __forceinline__ P* uniform_ptr(P* p) {  // in SGPRs (channel pointers are wave-uniform)
  const uint64_t x = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return (P*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

struct RingCtx {
  DevChannel* ch;
  const DevComm* comm;
  uint64_t recvStep, sendStep;
  int tid, nthreads;
  int slotBytes;
  int64_t ll128Slot;  // bytes per LL128 FIFO slot (LL128 ring only)
  VCCL_LDS int* shAbort;  // = &ws->abort
  VCCL_GLOBAL RingTraceRec* trace;  // this channel's timeline (DevComm::trace) or nullptr
  int traceN;           // records written by this launch
  // per-wave hand-off (prim_ws): this wave's position and its one pending
  // prim — stores issued, not yet known complete, flags not yet posted
  VCCL_LDS WaveSync* ws;
  // The channel's and comm's fields, read once at kernel start (load()):
  // read through their pointers later, each would be a memory load whose
  // value waits for every older store of the wave (vmcnt retires in order)
  // — the store drain the per-wave hand-off overlaps.  The ring order sits
  // in LDS (ds_read: lgkmcnt only).
  char* recvFifo;
  char* sendFifo;
  const uint64_t* recvTail;
  const uint64_t* sendHead;
  uint64_t* nextRecvTail;
  uint64_t* prevSendHead;
  uint32_t* sendSizes;
  const uint32_t* recvSizes;
  char* ll128Recv;
  char* ll128Send;
  int ringPos;
  VCCL_LDS int* ringRanks;
  volatile int* abortFlag;
  int* errorFlag;
  uint64_t spinTimeout;
  int useFences, pollMode, traceCap;
  int64_t waveMin;  // prim_ws: slots of at least this many bytes hand over per wave
  int lane, nWaves;
  uint32_t seq;  // prims this workgroup has started in this launch (same in every wave)
  bool pend;
  bool pSend, pRecv, pTrace;
  uint32_t pSeq, pBytes, pTraceIx;
  uint64_t pSendStep, pRecvStep;

  // Bounded spin on `flag` until pred(value); returns false on abort/timeout.
  // The timeout is per wait (no progress for spinTimeoutTicks), not per call.
  __device__ uint64_t poll(const uint64_t* flag) const {
    // pollMode 1: atomic RMW (resolved at the point of coherence, never a
    // cached copy); 0: relaxed system-scope load.
    if (pollMode == 1)
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
        if (*abortFlag) return false;
        if (now - start > spinTimeout) {
          __hip_atomic_store(errorFlag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          return false;
        }
        if (__hip_atomic_load(errorFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
          return false;
      }
    }
    return true;
  }

  // Every thread: the fields above from `c` / `m`; ringRanks (nRanks
  // entries) copied into `shRing` — the caller's barrier publishes them.
  __device__ __forceinline__ void load(DevChannel* c, const DevComm* m, int nRanks, VCCL_LDS int* shRing) {
    ch = c;
    comm = m;
    recvFifo = c->recvFifo;
    sendFifo = c->sendFifo;
    recvTail = uniform_ptr(c->recvTail);
    sendHead = uniform_ptr(c->sendHead);
    nextRecvTail = c->nextRecvTail;
    prevSendHead = c->prevSendHead;
    sendSizes = c->sendSizes;
    recvSizes = c->recvSizes;
    ll128Recv = c->ll128Recv;
    ll128Send = c->ll128Send;
    ringPos = c->ringPos;
    recvStep = c->recvStep;
    sendStep = c->sendStep;
    for (int k = tid; k < nRanks; k += nthreads) shRing[k] = c->ringRanks[k];
    ringRanks = shRing;
    abortFlag = m->abortFlag;
    errorFlag = m->errorFlag;
    spinTimeout = m->spinTimeoutTicks;
    useFences = m->useFences;
    pollMode = m->pollMode;
    traceCap = m->traceCap;
    waveMin = m->ringWaveMin;
  }

  // Net slots only (recvSizes set): the bytes the proxy landed for receive
  // step `step` must be the slice this prim computes — the sender's sendOff +
  // nelem * sizeof(T) for the same step.  A short or stale slot raises
  // kErrSlotSize (ncclInternalError) instead of being reduced.
  __device__ bool recv_size_ok(uint64_t step, uint32_t expect) {
    const uint32_t got = __hip_atomic_load((VCCL_GLOBAL uint32_t*)(recvSizes + step % kSteps), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
    if (got == expect) return true;
    __hip_atomic_store(errorFlag, kErrSlotSize, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return false;
  }

  __device__ bool aborted() const { return __hip_atomic_load(shAbort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0; }
  __device__ void set_aborted() { __hip_atomic_store(shAbort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

  // ---------------------------------------------------- per-wave hand-off
  // VCCL hands a slot over after the whole workgroup's stores have drained
  // (prims_simple.h:183-319: postPeer after the barrier).  Round 4's trace put
  // that drain at 13.2 of 65.7 us per two-destination slot (profiles/r04ap):
  // every wave idles until the slowest wave's stores are acknowledged.  Here
  // each wave hands over on its own: a wave issues slot k, moves on to slot
  // k + 1, issues k + 1's first loads, and only then waits for slot k's
  // stores with a PARTIAL `s_waitcnt vmcnt(NS * UNROLL)` (vmcnt retires loads
  // and stores in issue order, MI355X_MICROARCH.md: all but the N youngest
  // — k + 1's loads — are done), so its drain overlaps its next loads.  It
  // then counts itself done for slot k in LDS; the wave that completes the
  // count posts slot k's flags (tail to next, head to prev).  No workgroup
  // barrier per slot.  Posts stay in slot order: the poster of k + 1 counted
  // after every wave completed k + 1, which each wave does only after its
  // own earlier flag stores retired (same vmcnt, in order).  Credits: a wave
  // checks the highest values any wave has seen (LDS) and polls the flag
  // itself only when they are not enough, completing its pending slot first
  // (so no post ever waits on a peer).  A wave runs at most kSyncDepth prims
  // ahead of the slowest (the done[] ring).
  __device__ __forceinline__ void post_pending() {
    if (useFences) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system-scope release (L2 writeback)
      drain_vmem();
    }
    if (pSend && sendSizes) {
      // the net proxy reads the size once it sees the tail (proxy.cc
      // send_loop): the size must be visible first — two relaxed stores to
      // different words carry no order of their own (found when the per-wave
      // hand-off let these stores overlap the poster's next loads: a stale
      // size, hence a short slot, in test_multi_process_ranks[3-net])
      __hip_atomic_store((VCCL_GLOBAL uint32_t*)(sendSizes + pSendStep % kSteps), pBytes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      drain_vmem();
    }
    if (pSend) st_sys(nextRecvTail, pSendStep + 1);
    if (pRecv) st_sys(prevSendHead, pRecvStep + 1);
    if (pTrace) trace[pTraceIx].t4 = __builtin_amdgcn_s_memrealtime();
  }
  // Completes this wave's pending prim: its stores (all but the N youngest
  // memory operations) are done; count it, post when this wave is the last.
  template <int N>
  __device__ __forceinline__ void complete_pending() {
    if (!pend) return;
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
    if (lane == 0) {
      if (pTrace && tid == 0) trace[pTraceIx].t3 = __builtin_amdgcn_s_memrealtime();
      const uint32_t old = __hip_atomic_fetch_add(&ws->done[pSeq % kSyncDepth], 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_WORKGROUP);
      if (old + 1 == (uint32_t)nWaves * (pSeq / kSyncDepth + 1) && !aborted()) post_pending();
    }
    pend = false;
  }
  // Every wave, before the workgroup's final barrier (k_ring).
  __device__ __forceinline__ void finish() { complete_pending<0>(); }
  // Wait (LDS) until every wave completed prim q; false on abort.
  __device__ __forceinline__ bool wait_done(uint32_t q) {
    const uint32_t want = (uint32_t)nWaves * (q / kSyncDepth + 1);
    while (__hip_atomic_load(&ws->done[q % kSyncDepth], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < want) {
      if (aborted()) return false;
      __builtin_amdgcn_s_sleep(1);
    }
    return true;
  }
  // Bounded spin on a flag until it reaches `target`; every value seen goes
  // to the LDS cache `*cache` (max) at once — other waves wait on that cache
  // for targets of their own, possibly lower ones this spin passes on the way
  // (a wave behind must not wait for the poller's higher target: its own
  // slot may be what lets the peer reach it).  Lane 0 only.
  __device__ bool spin_cache(const uint64_t* flag, uint64_t target, VCCL_LDS uint64_t* cache) {
    uint64_t spins = 0, start = 0, seen = 0;
    for (;;) {
      const uint64_t v = poll(flag);
      if (v > seen) {
        seen = v;
        __hip_atomic_fetch_max(cache, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (v >= target) return true;
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 255) == 0) {
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (start == 0) start = now;
        if (*abortFlag) return false;
        if (now - start > spinTimeout) {
          __hip_atomic_store(errorFlag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          return false;
        }
        if (__hip_atomic_load(errorFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return false;
      }
    }
  }

  // The poller's spin (lane 0): BOTH flags every round, every value seen
  // published to the LDS cache at once, until its own targets are met —
  // whatever another wave waits for (tail or head, a lower target or a
  // higher one) shows in the cache as soon as it is in memory, so no wave
  // waits on the poller's own target.
  __device__ bool poll_both(uint64_t needTail, uint64_t needHead) {
    uint64_t spins = 0, start = 0, seenT = 0, seenH = 0;
    for (;;) {
      const uint64_t t = poll(recvTail), h = poll(sendHead);
      if (t > seenT) {
        seenT = t;
        __hip_atomic_fetch_max(&ws->tail, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (h > seenH) {
        seenH = h;
        __hip_atomic_fetch_max(&ws->head, h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (t >= needTail && h >= needHead) return true;
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 255) == 0) {
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (start == 0) start = now;
        if (*abortFlag) return false;
        if (now - start > spinTimeout) {
          __hip_atomic_store(errorFlag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          return false;
        }
        if (__hip_atomic_load(errorFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return false;
      }
    }
  }
  // This wave polls the flags itself (lane 0) until they reach the targets
  // (system-scope acquire after them with VCCL_FENCES); false on abort /
  // peer error / timeout.
  template <bool RECV>
  __device__ __forceinline__ bool poll_credits(uint64_t needTail, uint64_t needHead) {
    int ok = 1;
    if (lane == 0) {
      if (RECV && !spin_cache(recvTail, needTail, &ws->tail)) ok = 0;
      if (ok && needHead && !spin_cache(sendHead, needHead, &ws->head)) ok = 0;
      if (!ok) set_aborted();
      if (ok && useFences) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system-scope acquire
        drain_vmem();
      }
    }
    return __builtin_amdgcn_readfirstlane(ok) != 0;
  }
  // One poller per workgroup: the first wave that needs a credit the LDS
  // cache lacks takes the poller token and polls the flags; the others watch
  // the cache (an LDS read, no memory traffic) and take the token over when
  // it is free and the cache still falls short.  With every wave polling on
  // its own, the slot starts when the LAST wave happens to re-read the flag
  // (+1 µs per step on 256 KiB - 8 MiB rings, profiles/r05k).
  template <bool RECV>
  __device__ __forceinline__ bool wait_credits(uint64_t needTail, uint64_t needHead) {
    for (;;) {
      if (__hip_atomic_load(&ws->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= needTail &&
          __hip_atomic_load(&ws->head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= needHead)
        return true;
      if (aborted()) return false;
      int got = 0;
      if (lane == 0) {
        int expect = 0;
        got = __hip_atomic_compare_exchange_strong(&ws->poller, &expect, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP) ? 1 : 0;
      }
      if (__builtin_amdgcn_readfirstlane(got)) {
        int ok = 1;
        if (lane == 0) {
          ok = poll_both(needTail, needHead) ? 1 : 0;
          if (!ok) set_aborted();
          __hip_atomic_store(&ws->poller, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        return __builtin_amdgcn_readfirstlane(ok) != 0;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }

  template <class Fn, bool RECV, bool SEND, bool SRC, bool DST, int UNROLL>
  __device__ __forceinline__ void prim_ws(const Fn& fn, const void* src, void* dst, int64_t nelem, bool postOp, int recvOff,
                          int sendOff) {
    using T = typename Fn::EltType;
    // Slots below VCCL_RING_WAVE_MIN (latency-bound: a few KiB per wave)
    // hand over as a workgroup: without the barrier the waves drift apart and
    // every step waits for the last of them (+1 us per step from 256 KiB to
    // 8 MiB, profiles/r05k / r05m); the overlap pays from full slots up.
    // Decided before any abort check: every wave of the workgroup reaches
    // prim_wg's barriers whatever it has seen of the abort word (each wave
    // sees it at its own time; prim_wg reads it after a barrier), so barrier
    // instances keep pairing up on a failing launch.
    const bool waveMode = (nelem > 0 ? nelem * (int64_t)sizeof(T) : 0) >= waveMin;  // workgroup-uniform
    if (!waveMode) {
      complete_pending<0>();
      drain_vmem();  // a per-wave post of the previous slot retires before this slot's post
      prim_wg<Fn, RECV, SEND, SRC, DST, UNROLL>(fn, src, dst, nelem, postOp, recvOff, sendOff);
      // prim_wg stepped the counters; count the slot done for every wave
      if (tid == 0)
        __hip_atomic_fetch_add(&ws->done[seq % kSyncDepth], (uint32_t)nWaves, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
      seq++;
      return;
    }
    if (aborted()) return;
    const bool tr = trace != nullptr && traceN < traceCap && tid == 0;
    uint64_t t0 = tr ? __builtin_amdgcn_s_memrealtime() : 0;
    if (seq >= (uint32_t)kSyncDepth && !wait_done(seq - kSyncDepth)) return;
    const uint64_t needTail = RECV ? recvStep + 1 : 0;
    const uint64_t needHead = SEND && sendStep + 1 > (uint64_t)kSteps ? sendStep + 1 - kSteps : 0;
    bool have = __hip_atomic_load(&ws->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= needTail &&
                __hip_atomic_load(&ws->head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= needHead;
#if VCCL_RING_SPOLL
    if (!have && !useFences) {  // one fresh scalar read of each flag, stores still in flight
      const uint64_t t = RECV ? sread_u64(recvTail) : 0, h = needHead ? sread_u64(sendHead) : 0;
      if (lane == 0) {
        if (RECV) __hip_atomic_fetch_max(&ws->tail, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (needHead) __hip_atomic_fetch_max(&ws->head, h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      have = t >= needTail && h >= needHead;
    }
#endif
    if (!have || useFences) {
      complete_pending<0>();  // never hold a post while waiting on a peer
      if (!(useFences ? poll_credits<RECV>(needTail, needHead) : wait_credits<RECV>(needTail, needHead))) return;
    }
    if (RECV && recvSizes) {  // a net slot: the landed bytes must be this slice
      int ok = 1;
      if (lane == 0) ok = recv_size_ok(recvStep, (uint32_t)(nelem > 0 ? recvOff + nelem * (int64_t)sizeof(T) : 0));
      if (!__builtin_amdgcn_readfirstlane(ok)) {
        set_aborted();
        return;
      }
    }
    const uint64_t t1 = tr ? __builtin_amdgcn_s_memrealtime() : 0;
    constexpr int NS = (SRC ? 1 : 0) + (RECV ? 1 : 0);
    constexpr int ND = (SEND ? 1 : 0) + (DST ? 1 : 0);
    constexpr int S0 = SRC ? VCCL_RING_SRC_POL : kSys, S1 = kSys;
    constexpr int D0 = SEND ? kSys : VCCL_RING_OUT_POL, D1 = VCCL_RING_OUT2_POL;
    constexpr int POLS = mkpol(S0, S1, S1, S1, D0, D1, D1, D1);
    if (nelem > 0) {
      RCArgs a;
      int s = 0, d = 0;
      if (SRC) a.srcs[s++] = (const char*)src;
      if (RECV) a.srcs[s++] = recvFifo + (int64_t)(recvStep % kSteps) * slot_stride(slotBytes) + recvOff;
      if (SEND) a.dsts[d++] = sendFifo + (int64_t)(sendStep % kSteps) * slot_stride(slotBytes) + sendOff;
      if (DST) a.dsts[d++] = (char*)dst;
      a.nSrcs = NS;
      a.nDsts = ND;
      a.preOpSrcs = SRC ? 1 : 0;
      a.postOp = postOp ? 1 : 0;
      // the hook fires only on the aligned engine's first full hunk; every
      // other shape completes the pending prim before issuing anything
      const bool hooked = rc_all_aligned16(a) && nelem * (int64_t)sizeof(T) >= (int64_t)nthreads * UNROLL * 16;
      if (!hooked) complete_pending<0>();
      reduce_copy<Fn, NS, ND, UNROLL, POLS, 0, true>(fn, a, nelem, 0, 1, tid, nthreads,
                                                     [&]() __attribute__((always_inline)) {
                                                       complete_pending<NS * UNROLL>();
                                                     });
    } else {
      complete_pending<0>();
    }
    if (tr) {
      VCCL_GLOBAL RingTraceRec& rec = trace[traceN];
      rec.t0 = t0;
      rec.t1 = t1;
      rec.t2 = t1;
      rec.tc = __builtin_amdgcn_s_memrealtime();
      rec.shape = (RECV ? 1u : 0u) | (SEND ? 2u : 0u) | (SRC ? 4u : 0u) | (DST ? 8u : 0u);
      rec.bytes = (uint32_t)(nelem > 0 ? nelem * (int64_t)sizeof(T) : 0);
      rec.step = SEND ? sendStep : recvStep;
    }
    pSend = SEND;
    pRecv = RECV;
    pSeq = seq;
    pSendStep = sendStep;
    pRecvStep = recvStep;
    pBytes = (uint32_t)(nelem > 0 ? sendOff + nelem * (int64_t)sizeof(T) : 0);
    pTrace = trace != nullptr && traceN < traceCap;
    pTraceIx = (uint32_t)traceN;
    pend = true;
    // The last wave to finish issuing this slot is the one whose drain gates
    // the post (every other wave has moved on and counted itself): it drains
    // now instead of after its next credit check and loads, so the post comes
    // as early as the workgroup hand-off's (the others still overlap).
#if VCCL_RING_LAST_DRAINS
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&ws->done[seq % kSyncDepth], __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_WORKGROUP)) + 1 ==
        (uint32_t)nWaves * (seq / kSyncDepth + 1))
      complete_pending<0>();
#endif
    if (trace != nullptr && traceN < traceCap) traceN++;
    seq++;
    if (SEND) sendStep++;
    if (RECV) recvStep++;
  }

  // One primitive call: at most one slot of payload.
  //   srcs = [SRC ? own input] ++ [RECV ? recv slot]
  //   dsts = [SEND ? peer slot] ++ [DST ? own output]
  //   recvOff / sendOff: byte offset of the chunk inside its slot (< 16)
  // The workgroup hand-off (every ring kernel but the per-wave ones).
  template <class Fn, bool RECV, bool SEND, bool SRC, bool DST, int UNROLL>
  __device__ __forceinline__ void prim_wg(const Fn& fn, const void* src, void* dst, int64_t nelem, bool postOp,
                          int recvOff = 0, int sendOff = 0) {
    // The abort word is read by every wave only after the first barrier
    // (thread 0 skips its spins once it is set): in the per-wave kernels the
    // waves may each have seen it at a different moment before this slot.
    const bool tr = trace != nullptr && traceN < traceCap;
    uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, tc = 0;
    if (tid == 0 && !aborted()) {
      if (tr) t0 = __builtin_amdgcn_s_memrealtime();
      bool ok = true;
      if (RECV) ok = spin_ge(recvTail, recvStep + 1);
      if (SEND && ok && sendStep + 1 > (uint64_t)kSteps) ok = spin_ge(sendHead, sendStep + 1 - kSteps);
      if (RECV && ok && recvSizes)  // a net slot: the landed bytes must be this slice
        ok = recv_size_ok(recvStep, (uint32_t)(nelem > 0 ? recvOff + nelem * (int64_t)sizeof(typename Fn::EltType) : 0));
      if (!ok) set_aborted();
      if (useFences) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system-scope acquire
        drain_vmem();
      }
      if (tr) t1 = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    if (aborted()) return;
    if (tid == 0 && tr) t2 = __builtin_amdgcn_s_memrealtime();
    if (nelem > 0) {
      // Operand order and memory policy: own input streamed once (nt), FIFO
      // slots system-coherent write-through (sc0 sc1).  Own output: nt
      // (VCCL_RING_OUT_POL) when it is the only destination, nt beside a FIFO slot — the
      // two-destination shape runs at 7.13 TB/s with one write-through and
      // one nt destination, 6.0 with both write-through, 5.5 with both plain
      // (tools/sweep_rc.py twodst, profiles/r03a; PMC traffic = algorithmic
      // in every case, so the policy mix, not the bytes, sets the rate).
      constexpr int NS = (SRC ? 1 : 0) + (RECV ? 1 : 0);
      constexpr int ND = (SEND ? 1 : 0) + (DST ? 1 : 0);
      constexpr int S0 = SRC ? VCCL_RING_SRC_POL : kSys, S1 = kSys;
      constexpr int D0 = SEND ? kSys : VCCL_RING_OUT_POL, D1 = VCCL_RING_OUT2_POL;
      constexpr int POLS = mkpol(S0, S1, S1, S1, D0, D1, D1, D1);
      RCArgs a;
      int s = 0, d = 0;
      if (SRC) a.srcs[s++] = (const char*)src;
      if (RECV) a.srcs[s++] = recvFifo + (int64_t)(recvStep % kSteps) * slot_stride(slotBytes) + recvOff;
      if (SEND) a.dsts[d++] = sendFifo + (int64_t)(sendStep % kSteps) * slot_stride(slotBytes) + sendOff;
      if (DST) a.dsts[d++] = (char*)dst;
      a.nSrcs = NS;
      a.nDsts = ND;
      a.preOpSrcs = SRC ? 1 : 0;
      a.postOp = postOp ? 1 : 0;
      reduce_copy<Fn, NS, ND, UNROLL, POLS, 0, true>(fn, a, nelem, 0, 1, tid, nthreads);
    }
    if (tid == 0 && tr) tc = __builtin_amdgcn_s_memrealtime();
    drain_vmem();  // every storing wave: its write-through payload stores are complete
    __syncthreads();
    if (tid == 0) {
      if (tr) t3 = __builtin_amdgcn_s_memrealtime();
      if (useFences) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system-scope release (L2 writeback)
        drain_vmem();
      }
      if (SEND && sendSizes) {  // visible before the tail (post_pending)
        __hip_atomic_store((VCCL_GLOBAL uint32_t*)(sendSizes + sendStep % kSteps),
                           (uint32_t)(nelem > 0 ? sendOff + nelem * (int64_t)sizeof(typename Fn::EltType) : 0),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        drain_vmem();
      }
      if (SEND) st_sys(nextRecvTail, sendStep + 1);
      if (RECV) st_sys(prevSendHead, recvStep + 1);
      if (tr) {
        VCCL_GLOBAL RingTraceRec& rec = trace[traceN];
        rec.t0 = t0;
        rec.t1 = t1;
        rec.t2 = t2;
        rec.t3 = t3;
        rec.t4 = __builtin_amdgcn_s_memrealtime();
        rec.shape = (RECV ? 1u : 0u) | (SEND ? 2u : 0u) | (SRC ? 4u : 0u) | (DST ? 8u : 0u);
        rec.bytes = (uint32_t)(nelem > 0 ? nelem * (int64_t)sizeof(typename Fn::EltType) : 0);
        rec.step = SEND ? sendStep : recvStep;
        rec.tc = tc;
      }
    }
    if (tr) traceN++;
    if (SEND) sendStep++;
    if (RECV) recvStep++;
  }
};

// ---------------------------------------------------------------- LL128
// LL128 protocol (prims_ll128.h:176-324, recvReduceSendCopy / GenericOp),
// gfx950 wire format (ring_types.hpp kLL128*).  A step's data travels as
// lines of S = kLL128LaneSpan lanes x 16 bytes: lane S i + j (j < S - 1)
// carries a 16-byte data piece, lane S i + S - 1 an 8-byte data piece and the
// 8-byte flag (step + 1, as recvFlag / sendFlag).  One wave instruction moves
// 1 KiB ("a round") of 64 / S lines: lane l's piece is bytes
// [16 ((S - 1) (l / S) + l % S), +16) of the round's data, or for a flag lane
// [16 (S - 1) 64 / S + 8 (l / S), +8).  The receiver polls its round's lines
// (one 16-byte sc0 sc1 load per lane) until every flag lane shows the step,
// and uses the data of that same load: the sender's wave store (sc0 sc1
// write-through) must deliver a line whole — with 64-byte lines (default)
// the flag covers one 64-byte write request (the granule the PMC passes
// show); the 128-byte line (VCCL's 15/16 NVLink line, -DVCCL_LL128_LINE=128)
// spans two requests with no order between them and tore in r04l (the first
// 64 bytes stale under a fresh flag), so it is a probe build only.  No tail
// flag and no drain per step: the
// sender waits for the credit (head) like SIMPLE, the receiver posts the
// head after the step.  Steps and credits are the channel's SIMPLE ones.
template <class T>
__device__ __forceinline__ void ll128_put(uint64_t& lo, uint64_t& hi, int q, T x) {
  uint64_t v;
  if constexpr (sizeof(T) == 1) v = __builtin_bit_cast(uint8_t, x);
  else if constexpr (sizeof(T) == 2) v = __builtin_bit_cast(uint16_t, x);
  else if constexpr (sizeof(T) == 4) v = __builtin_bit_cast(uint32_t, x);
  else v = __builtin_bit_cast(uint64_t, x);
  if (q < 8) lo |= v << (8 * q);
  else hi |= v << (8 * (q - 8));
}
template <class T>
__device__ __forceinline__ T ll128_get(uint64_t lo, uint64_t hi, int q) {
  const uint64_t w = q < 8 ? lo >> (8 * q) : hi >> (8 * (q - 8));
  if constexpr (sizeof(T) == 1) return __builtin_bit_cast(T, (uint8_t)w);
  else if constexpr (sizeof(T) == 2) return __builtin_bit_cast(T, (uint16_t)w);
  else if constexpr (sizeof(T) == 4) return __builtin_bit_cast(T, (uint32_t)w);
  else return __builtin_bit_cast(T, w);
}
// `len` (16 or 8) bytes at byte offset b0 of `p`, zero past `nbytes`;
// `al`: p is 16-byte aligned (whole-piece access), else element by element.
template <class T, int P>
__device__ __forceinline__ u32x4 ll128_ld_piece(const char* p, int64_t b0, int len, int64_t nbytes,
                                               bool al) {
  u32x4 v = {0, 0, 0, 0};
  if (b0 >= nbytes) return v;
  if (al && b0 + len <= nbytes) {
    if (len == 16) return ld16<P>(p, b0);
    const uint64_t x = *(const uint64_t*)(p + b0);
    v.x = (uint32_t)x;
    v.y = (uint32_t)(x >> 32);
    return v;
  }
  uint64_t lo = 0, hi = 0;
#pragma unroll
  for (int q = 0; q < 16; q += (int)sizeof(T))
    if (q < len && b0 + q < nbytes) ll128_put<T>(lo, hi, q, *(const T*)(p + b0 + q));
  v.x = (uint32_t)lo;
  v.y = (uint32_t)(lo >> 32);
  v.z = (uint32_t)hi;
  v.w = (uint32_t)(hi >> 32);
  return v;
}
template <class T, int P>
__device__ __forceinline__ void ll128_st_piece(char* p, int64_t b0, int len, int64_t nbytes, bool al,
                                               u32x4 v) {
  if (b0 >= nbytes) return;
  if (al && b0 + len <= nbytes) {
    if (len == 16) st16<P>(p, b0, v);
    else *(uint64_t*)(p + b0) = (uint64_t)v.x | ((uint64_t)v.y << 32);
    return;
  }
  const uint64_t lo = (uint64_t)v.x | ((uint64_t)v.y << 32), hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
#pragma unroll
  for (int q = 0; q < 16; q += (int)sizeof(T))
    if (q < len && b0 + q < nbytes) *(T*)(p + b0 + q) = ll128_get<T>(lo, hi, q);
}

#ifndef VCCL_LL128_UNROLL
// 4 rounds per wave in flight: RS 1 / 4 MiB 6-7 % faster than 2, AR 4 MiB 3 %,
// AR 256 KiB ~1 us slower (2 ranks, 3 interleaved reps, profiles/r03k)
#define VCCL_LL128_UNROLL 4
#endif
constexpr int kLL128Unroll = VCCL_LL128_UNROLL;  // rounds in flight per wave

// One LL128 primitive call: a whole ring chunk (<= one LL128 slot).
//   src = own input (SRC), dst = own output (DST); recv / send = the slots.
template <class Fn, bool RECV, bool SEND, bool SRC, bool DST>
__device__ void ll128_prim(RingCtx& R, const Fn& fn, const void* srcv, void* dstv, int64_t nelem,
                           bool preOp, bool postOp) {
  using T = typename Fn::EltType;
  if (R.aborted()) return;
  if (R.tid == 0) {
    bool ok = true;
    if (SEND && R.sendStep + 1 > (uint64_t)kSteps) ok = R.spin_ge(R.sendHead, R.sendStep + 1 - kSteps);
    if (!ok) R.set_aborted();
  }
  __syncthreads();
  if (R.aborted()) return;
  const char* src = (const char*)srcv;
  char* dst = (char*)dstv;
  const int64_t nbytes = nelem > 0 ? nelem * (int64_t)sizeof(T) : 0;
  const int64_t nRounds = (nbytes + kLL128RoundData - 1) / kLL128RoundData;
  const uint64_t rflag = R.recvStep + 1, sflag = R.sendStep + 1;
  const char* rslot = RECV ? R.ll128Recv + (int64_t)(R.recvStep % kSteps) * R.ll128Slot : nullptr;
  char* sslot = SEND ? R.ll128Send + (int64_t)(R.sendStep % kSteps) * R.ll128Slot : nullptr;
  const int lane = R.tid & 63, wave = R.tid >> 6, nw = R.nthreads >> 6;
  constexpr int S = kLL128LaneSpan;
  const int line = lane / S, sub = lane % S;
  const bool flagLane = sub == S - 1;
  const int dOff = flagLane ? 16 * (S - 1) * kLL128LinesPerRound + 8 * line : (line * (S - 1) + sub) * 16;
  const int dLen = flagLane ? 8 : 16;
  const bool srcAl = SRC && (((uintptr_t)src & 15) == 0);
  const bool dstAl = DST && (((uintptr_t)dst & 15) == 0);
  bool fail = false;
  for (int64_t r0 = wave; r0 < nRounds && !fail; r0 += (int64_t)nw * kLL128Unroll) {
    u32x4 own[kLL128Unroll], rv[kLL128Unroll];
#pragma unroll
    for (int u = 0; u < kLL128Unroll; u++) {
      const int64_t r = r0 + (int64_t)u * nw;
      if (SRC && r < nRounds) own[u] = ll128_ld_piece<T, VCCL_RING_SRC_POL>(src, r * kLL128RoundData + dOff, dLen, nbytes, srcAl);
      if (RECV && r < nRounds) rv[u] = ld16<kSys>(rslot, r * kLL128RoundWire + lane * 16);
    }
    if (RECV) {
#pragma unroll
      for (int u = 0; u < kLL128Unroll; u++) {
        const int64_t r = r0 + (int64_t)u * nw;
        if (r >= nRounds) break;
        uint64_t spins = 0, start = 0;
        for (;;) {
          const bool ok = !flagLane || ((uint64_t)rv[u].z | ((uint64_t)rv[u].w << 32)) == rflag;
          if (__all(ok)) break;
          if ((++spins & 255) == 0) {
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            if (start == 0) start = now;
            if (*R.abortFlag ||
                __hip_atomic_load(R.errorFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ||
                now - start > R.spinTimeout) {
              __hip_atomic_store(R.errorFlag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              fail = true;
              break;
            }
          }
          __builtin_amdgcn_s_sleep(1);
          rv[u] = ld16<kSys>(rslot, r * kLL128RoundWire + lane * 16);
        }
        if (fail) break;
      }
      if (fail) break;
    }
#pragma unroll
    for (int u = 0; u < kLL128Unroll; u++) {
      const int64_t r = r0 + (int64_t)u * nw;
      if (r >= nRounds) break;
      u32x4 acc;
      if constexpr (SRC) {
        acc = own[u];
        if (Fn::kPreOp && preOp) acc = pack_preop(fn, acc);
        if constexpr (RECV) acc = pack_reduce(fn, acc, rv[u]);  // own (+) recv, as the SIMPLE ring
      } else {
        acc = rv[u];
      }
      if (Fn::kPostOp && postOp) acc = pack_postop(fn, acc);
      if constexpr (SEND) {
        u32x4 o = acc;
        if (flagLane) {
          o.z = (uint32_t)sflag;
          o.w = (uint32_t)(sflag >> 32);
        }
        st16<kSys>(sslot, r * kLL128RoundWire + lane * 16, o);
      }
      if constexpr (DST) ll128_st_piece<T, kNT>(dst, r * kLL128RoundData + dOff, dLen, nbytes, dstAl, acc);
    }
  }
  if (fail) R.set_aborted();
  __syncthreads();  // every lane's reads of the receive slot are done
  if (R.tid == 0 && RECV && !R.aborted()) st_sys(R.prevSendHead, R.recvStep + 1);
  if (SEND) R.sendStep++;
  if (RECV) R.recvStep++;
}

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
template <class Fn, bool RECV, bool SEND, bool SRC, bool DST, int UNROLL, int PROTO = kProtoSimple>
__device__ __forceinline__ void ring_step(RingCtx& r, const Fn& fn, const void* src, void* dst,
                                          int64_t nelem, bool postOp, int recvOff = 0,
                                          int sendOff = 0) {
  using T = typename Fn::EltType;
  if constexpr (PROTO == kProtoLL128) {  // a whole chunk is one LL128 step
    (void)recvOff;
    (void)sendOff;
    ll128_prim<Fn, RECV, SEND, SRC, DST>(r, fn, src, dst, nelem > 0 ? nelem : 0, SRC, postOp);
    return;
  }
  const int64_t slotElts = (int64_t)r.slotBytes / (int64_t)sizeof(T);
  const int64_t nSlices = nelem > 0 ? div_up(nelem, slotElts) : 1;
  for (int64_t s = 0; s < nSlices; s++) {
    const int64_t o = s * slotElts;
    const int64_t len = nelem - o < slotElts ? nelem - o : slotElts;
    const void* sp = SRC ? (const void*)((const T*)src + o) : nullptr;
    void* dp = DST ? (void*)((T*)dst + o) : nullptr;
    // the slot hand-off is part of the kernel's protocol (a template
    // parameter, so the workgroup and per-wave objects never define one
    // symbol two ways)
    if constexpr (PROTO == kProtoSimpleWave)
      r.template prim_ws<Fn, RECV, SEND, SRC, DST, UNROLL>(fn, sp, dp, len > 0 ? len : 0, postOp, recvOff, sendOff);
    else
      r.template prim_wg<Fn, RECV, SEND, SRC, DST, UNROLL>(fn, sp, dp, len > 0 ? len : 0, postOp, recvOff, sendOff);
  }
}

// ----------------------------------------------------------------- AllReduce
// all_reduce.h:12-83 (runRing): RS then AG within one kernel, chunk c of each
// round finishing at ring position c.
template <class Fn, int UNROLL, int PROTO = kProtoSimple>
__device__ __forceinline__ void ring_allreduce(RingCtx& r, const Fn& fn, const RingWork& w, int c) {
  using T = typename Fn::EltType;
  const int n = w.nRanks;
  const int64_t eltAlign = 16 / sizeof(T) ? 16 / sizeof(T) : 1;
  int64_t gridOff, chCount, chunkCount;
  if (!cbd_part(w, c, &gridOff, &chCount, &chunkCount)) return;
  const T* in = (const T*)w.sendbuff;
  T* out = (T*)w.recvbuff;
  const int ringIx = r.ringPos;
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
    ring_step<Fn, false, true, true, false, UNROLL, PROTO>(r, fn, in + off_of(chunk), nullptr, len_of(chunk), false);
    for (int j = 2; j < n; ++j) {          // n-2 recv-reduce-send
      chunk = modRanks(ringIx + n - j);
      ring_step<Fn, true, true, true, false, UNROLL, PROTO>(r, fn, in + off_of(chunk), nullptr, len_of(chunk),
                                                     false);
    }
    chunk = ringIx;                         // final reduce: output + send
    ring_step<Fn, true, true, true, true, UNROLL, PROTO>(r, fn, in + off_of(chunk), out + off_of(chunk),
                                                  len_of(chunk), true);
    for (int j = 1; j < n - 1; ++j) {      // n-2 recv-copy-send
      chunk = modRanks(ringIx + n - j);
      ring_step<Fn, true, true, false, true, UNROLL, PROTO>(r, fn, nullptr, out + off_of(chunk), len_of(chunk),
                                                     false);
    }
    chunk = modRanks(ringIx + 1);          // final recv
    ring_step<Fn, true, false, false, true, UNROLL, PROTO>(r, fn, nullptr, out + off_of(chunk), len_of(chunk),
                                                    false);
  }
}

// ------------------------------------------------------------- ReduceScatter
// reduce_scatter.h:12-55: the chunk owned by rank ringRanks[k] starts at its
// ring successor; the owner writes output[off] with postOp.
template <class Fn, int UNROLL, int PROTO = kProtoSimple>
__device__ __forceinline__ void ring_reducescatter(RingCtx& r, const Fn& fn, const RingWork& w, int c) {
  using T = typename Fn::EltType;
  const int n = w.nRanks;
  const int64_t count = (int64_t)w.count;
  int64_t gridOff, chCount, chunkCount;
  if (!cbd_part(w, c, &gridOff, &chCount, &chunkCount)) return;
  const T* in = (const T*)w.sendbuff;
  T* out = (T*)w.recvbuff;
  const VCCL_LDS int* ringRanks = r.ringRanks;
  // A chunk for rank k sits in its slots at k's block misalignment (the same
  // on every rank: dataOff is a 16-byte multiple), so the FIFO operand shares
  // the input block's alignment (reduce_copy_misaligned).
  auto mis = [&](int k) { return (int)(((int64_t)k * count * (int64_t)sizeof(T)) & 15); };
  for (int64_t eo = 0; eo < chCount; eo += chunkCount) {
    const int64_t nelem = chCount - eo < chunkCount ? chCount - eo : chunkCount;
    const int64_t dataOff = gridOff + eo;
    int rankDest = ringRanks[n - 1];
    ring_step<Fn, false, true, true, false, UNROLL, PROTO>(r, fn, in + dataOff + rankDest * count, nullptr, nelem,
                                                    false, 0, mis(rankDest));
    for (int j = 2; j < n; ++j) {
      rankDest = ringRanks[n - j];
      ring_step<Fn, true, true, true, false, UNROLL, PROTO>(r, fn, in + dataOff + rankDest * count, nullptr,
                                                     nelem, false, mis(rankDest), mis(rankDest));
    }
    rankDest = ringRanks[0];
    ring_step<Fn, true, false, true, true, UNROLL, PROTO>(r, fn, in + dataOff + rankDest * count, out + dataOff,
                                                   nelem, true, mis(rankDest), 0);
  }
}

// -------------------------------------------------------------------- Reduce
// reduce.h:12-55 (runRing): each chunk starts at the root's ring successor
// (send), every rank but the root adds its own input to what it receives and
// forwards it (recvReduceSend, own input as src0), and the root writes
// own ⊕ recv to its output with the postOp (recvReduceCopy) — the fold of
// the reduce-scatter chunk the root owns.  One FIFO step per chunk
// (REDUCE_CHUNKSTEPS 1).
template <class Fn, int UNROLL, int PROTO = kProtoSimple>
__device__ __forceinline__ void ring_reduce(RingCtx& r, const Fn& fn, const RingWork& w, int c) {
  using T = typename Fn::EltType;
  const int n = w.nRanks;
  int64_t partOff, partCount, chunkCount;
  if (!cbd_part(w, c, &partOff, &partCount, &chunkCount)) return;
  const T* in = (const T*)w.sendbuff;
  T* out = (T*)w.recvbuff;
  const int me = r.ringRanks[0], prev = r.ringRanks[n - 1];
  for (int64_t eo = 0; eo < partCount; eo += chunkCount) {
    const int64_t nelem = partCount - eo < chunkCount ? partCount - eo : chunkCount;
    const int64_t off = partOff + eo;
    // slot offset from the element offset: the same on every rank
    const int m = (int)((off * (int64_t)sizeof(T)) & 15);
    if (prev == w.root)
      ring_step<Fn, false, true, true, false, UNROLL, PROTO>(r, fn, in + off, nullptr, nelem, false, 0, m);
    else if (me == w.root)
      ring_step<Fn, true, false, true, true, UNROLL, PROTO>(r, fn, in + off, out + off, nelem, true, m, 0);
    else
      ring_step<Fn, true, true, true, false, UNROLL, PROTO>(r, fn, in + off, nullptr, nelem, false, m, m);
  }
}

// ----------------------------------------------------------------- AllGather
// all_gather.h:12-83: byte copies (enqueue.cc:2400-2404 rewrites AG as int8).
template <int UNROLL, int PROTO = kProtoSimple>
__device__ __forceinline__ void ring_allgather(RingCtx& r, const RingWork& w, int c) {
  using Fn = FnCopy<uint8_t>;
  const Fn fn(0);
  const int n = w.nRanks;
  const int64_t count = (int64_t)w.count;  // bytes per rank
  int64_t partOff, partCount, chunkCount;
  if (!cbd_part(w, c, &partOff, &partCount, &chunkCount)) return;
  const uint8_t* in = (const uint8_t*)w.sendbuff;
  uint8_t* out = (uint8_t*)w.recvbuff;
  const VCCL_LDS int* ringRanks = r.ringRanks;
  // A block for rank k travels at k's output misalignment inside the slots
  // (same on every rank), so the slot and the output block share alignment.
  auto mis = [&](int k) { return (int)(((int64_t)k * count) & 15); };
  for (int64_t eo = 0; eo < partCount; eo += chunkCount) {
    const int64_t nelem = partCount - eo < chunkCount ? partCount - eo : chunkCount;
    const int64_t dataOff = partOff + eo;
    int rankDest = ringRanks[0];
    int64_t off = dataOff + rankDest * count;
    if (in + dataOff == out + off)
      ring_step<Fn, false, true, true, false, UNROLL, PROTO>(r, fn, in + dataOff, nullptr, nelem, false, 0,
                                                      mis(rankDest));
    else
      ring_step<Fn, false, true, true, true, UNROLL, PROTO>(r, fn, in + dataOff, out + off, nelem, false, 0,
                                                     mis(rankDest));
    for (int j = 1; j < n - 1; ++j) {
      rankDest = ringRanks[n - j];
      off = dataOff + rankDest * count;
      ring_step<Fn, true, true, false, true, UNROLL, PROTO>(r, fn, nullptr, out + off, nelem, false, mis(rankDest),
                                                     mis(rankDest));
    }
    rankDest = ringRanks[1];
    off = dataOff + rankDest * count;
    ring_step<Fn, true, false, false, true, UNROLL, PROTO>(r, fn, nullptr, out + off, nelem, false, mis(rankDest),
                                                    0);
  }
}

// ----------------------------------------------------------------- Broadcast
// broadcast.h:12-60 (runRing): byte copies along the ring from the root —
// the root sends (copying to its output when out of place), every other
// rank receives into its output and forwards, the root's predecessor only
// receives.  One FIFO step per chunk (BROADCAST_CHUNKSTEPS 1).
template <int UNROLL, int PROTO = kProtoSimple>
__device__ __forceinline__ void ring_broadcast(RingCtx& r, const RingWork& w, int c) {
  using Fn = FnCopy<uint8_t>;
  const Fn fn(0);
  int64_t partOff, partCount, chunkCount;
  if (!cbd_part(w, c, &partOff, &partCount, &chunkCount)) return;
  const uint8_t* in = (const uint8_t*)w.sendbuff;
  uint8_t* out = (uint8_t*)w.recvbuff;
  const int me = r.ringRanks[0], next = r.ringRanks[1];
  for (int64_t eo = 0; eo < partCount; eo += chunkCount) {
    const int64_t nelem = partCount - eo < chunkCount ? partCount - eo : chunkCount;
    const int64_t off = partOff + eo;
    // the chunk travels at its offset's misalignment inside the slots (the
    // same on every rank, so sender and receiver agree)
    const int m = (int)(off & 15);
    if (me == w.root) {
      if (in == out)
        ring_step<Fn, false, true, true, false, UNROLL, PROTO>(r, fn, in + off, nullptr, nelem, false, 0, m);
      else
        ring_step<Fn, false, true, true, true, UNROLL, PROTO>(r, fn, in + off, out + off, nelem, false, 0, m);
    } else if (next == w.root) {
      ring_step<Fn, true, false, false, true, UNROLL, PROTO>(r, fn, nullptr, out + off, nelem, false, m, 0);
    } else {
      ring_step<Fn, true, true, false, true, UNROLL, PROTO>(r, fn, nullptr, out + off, nelem, false, m, m);
    }
  }
}

}  // namespace vccl
