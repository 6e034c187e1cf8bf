// Two-shot direct all-reduce over the fully connected xGMI mesh, for
// mid-size buckets (between the one-shot LL path and the SIMPLE ring).
//
// Reference role: the mid-range protocol slot of VCCL's tuner (LL128 ring,
// prims_ll128.h:11-434, chosen by enqueue.cc:2032 for 64 KiB - 8 MiB).  NCCL
// fills that slot with a cheaper-per-byte protocol on the SAME 2(n-1)-hop
// ring; on MI355X every GPU pair has its own xGMI link, so the mid range is
// served by a different dependency structure instead: two hops in total.
//
//   shard o = elements [o*shardElts, (o+1)*shardElts), owned by rank o;
//   each shard is cut into nBlocks blocks, block b handled by workgroup b
//   on every rank (so a workgroup only ever waits for its namesakes).
//   phase 1 (scatter): rank r writes block b of every foreign shard p into
//            p's inbox region (0, r), then raises flag (0, r, b) at p;
//   phase 2 (reduce):  rank o waits for the n-1 flags (0, *, b) and folds
//            its block exactly as VCCL's ring all-reduce folds those elements:
//            every element belongs to a ring chunk c of one loop of its
//            channel's ncclCollCbdPart (ar_chunk_of, the ring's own partition
//            on the comm's channels and ring set), which the ring folds from
//            position c+1 around to c, x_{R[c+1]} (+) ... (+) x_{R[c]}, preOp
//            on every input, postOp once (all_reduce.h:42-64); each wave of
//            the workgroup walks its span of the block chunk by chunk in that
//            order — then writes the result to its own output and to every
//            peer's inbox region (1, o), and raises flag (1, o, b) there;
//   phase 3 (gather):  every rank waits for the n-1 flags (1, *, b) and copies
//            the owners' blocks from its inbox into its output.
// Buckets larger than the inbox move through it in chunks (the three phases
// per chunk, one launch); shards and blocks are laid out per chunk.
// Payload moves with sc0 sc1 (write-through, L2-bypassing) 16-byte accesses,
// each storing wave drains (s_waitcnt vmcnt(0)) before the workgroup barrier
// and the relaxed system-scope flag store: the same hand-off as the ring
// slots (ring.hpp).  Flags carry the call epoch (device-resident, see
// epoch_next), so no buffer is ever cleared and graph replays stay in step.
//
// Buffer reuse.  Every guarantee is per block: workgroup b of every rank
// only ever touches the inbox bytes [b * blkElts, (b + 1) * blkElts) of a
// region, so the per-block flags order all reuse of those bytes.  A fused
// batch (DirectBatch) keeps that true across its parts by giving every part
// ONE block length (host/enqueue.cc launch_direct).
//  * the all-reduce double-buffers its chunks by parity (regions and flags,
//    direct_allreduce_part): parity p is rewritten for chunk c+2 only after
//    the readers' flags of chunk c were awaited;
//  * the one-hop reduce-scatter / all-gather use parity 0 only and guard
//    reuse with explicit acknowledgements (phase 3 below);
// and a region of one parity is rewritten by its writer's next chunk, part
// or call only after its reader's flag for the previous use, so any of the
// three kernels may follow any other on the same inbox (a peer one call
// ahead writes only (0, *) regions, which the previous call has finished
// reading before that peer could complete it).
#pragma once
#include "coll_types.hpp"
#include "ll.hpp"
#include "reduce_copy.hpp"
#include "ring_types.hpp"

namespace vccl {

// 16-byte packs per thread in flight in the single-source copies (scatter,
// broadcast, gather); the n-source folds keep kDirectUnroll.  4 was A/B'd in
// the 4-rank rehearsal (profiles/r02x): reduce-scatter 64 MiB -10 %, all-
// reduce / all-gather level, small buckets noisier — left at 2.
#ifndef VCCL_DIRECT_COPY_UNROLL
#define VCCL_DIRECT_COPY_UNROLL 2
#endif
constexpr int kDirectCopyUnroll = VCCL_DIRECT_COPY_UNROLL;

// Fold up to kDirectMaxRanks sources into up to kDirectMaxRanks destinations:
// dst_d[i] = postOp(pre?(src_0[i]) (+) pre?(src_1[i]) (+) ...), preOp on
// sources s < preN.  All sources' loads of a hunk are issued before the first
// reduce (the inbox latency is paid once per hunk, not once per source).
// STP_LAST: policy of the last destination (the own output); others STP.
// Own outputs that are the only destination are stored write-through (sc0
// sc1): the copy shape runs at 7.13 TB/s that way against 6.68 with plain
// stores (tools/sweep_rc.py twodst, profiles/r03a).
template <class Fn, int U, int LDP, int STP, int STP_LAST>
__device__ __forceinline__ void direct_rc(const Fn& fn, const char* const (&src)[kDirectMaxRanks],
                                          int nS, int preN, bool post,
                                          char* const (&dst)[kDirectMaxRanks], int nD,
                                          int64_t nElts, int tid, int nthreads) {
  using T = typename Fn::EltType;
  if (nElts <= 0) return;
  uintptr_t bits = 0;
#pragma unroll
  for (int s = 0; s < kDirectMaxRanks; s++)
    if (s < nS) bits |= (uintptr_t)src[s];
#pragma unroll
  for (int d = 0; d < kDirectMaxRanks; d++)
    if (d < nD) bits |= (uintptr_t)dst[d];
#ifdef VCCL_DIRECT_MIS_ELEMENTS  // A/B: the element path for any misalignment
  const bool elemOnly = (bits & 15) != 0;
  if (false) {
#else
  const bool elemOnly = false;
  if (bits & 15) {
#endif
    // Misaligned user buffers: the reduce-copy engine (reduce_copy.hpp) keeps
    // 16-byte packs whenever the destinations share one misalignment —
    // sources at other offsets are realigned by wavefront shuffle + funnel
    // shift.  The callers below arrange that (a misaligned own output is
    // staged through the aligned inbox).  Stores all write-through here.
    RCArgs a;
#pragma unroll
    for (int q = 0; q < kDirectMaxRanks; q++) {
      a.srcs[q] = q < nS ? src[q] : src[0];
      a.dsts[q] = q < nD ? dst[q] : dst[0];
    }
    a.nSrcs = nS;
    a.nDsts = nD;
    a.preOpSrcs = preN;
    a.postOp = post ? 1 : 0;
    a.argPtr = nullptr;
    a.argBytes = 0;
    constexpr int P = uniform_pol(LDP, kSys);
    // Compile-time operand counts select the engine's batched shifted loop
    // (every load of a hunk issued before the shuffles): the scatter / gather
    // copies (1 -> 1) and the phase-2 fold (n -> n).
    if (nS == 1 && nD == 1) {
      reduce_copy<Fn, 1, 1, 2, P, 0, false, false>(fn, a, nElts, 0, 1, tid, nthreads);
      return;
    }
    if (nD == 1 && nS > 1) {  // reduce-scatter fold: n -> 1
      switch (nS) {
        case 2: reduce_copy<Fn, 2, 1, 1, P, 0, false, false>(fn, a, nElts, 0, 1, tid, nthreads); return;
        case 3: reduce_copy<Fn, 3, 1, 1, P, 0, false, false>(fn, a, nElts, 0, 1, tid, nthreads); return;
        case 4: reduce_copy<Fn, 4, 1, 1, P, 0, false, false>(fn, a, nElts, 0, 1, tid, nthreads); return;
        case 8: reduce_copy<Fn, 8, 1, 1, P, 0, false, false>(fn, a, nElts, 0, 1, tid, nthreads); return;
        default: break;
      }
    }
    if (nS == nD) {
      switch (nS) {
        case 2: reduce_copy<Fn, 2, 2, 1, P, 0, false, false>(fn, a, nElts, 0, 1, tid, nthreads); return;
        case 3: reduce_copy<Fn, 3, 3, 1, P, 0, false, false>(fn, a, nElts, 0, 1, tid, nthreads); return;
        case 4: reduce_copy<Fn, 4, 4, 1, P, 0, false, false>(fn, a, nElts, 0, 1, tid, nthreads); return;
        case 8: reduce_copy<Fn, 8, 8, 1, P, 0, false, false>(fn, a, nElts, 0, 1, tid, nthreads); return;
        default: break;
      }
    }
    reduce_copy<Fn, 0, 0, 1, P, 0, true, false>(fn, a, nElts, 0, 1, tid, nthreads);
    return;
  }
  const int64_t nPacks = elemOnly ? 0 : nElts * (int64_t)sizeof(T) / 16;
  const int64_t hunk = (int64_t)nthreads * U;
  for (int64_t base = 0; base < nPacks; base += hunk) {
    u32x4 v[kDirectMaxRanks][U];
#pragma unroll
    for (int s = 0; s < kDirectMaxRanks; s++) {
      if (s < nS) {
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int64_t p = base + u * nthreads + tid;
          if (p < nPacks) v[s][u] = ld16<LDP>(src[s], p * 16);
        }
      }
    }
    u32x4 acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      acc[u] = v[0][u];
      if (Fn::kPreOp && preN > 0) acc[u] = pack_preop(fn, acc[u]);
#pragma unroll
      for (int s = 1; s < kDirectMaxRanks; s++) {
        if (s < nS) {
          u32x4 t = v[s][u];
          if (Fn::kPreOp && s < preN) t = pack_preop(fn, t);
          acc[u] = pack_reduce(fn, acc[u], t);
        }
      }
      if (Fn::kPostOp && post) acc[u] = pack_postop(fn, acc[u]);
    }
#pragma unroll
    for (int d = 0; d < kDirectMaxRanks; d++) {
      if (d < nD) {
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int64_t p = base + u * nthreads + tid;
          if (p < nPacks) {
            if (d == nD - 1) st16<STP_LAST>(dst[d], p * 16, acc[u]);
            else st16<STP>(dst[d], p * 16, acc[u]);
          }
        }
      }
    }
  }
  // Element path: the < 16-byte tail.
  for (int64_t i = nPacks * 16 / (int64_t)sizeof(T) + tid; i < nElts; i += nthreads) {
    T acc = ldT<LDP, T>(src[0], i);
    if (Fn::kPreOp && preN > 0) acc = fn.preOp(acc);
#pragma unroll
    for (int s = 1; s < kDirectMaxRanks; s++) {
      if (s < nS) {
        T x = ldT<LDP, T>(src[s], i);
        if (Fn::kPreOp && s < preN) x = fn.preOp(x);
        acc = fn.reduce(acc, x);
      }
    }
    if (Fn::kPostOp && post) acc = fn.postOp(acc);
#pragma unroll
    for (int d = 0; d < kDirectMaxRanks; d++) {
      if (d < nD) {
        if (d == nD - 1) stT<STP_LAST, T>(dst[d], i, acc);
        else stT<STP, T>(dst[d], i, acc);
      }
    }
  }
}

// Copy nBytes from a 16-byte-aligned source to nD 16-byte-aligned
// destinations (write-through): the direct all-reduce's broadcast of a
// folded chunk (both ends are the output / inbox, aligned by construction),
// kept apart from the engine so no misaligned variant is instantiated.  The
// source was just stored by the same wave (plain stores, drained): plain
// loads read it back through the CU's own cache path.
template <int U>
__device__ __forceinline__ void direct_bcast(const char* src, char* const (&dst)[kDirectMaxRanks], int nD,
                                             int64_t nBytes, int tid, int nthreads) {
  const int64_t nPacks = nBytes / 16;
  for (int64_t base = 0; base < nPacks; base += (int64_t)nthreads * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t p = base + u * nthreads + tid;
      if (p < nPacks) v[u] = ld16<kPlain>(src, p * 16);
    }
#pragma unroll
    for (int d = 0; d < kDirectMaxRanks; d++) {
      if (d < nD) {
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int64_t p = base + u * nthreads + tid;
          if (p < nPacks) st16<kSys>(dst[d], p * 16, v[u]);
        }
      }
    }
  }
  for (int64_t i = nPacks * 16 + tid; i < nBytes; i += nthreads) {
    const uint8_t x = ldT<kPlain, uint8_t>(src, i);
#pragma unroll
    for (int d = 0; d < kDirectMaxRanks; d++)
      if (d < nD) stT<kSys, uint8_t>(dst[d], i, x);
  }
}

// Wait until every peer's flag (phase, parity, peer, b) in MY flag array
// equals e.  Lane p of wave 0 polls peer p; bounded like RingCtx::spin_ge.
__device__ __forceinline__ bool direct_wait(const DirectWork& w, const char* myFlags, int phase,
                                            int parity, int b, uint32_t e, int* shFail) {
  const int t = threadIdx.x;
  if (t < w.nRanks && t != w.rank) {
    const uint32_t* f = (const uint32_t*)(myFlags + direct_flag_off(phase, parity, t, b));
    const DevComm* comm = w.comm;
    uint64_t spins = 0, start = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != e) {
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 255) == 0) {
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (start == 0) start = now;
        if (*comm->abortFlag ||
            __hip_atomic_load(comm->errorFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
          *shFail = 1;
          break;
        }
        if (now - start > comm->spinTimeoutTicks) {
          __hip_atomic_store(comm->errorFlag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          *shFail = 1;
          break;
        }
      }
    }
    // VCCL_FENCES=1: the system-scope acquire the ring takes per slot (the
    // default needs none: sc0 sc1 loads of uncached inboxes)
    if (comm->useFences) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  return *shFail == 0;
}

// Every storing wave drains, then lane k of wave 0 raises flag (phase,
// parity, me, b) at peer (me + k) mod n.
__device__ __forceinline__ void direct_post(const DirectWork& w, const DirectPeers& P, int phase,
                                            int parity, int b, uint32_t e) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int k = threadIdx.x;
  if (k >= 1 && k < w.nRanks) {
    const int p = w.rank + k < w.nRanks ? w.rank + k : w.rank + k - w.nRanks;
    if (w.comm->useFences) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // VCCL_FENCES=1, as the ring
    __hip_atomic_store((uint32_t*)(P.flags[p] + direct_flag_off(phase, parity, w.rank, b)), e,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---------------------------------------------------------------- all-reduce
// One call (one part of a batch).  `e` carries the epoch across chunks and
// parts: chunk c raises the (c+1)-th successor of the value it enters with
// (epoch_after: never 0, the never-written flag value); the batch's last
// workgroup stores the final one back (epoch_retire: graph-replay safe).
//
// Chunks are double-buffered by parity c & 1 (inbox regions and flags), and
// chunk c+1's scatter is issued right after chunk c's fold, before chunk c's
// gather: the gather (local inbox -> output copies) overlaps the next chunk's
// outgoing traffic.  Reuse of parity p = (c+1) & 1 is safe: region (0, me)
// at peer q held chunk c-1, which q folded before raising flag (1, *, c-1)
// — awaited by this workgroup in the previous iteration; region (1, o) of
// parity p at a reader is rewritten by o for chunk c+2 only after o received
// the reader's scatter of chunk c+2, which the reader issues after its gather
// of chunk c.  Per-parity flags: a flag of parity p is raised again (chunk
// c+2) only after its reader awaited chunk c's value (same chains).
template <class Fn>
__device__ void direct_allreduce_part(const DirectWork& w, uint32_t& e, int& shFail) {
  using T = typename Fn::EltType;
  const Fn fn(load_op_arg(w.redArgPtr, w.redArgBytes, w.redArg));
  const DirectPeers& P = *w.peers;
  const int n = w.nRanks, me = w.rank, b = blockIdx.x;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int64_t eltAlign = 16 / sizeof(T) ? 16 / sizeof(T) : 1;
  constexpr int64_t esz = (int64_t)sizeof(T);
  char* myBuf = P.buf[me];
  const char* myFlags = P.flags[me];
  const int64_t inOff = (int64_t)b * w.blkElts * esz;  // block offset in a region

  auto chunk_geom = [&](int c, int64_t* c0, int64_t* cc, int64_t* shardElts) {
    *c0 = (int64_t)c * w.chunkElts;
    const int64_t rest = (int64_t)w.count - *c0;
    *cc = rest < w.chunkElts ? rest : w.chunkElts;
    *shardElts = direct_shard_elts(*cc, n, eltAlign);
  };
  auto block_of = [&](int64_t cc, int64_t shardElts, int o, int64_t* off, int64_t* len) {
    int64_t shardEnd = (int64_t)(o + 1) * shardElts;
    shardEnd = shardEnd < cc ? shardEnd : cc;
    const int64_t lo = (int64_t)o * shardElts + (int64_t)b * w.blkElts;
    const int64_t hi = lo + w.blkElts < shardEnd ? lo + w.blkElts : shardEnd;
    *off = lo;
    *len = hi > lo ? hi - lo : 0;
  };
  // Phase 1: scatter my blocks of chunk c's foreign shards into their
  // owners' inboxes (parity c & 1).  Workgroup b starts at peer offset
  // 1 + b mod (n-1), so a rank's workgroups feed all n-1 outgoing links.
  auto scatter = [&](int c) {
    int64_t c0, cc, shardElts;
    chunk_geom(c, &c0, &cc, &shardElts);
    const char* in = (const char*)w.sendbuff + c0 * esz;
    for (int i = 0; i < n - 1; i++) {
      const int k = 1 + (b + i) % (n - 1);
      const int p = me + k < n ? me + k : me + k - n;
      int64_t off, len;
      block_of(cc, shardElts, p, &off, &len);
      const char* s[kDirectMaxRanks] = {in + off * esz};
      char* d[kDirectMaxRanks] = {P.buf[p] + direct_region_off(0, c & 1, me, n, w.regionBytes) + inOff};
      direct_rc<Fn, kDirectCopyUnroll, kSys, kSys, kSys>(fn, s, 1, 0, false, d, 1, len, tid, nt);
    }
  };

  if (w.nChunks <= 0) return;
  uint32_t eCur = epoch_after(e);
  if (!shFail) {
    scatter(0);
    direct_post(w, P, 0, 0, b, eCur);
  }
  for (int c = 0; c < w.nChunks; c++) {
    const int par = c & 1;
    const uint32_t eNext = epoch_after(eCur);
    int64_t c0, cc, shardElts;
    chunk_geom(c, &c0, &cc, &shardElts);
    const char* in = (const char*)w.sendbuff + c0 * esz;
    char* out = (char*)w.recvbuff + c0 * esz;
    // Block offsets are 16-byte multiples, so every block of `out` shares the
    // chunk base's misalignment (the inbox regions are 16-byte aligned).
#ifdef VCCL_DIRECT_MIS_ELEMENTS
    const bool outMis = false;
#else
    const bool outMis = ((uintptr_t)out & 15) != 0;
#endif
    // Phase 2: fold my shard's block b in the ring's order; send it out.
    if (!shFail && direct_wait(w, myFlags, 0, par, b, eCur, &shFail)) {
      int64_t off, len;
      block_of(cc, shardElts, me, &off, &len);
      // Each wave takes a contiguous span of the block (whole 16-byte packs)
      // and walks it ring chunk by ring chunk: a chunk boundary splits one
      // wave's pass, not the workgroup's.
      // wave index made provably wave-uniform: everything derived from it
      // (span, chunk lookup, operand pointers) stays in SGPRs
      const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6), nw = nt >> 6;
      const int64_t span = ((len + eltAlign - 1) / eltAlign + nw - 1) / nw * eltAlign;
      int64_t cur = (int64_t)wv * span < len ? (int64_t)wv * span : len;
      const int64_t wend = cur + span < len ? cur + span : len;
      while (cur < wend) {
        int k;
        int64_t segEnd;
        const int ch = ar_chunk_of(w.cbd, w.arChunk, n, eltAlign, c0 + off + cur, &k, &segEnd);
        segEnd -= c0 + off;
        const int64_t end = segEnd < wend ? segEnd : wend;
        const int8_t* R = w.comm->ringAt[ch % w.comm->nRings];
        // (a) fold: sources in ring order, positions k+1, ..., k (my own
        // input where the position is mine, else my inbox region of that
        // rank) -> my output (staged in my own aligned region (1, me) when
        // the output is off 16-byte alignment, copied out in phase 3).
        char* res = outMis ? myBuf + direct_region_off(1, par, me, n, w.regionBytes) + inOff + cur * esz
                           : out + (off + cur) * esz;
        {
          const char* s[kDirectMaxRanks];
          char* d[kDirectMaxRanks] = {res};
#pragma unroll
          for (int j = 0; j < kDirectMaxRanks; j++) {
            int pos = k + 1 + j;
            pos = pos >= n ? pos - n : pos;
            pos = pos >= n ? pos - n : pos;
            const int q = j < n ? __builtin_amdgcn_readfirstlane(R[pos]) : me;
            s[j] = q == me ? in + (off + cur) * esz
                           : myBuf + direct_region_off(0, par, q, n, w.regionBytes) + inOff + cur * esz;
          }
          direct_rc<Fn, kDirectUnroll, kSys, kPlain, kPlain>(fn, s, n, w.preOp ? n : 0, true, d, 1,
                                                             end - cur, lane, 64);
        }
        // (b) broadcast: this wave reads back what it just stored (same
        // wave, drained) and writes it into every peer's region (1, me).
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        {
          const char* s[kDirectMaxRanks] = {res};
          char* d[kDirectMaxRanks];
#pragma unroll
          for (int j = 0; j < kDirectMaxRanks; j++) {
            const int dst = me + j + 1 < n ? me + j + 1 : me + j + 1 - n;
            d[j] = j < n - 1
                       ? P.buf[dst] + direct_region_off(1, par, me, n, w.regionBytes) + inOff + cur * esz
                       : nullptr;
          }
          direct_bcast<kDirectCopyUnroll>(s[0], d, n - 1, (end - cur) * esz, lane, 64);
        }
        cur = end;
      }
    }
    if (!shFail) direct_post(w, P, 1, par, b, eCur);
    // Chunk c+1's scatter before chunk c's gather (see above).
    if (c + 1 < w.nChunks && !shFail) {
      scatter(c + 1);
      direct_post(w, P, 0, par ^ 1, b, eNext);
    }
    // Phase 3: gather the other owners' reduced blocks (and my own, if staged).
    if (!shFail && direct_wait(w, myFlags, 1, par, b, eCur, &shFail)) {
      for (int k = outMis ? 0 : 1; k < n; k++) {
        const int o = me + k < n ? me + k : me + k - n;
        int64_t off, len;
        block_of(cc, shardElts, o, &off, &len);
        const char* s[kDirectMaxRanks] = {myBuf + direct_region_off(1, par, o, n, w.regionBytes) + inOff};
        char* d[kDirectMaxRanks] = {out + off * esz};
        direct_rc<Fn, kDirectCopyUnroll, kSys, kSys, kSys>(fn, s, 1, 0, false, d, 1, len, tid, nt);
      }
    }
    __syncthreads();  // this chunk's region reads precede later posts
    e = eCur;
    eCur = eNext;
  }
}

// ------------------------------------------------------------ reduce-scatter
// One-hop reduce-scatter over the full mesh (the mid-range slot of VCCL's
// tuner, LL128 ring, prims_ll128.h:176-324 / enqueue.cc:2032): my block p of
// the input goes straight to rank p.  Per chunk of the recvcount block:
//   phase 1 (scatter): block b of my contribution to every peer p's block
//            -> p's inbox region (0, me); raise flag (0, me, b) at p;
//   phase 2 (fold):    wait for the n-1 flags (0, *, b); fold my block b from
//            the n-1 regions and my own input, per channel part in the order
//            of that part's ring (DirectPeers::rsOrder, the ring's fold), preOp
//            on every input, postOp once, into my output; raise the
//            acknowledgement (1, me, b) at every peer;
//   phase 3 (ack):     wait for the n-1 acknowledgements (1, *, b): every peer
//            has consumed what I wrote into it, so the next chunk (or call)
//            may overwrite region (0, me) there.
// count = recvcount; shards are the n blocks of the input (stride count).
// Regions and flags of parity 0 only.
template <class Fn>
__device__ void direct_reducescatter_part(const DirectWork& w, uint32_t& e, int& shFail) {
  using T = typename Fn::EltType;
  constexpr int64_t esz = (int64_t)sizeof(T);
  const Fn fn(load_op_arg(w.redArgPtr, w.redArgBytes, w.redArg));
  const DirectPeers& P = *w.peers;
  const int n = w.nRanks, me = w.rank, b = blockIdx.x;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int64_t count = (int64_t)w.count;
  char* myBuf = P.buf[me];
  const char* myFlags = P.flags[me];
  const char* in = (const char*)w.sendbuff;
  char* out = (char*)w.recvbuff;
  for (int c = 0; c < w.nChunks; c++) {
    e = epoch_after(e);
    if (shFail) continue;
    const int64_t c0 = (int64_t)c * w.chunkElts;
    const int64_t cc = count - c0 < w.chunkElts ? count - c0 : w.chunkElts;
    const int64_t lo = c0 + (int64_t)b * w.blkElts;           // my block b, element range
    const int64_t hi = lo + w.blkElts < c0 + cc ? lo + w.blkElts : c0 + cc;
    const int64_t len = hi > lo ? hi - lo : 0;
    const int64_t rOff = (int64_t)b * w.blkElts * esz;          // its offset in a region
    // Phase 1: scatter (workgroup b starts at peer offset 1 + b mod (n-1)).
    for (int i = 0; i < n - 1; i++) {
      const int k = 1 + (b + i) % (n - 1);
      const int p = me + k < n ? me + k : me + k - n;
      const char* s[kDirectMaxRanks] = {in + ((int64_t)p * count + lo) * esz};
      char* d[kDirectMaxRanks] = {P.buf[p] + direct_region_off(0, 0, me, n, w.regionBytes) + rOff};
      direct_rc<Fn, kDirectCopyUnroll, kSys, kSys, kSys>(fn, s, 1, 0, false, d, 1, len, tid, nt);
    }
    direct_post(w, P, 0, 0, b, e);
    // Phase 2: fold per channel part in its ring's order.
    if (direct_wait(w, myFlags, 0, 0, b, e, &shFail)) {
      for (int64_t cur = lo; cur < hi;) {
        int64_t end;
        const int ch = cbd_channel_of(w.cbd, cur, &end);
        end = end < hi ? end : hi;
        const int8_t* order = w.comm->rsOrder[ch % w.comm->nRings];
        const int64_t ro = rOff + (cur - lo) * esz;
        const char* s[kDirectMaxRanks];
        char* d[kDirectMaxRanks] = {out + cur * esz};
#pragma unroll
        for (int j = 0; j < kDirectMaxRanks; j++) {
          const int q = j < n ? order[j] : me;
          s[j] = q == me ? in + ((int64_t)me * count + cur) * esz
                         : myBuf + direct_region_off(0, 0, q, n, w.regionBytes) + ro;
        }
        direct_rc<Fn, kDirectUnroll, kSys, kSys, kSys>(fn, s, n, w.preOp ? n : 0, true, d, 1,
                                                       end - cur, tid, nt);
        cur = end;
      }
    }
    direct_post(w, P, 1, 0, b, e);
    // Phase 3: the peers' acknowledgements for this chunk.
    (void)direct_wait(w, myFlags, 1, 0, b, e, &shFail);
  }
}

// ---------------------------------------------------------------- all-gather
// One-hop all-gather (byte copies, as the reference runs AG as int8,
// enqueue.cc:2398-2404): count = bytes per rank.  Per chunk:
//   phase 1 (deliver): block b of my input -> every peer's region (0, me);
//            raise (0, me, b) there;
//   phase 2 (gather):  wait for (0, *, b); copy every rank's block b (mine
//            from my input) into the output at rank * count; raise the
//            acknowledgement (1, me, b) at every peer;
//   phase 3 (ack):     wait for (1, *, b) before the next chunk (or call)
//            overwrites region (0, me) at the peers.
// Data goes through region (0, *) like the other collectives' first phase:
// a peer that finished the previous call may start this one while I still
// read (1, *) regions of a direct all-reduce's phase 3, never (0, *) ones
// (its all-reduce could only finish after my phase-2 post, i.e. after my
// last read of (0, *)).  Regions and flags of parity 0 only.
__device__ __forceinline__ void direct_allgather_part(const DirectWork& w, uint32_t& e, int& shFail) {
  using Fn = FnCopy<uint8_t>;
  const Fn fn(0);
  const DirectPeers& P = *w.peers;
  const int n = w.nRanks, me = w.rank, b = blockIdx.x;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int64_t count = (int64_t)w.count;
  char* myBuf = P.buf[me];
  const char* myFlags = P.flags[me];
  const char* in = (const char*)w.sendbuff;
  char* out = (char*)w.recvbuff;
  for (int c = 0; c < w.nChunks; c++) {
    e = epoch_after(e);
    if (shFail) continue;
    const int64_t c0 = (int64_t)c * w.chunkElts;
    const int64_t cc = count - c0 < w.chunkElts ? count - c0 : w.chunkElts;
    const int64_t lo = c0 + (int64_t)b * w.blkElts;
    const int64_t hi = lo + w.blkElts < c0 + cc ? lo + w.blkElts : c0 + cc;
    const int64_t len = hi > lo ? hi - lo : 0;
    const int64_t rOff = (int64_t)b * w.blkElts;
    // Phase 1: one read of my block, n-1 write-through stores (aligned regions).
    {
      const char* s[kDirectMaxRanks] = {in + lo};
      char* d[kDirectMaxRanks];
#pragma unroll
      for (int j = 0; j < kDirectMaxRanks; j++) {
        const int p = me + 1 + j < n ? me + 1 + j : me + 1 + j - n;
        d[j] = j < n - 1 ? P.buf[p] + direct_region_off(0, 0, me, n, w.regionBytes) + rOff : nullptr;
      }
      direct_rc<Fn, kDirectCopyUnroll, kSys, kSys, kSys>(fn, s, 1, 0, false, d, n - 1, len, tid, nt);
    }
    direct_post(w, P, 0, 0, b, e);
    // Phase 2: gather every rank's block b into the output.
    if (direct_wait(w, myFlags, 0, 0, b, e, &shFail)) {
      for (int k = 0; k < n; k++) {
        const int o = me + k < n ? me + k : me + k - n;
        const char* s[kDirectMaxRanks] = {o == me ? in + lo
                                                  : myBuf + direct_region_off(0, 0, o, n, w.regionBytes) + rOff};
        char* d[kDirectMaxRanks] = {out + (int64_t)o * count + lo};
        if (o == me && s[0] == d[0]) continue;  // in place: my block is already there
        direct_rc<Fn, kDirectCopyUnroll, kSys, kSys, kSys>(fn, s, 1, 0, false, d, 1, len, tid, nt);
      }
    }
    direct_post(w, P, 1, 0, b, e);
    (void)direct_wait(w, myFlags, 1, 0, b, e, &shFail);
  }
}

// A batch (group aggregation, DirectBatch): the parts in order, one epoch
// sequence, retired once by the last workgroup.  Every rank launches the
// same grid (the largest part's block count); a workgroup past a part's
// blocks moves nothing but still raises and awaits its namesakes' flags.
template <class Body>
__device__ __forceinline__ void direct_batch(const DirectBatch& bt, Body body) {
  __shared__ int shFail;
  const DirectWork& w = bt.w;
  uint32_t e = __hip_atomic_load(&w.comm->dEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x == 0) shFail = 0;
  __syncthreads();
  body(w, e, shFail);
  for (int i = 1; i < bt.nParts; i++) body(direct_work_with(w, bt.more[i - 1]), e, shFail);
  epoch_retire(&w.comm->dEpoch, &w.comm->dDone, e);
}

}  // namespace vccl
