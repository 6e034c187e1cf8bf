// Reduce-copy engine: dst_j[i] = postOp( preOp(src_0[i]) (+) src_1[i] (+) ... )
//
// Semantics: VCCL src/device/common_kernel.h:28-285 (reduceCopyPacks /
// reduceCopy): preOp on sources s < preOpSrcs, left-to-right fold, optional
// postOp, result stored to every destination; 16-byte packs only when every
// pointer is 16-byte aligned (common_kernel.h:237-241), element packs otherwise.
//
// gfx950 layout (not the reference's warp-hunk scheme): a "hunk" is
// nthreads * UNROLL packs of 16 B; lane l of the workgroup touches packs
// hunk_base + u*nthreads + l, so every wave-instruction is one contiguous
// 1 KiB global_load_dwordx4 / global_store_dwordx4 and each thread keeps
// UNROLL*NSRC 16-byte loads in flight before its first reduce.  Hunks are
// dealt to "workers" (workgroups for a grid-wide copy, one for an in-ring
// slice) round-robin.  No LDS: there is no data reuse, so staging through LDS
// would add traffic, not remove it.
//
// Memory policy per operand (POLS template word, 2 bits per operand):
//   kPlain  global_load/store
//   kNT     nontemporal (streamed once; the tuned default for user buffers)
//   kSys    buffer_load/store ... sc0 sc1: system-coherent, write-through —
//           used for ring FIFO slots shared with a peer GPU over xGMI, so a
//           drained store is visible at the peer without an L2 writeback and
//           a load never hits a stale cached line (no acquire/release fence).
#pragma once
#include "ops.hpp"

namespace vccl {

constexpr int kMaxSrcs = 8;
constexpr int kMaxDsts = 8;

enum : int { kPlain = 0, kNT = 1, kSys = 2, kSc1NT = 3 };
// Legacy names used by the launch sweep.
enum : int { kLdPlain = kPlain, kLdNT = kNT };
enum : int { kStPlain = kPlain, kStNT = kNT };

// Policy word: bits [2s, 2s+1] = source s (s < 4), bits [8+2d, 9+2d] = dest d
// (d < 4); operands beyond index 3 use the policy of index 3.
constexpr int mkpol(int s0, int s1, int s2, int s3, int d0, int d1, int d2, int d3) {
  return s0 | s1 << 2 | s2 << 4 | s3 << 6 | d0 << 8 | d1 << 10 | d2 << 12 | d3 << 14;
}
constexpr int uniform_pol(int ld, int st) { return mkpol(ld, ld, ld, ld, st, st, st, st); }
constexpr int src_pol(int POLS, int s) { return (POLS >> (2 * (s < 3 ? s : 3))) & 3; }
constexpr int dst_pol(int POLS, int d) { return (POLS >> (8 + 2 * (d < 3 ? d : 3))) & 3; }

constexpr int kSysAux = 1 | 16;  // cache-policy bits sc0 | sc1 (gfx940+ CPol)
constexpr int kSc1NTAux = 2 | 16;  // nt | sc1: streamed, L1-bypassing

// Buffer descriptor + lane offset for a system-coherent access to `a`.  The
// descriptor is built from the FIRST ACTIVE LANE's address (readfirstlane),
// so hipcc can prove it wave-uniform and emits no waterfall loop around the
// buffer op (cdna_hip_programming.md T20); every other lane's distance from
// it is the 32-bit voffset.  Every caller's lane addresses grow with the lane
// index and span < 2 GiB within a wave, so voffset >= 0 and buffers past
// 2 GiB are addressed correctly (an offset folded into a 32-bit voffset from
// a fixed base would not be).
struct SysAddr {
  __amdgpu_buffer_rsrc_t r;
  int voff;
};
__device__ __forceinline__ SysAddr sys_addr(const char* a) {
  const uint64_t x = (uint64_t)(uintptr_t)a;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  const uint64_t x0 = ((uint64_t)hi << 32) | lo;
  return {__builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)x0, 0, 0x7fffffff, 0x00020000),
          (int)(x - x0)};
}

// The same for lanes whose addresses need NOT grow with the lane index (the
// LL reduce-scatter's fold reads, where lanes of one wave may sit in
// different channel parts and so read different ranks' slots): the
// descriptor base is 1 GiB below the first active lane's address, so every
// lane within +-1 GiB of it gets a valid non-negative voffset.  Callers keep
// all of a wave's addresses inside one buffer far smaller than that.
__device__ __forceinline__ SysAddr sys_addr_window(const char* a) {
  const uint64_t x = (uint64_t)(uintptr_t)a;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  const uint64_t x0 = (((uint64_t)hi << 32) | lo) - (1ull << 30);
  return {__builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)x0, 0, 0x7fffffff, 0x00020000),
          (int)(x - x0)};
}

template <int P>
__device__ __forceinline__ u32x4 ld16(const char* base, int64_t off) {
  if constexpr (P == kNT) return __builtin_nontemporal_load((const u32x4*)(base + off));
  else if constexpr (P == kSys || P == kSc1NT) {
    const SysAddr s = sys_addr(base + off);
    return __builtin_amdgcn_raw_buffer_load_b128(s.r, s.voff, 0, P == kSys ? kSysAux : kSc1NTAux);
  } else return *(const u32x4*)(base + off);
}
template <int P>
__device__ __forceinline__ void st16(char* base, int64_t off, u32x4 v) {
  if constexpr (P == kNT) __builtin_nontemporal_store(v, (u32x4*)(base + off));
  else if constexpr (P == kSys || P == kSc1NT) {
    const SysAddr s = sys_addr(base + off);
    __builtin_amdgcn_raw_buffer_store_b128(v, s.r, s.voff, 0, P == kSys ? kSysAux : kSc1NTAux);
  } else *(u32x4*)(base + off) = v;
}

// Element-sized accesses (T = 1, 2, 4 or 8 bytes), same policies.
template <int P, typename T>
__device__ __forceinline__ T ldT(const char* base, int64_t i) {
  if constexpr (P == kSys) {
    const SysAddr s = sys_addr(base + i * (int64_t)sizeof(T));
    const auto r = s.r;
    const int off = s.voff;
    if constexpr (sizeof(T) == 1) return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, kSysAux));
    else if constexpr (sizeof(T) == 2) return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, kSysAux));
    else if constexpr (sizeof(T) == 4) return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kSysAux));
    else return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kSysAux));
  } else {
    return ((const T*)base)[i];
  }
}
template <int P, typename T>
__device__ __forceinline__ void stT(char* base, int64_t i, T v) {
  if constexpr (P == kSys) {
    const SysAddr s = sys_addr(base + i * (int64_t)sizeof(T));
    const auto r = s.r;
    const int off = s.voff;
    if constexpr (sizeof(T) == 1) __builtin_amdgcn_raw_buffer_store_b8(__builtin_bit_cast(uint8_t, v), r, off, 0, kSysAux);
    else if constexpr (sizeof(T) == 2) __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, v), r, off, 0, kSysAux);
    else if constexpr (sizeof(T) == 4) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, kSysAux);
    else {
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, kSysAux);
    }
  } else {
    ((T*)base)[i] = v;
  }
}

struct RCArgs {
  const char* srcs[kMaxSrcs];
  char* dsts[kMaxDsts];
  int nSrcs, nDsts;
  int preOpSrcs;   // preOp applied to sources s < preOpSrcs
  int postOp;      // apply postOp to the folded value
  const void* argPtr;  // ncclScalarDevice: op argument read on the device
  int argBytes;
};

// Op argument resolution, as RedOpArg::loadArg / onerank.cu:32-42.
__device__ __forceinline__ uint64_t load_op_arg(const void* p, int bytes, uint64_t deflt) {
  if (p == nullptr) return deflt;
  switch (bytes) {
    case 1: return *(const uint8_t*)p;
    case 2: return *(const uint16_t*)p;
    case 4: return *(const uint32_t*)p;
    default: return *(const uint64_t*)p;
  }
}

// Operand pointers by runtime index, through constant indices only: a dynamic
// index into the by-value kernel argument would force a private (scratch)
// copy of RCArgs.
__device__ __forceinline__ const char* src_ptr(const RCArgs& a, int s) {
  switch (s) {
    case 0: return a.srcs[0]; case 1: return a.srcs[1]; case 2: return a.srcs[2];
    case 3: return a.srcs[3]; case 4: return a.srcs[4]; case 5: return a.srcs[5];
    case 6: return a.srcs[6]; default: return a.srcs[7];
  }
}
__device__ __forceinline__ char* dst_ptr(const RCArgs& a, int d) {
  switch (d) {
    case 0: return a.dsts[0]; case 1: return a.dsts[1]; case 2: return a.dsts[2];
    case 3: return a.dsts[3]; case 4: return a.dsts[4]; case 5: return a.dsts[5];
    case 6: return a.dsts[6]; default: return a.dsts[7];
  }
}

// Runtime-index dispatch onto the compile-time policy of operand s / d.
template <int POLS>
__device__ __forceinline__ u32x4 ld16_src(const RCArgs& a, int s, int64_t off) {
  switch (s) {
    case 0: return ld16<src_pol(POLS, 0)>(a.srcs[0], off);
    case 1: return ld16<src_pol(POLS, 1)>(a.srcs[1], off);
    case 2: return ld16<src_pol(POLS, 2)>(a.srcs[2], off);
    default: return ld16<src_pol(POLS, 3)>(src_ptr(a, s), off);
  }
}
template <int POLS>
__device__ __forceinline__ void st16_dst(const RCArgs& a, int d, int64_t off, u32x4 v) {
  switch (d) {
    case 0: st16<dst_pol(POLS, 0)>(a.dsts[0], off, v); return;
    case 1: st16<dst_pol(POLS, 1)>(a.dsts[1], off, v); return;
    case 2: st16<dst_pol(POLS, 2)>(a.dsts[2], off, v); return;
    default: st16<dst_pol(POLS, 3)>(dst_ptr(a, d), off, v); return;
  }
}
template <int POLS, typename T>
__device__ __forceinline__ T ldT_src(const RCArgs& a, int s, int64_t i) {
  switch (s) {
    case 0: return ldT<src_pol(POLS, 0), T>(a.srcs[0], i);
    case 1: return ldT<src_pol(POLS, 1), T>(a.srcs[1], i);
    case 2: return ldT<src_pol(POLS, 2), T>(a.srcs[2], i);
    default: return ldT<src_pol(POLS, 3), T>(src_ptr(a, s), i);
  }
}
template <int POLS, typename T>
__device__ __forceinline__ void stT_dst(const RCArgs& a, int d, int64_t i, T v) {
  switch (d) {
    case 0: stT<dst_pol(POLS, 0), T>(a.dsts[0], i, v); return;
    case 1: stT<dst_pol(POLS, 1), T>(a.dsts[1], i, v); return;
    case 2: stT<dst_pol(POLS, 2), T>(a.dsts[2], i, v); return;
    default: stT<dst_pol(POLS, 3), T>(dst_ptr(a, d), i, v); return;
  }
}

// Full hunks over [0, nPacks) packs.  NS/ND: compile-time source/destination
// counts (0 = runtime, <= kMax*).
template <class Fn, int NS, int ND, int UNROLL, int POLS, int ORDER = 0>
__device__ __forceinline__ void rc_hunks(const Fn& fn, const RCArgs& a, int64_t nPacks,
                                         int64_t worker, int64_t nWorkers, int tid,
                                         int nthreads) {
  // ORDER 1: workgroups b, b+8, b+16, ... (one XCD under round-robin
  // dispatch) take consecutive hunks, so each XCD streams one contiguous
  // eighth of the buffer (speed only: any placement is correct).
  // ORDER 3: destination stores interleaved (pack u to every destination,
  // then pack u + 1) instead of destination by destination.
  if constexpr (ORDER == 1) {
    if (nWorkers % 8 == 0) worker = (worker % 8) * (nWorkers / 8) + worker / 8;
  }
  const int nS = NS ? NS : a.nSrcs;
  const int nD = ND ? ND : a.nDsts;
  const int64_t hunkPacks = (int64_t)nthreads * UNROLL;
  const int64_t nHunks = nPacks / hunkPacks;
  for (int64_t h = worker; h < nHunks; h += nWorkers) {
    const int64_t off = (h * hunkPacks + tid) * 16;
    const int64_t ustride = (int64_t)nthreads * 16;
    u32x4 acc[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) acc[u] = ld16<src_pol(POLS, 0)>(a.srcs[0], off + u * ustride);
    if (Fn::kPreOp && a.preOpSrcs > 0) {
#pragma unroll
      for (int u = 0; u < UNROLL; u++) acc[u] = pack_preop(fn, acc[u]);
    }
    auto fold_src = [&](int s) __attribute__((always_inline)) {
      u32x4 tmp[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; u++) tmp[u] = ld16_src<POLS>(a, s, off + u * ustride);
#pragma unroll
      for (int u = 0; u < UNROLL; u++) {
        if (Fn::kPreOp && s < a.preOpSrcs) tmp[u] = pack_preop(fn, tmp[u]);
        acc[u] = pack_reduce(fn, acc[u], tmp[u]);
      }
    };
    if constexpr (NS > 1) {
#pragma unroll
      for (int s = 1; s < NS; s++) fold_src(s);
    } else if constexpr (NS == 0) {
#pragma unroll 1
      for (int s = 1; s < nS; s++) fold_src(s);
    }
    if (Fn::kPostOp && a.postOp) {
#pragma unroll
      for (int u = 0; u < UNROLL; u++) acc[u] = pack_postop(fn, acc[u]);
    }
    auto store_dst = [&](int d) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < UNROLL; u++) st16_dst<POLS>(a, d, off + u * ustride, acc[u]);
    };
    if constexpr (ORDER == 3 && ND > 0) {
      // measurement variant: stores interleaved across destinations
#pragma unroll
      for (int u = 0; u < UNROLL; u++)
#pragma unroll
        for (int d = 0; d < ND; d++) st16_dst<POLS>(a, d, off + u * ustride, acc[u]);
    } else if constexpr (ND > 0) {
#pragma unroll
      for (int d = 0; d < ND; d++) store_dst(d);
    } else {
#pragma unroll 1
      for (int d = 0; d < nD; d++) store_dst(d);
    }
  }
  (void)nS;
  (void)nD;
}

// Software-pipelined variant for compile-time source counts: the loads of
// hunk h + nWorkers are issued BEFORE the stores of hunk h.  vmcnt counts
// loads and stores in issue order, so waiting for the next hunk's loads then
// leaves this hunk's stores in flight instead of draining them — which
// matters when stores are slow to acknowledge (write-through sc0 sc1 stores
// to a peer GPU's FIFO over xGMI): without it every iteration pays a full
// store round trip.
//
// `hook` runs once, right after the first hunk's NS * UNROLL loads are issued
// (the ring's per-wave slot hand-off completes the previous slot there with a
// partial vmcnt, so its store drain overlaps these loads: ring.hpp).
struct NoHook {
  __device__ __forceinline__ void operator()() const {}
};
template <class Fn, int NS, int ND, int UNROLL, int POLS, class Hook = NoHook>
__device__ __forceinline__ void rc_hunks_pipelined(const Fn& fn, const RCArgs& a, int64_t nPacks,
                                                   int64_t worker, int64_t nWorkers, int tid,
                                                   int nthreads, Hook&& hook = Hook{}) {
  static_assert(NS >= 1 && ND >= 1, "compile-time operand counts only");
  const int64_t hunkPacks = (int64_t)nthreads * UNROLL;
  const int64_t nHunks = nPacks / hunkPacks;
  const int64_t ustride = (int64_t)nthreads * 16;
  int64_t h = worker;
  if (h >= nHunks) return;
  u32x4 cur[NS][UNROLL];
  auto load_hunk = [&](u32x4 (&v)[NS][UNROLL], int64_t hh) __attribute__((always_inline)) {
    const int64_t off = (hh * hunkPacks + tid) * 16;
#pragma unroll
    for (int s = 0; s < NS; s++)
#pragma unroll
      for (int u = 0; u < UNROLL; u++) v[s][u] = ld16_src<POLS>(a, s, off + u * ustride);
  };
  load_hunk(cur, h);
  hook();
  for (;;) {
    const int64_t hn = h + nWorkers;
    const bool more = hn < nHunks;
    u32x4 nxt[NS][UNROLL];
    if (more) load_hunk(nxt, hn);
    u32x4 acc[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      acc[u] = cur[0][u];
      if (Fn::kPreOp && a.preOpSrcs > 0) acc[u] = pack_preop(fn, acc[u]);
#pragma unroll
      for (int s = 1; s < NS; s++) {
        u32x4 t = cur[s][u];
        if (Fn::kPreOp && s < a.preOpSrcs) t = pack_preop(fn, t);
        acc[u] = pack_reduce(fn, acc[u], t);
      }
      if (Fn::kPostOp && a.postOp) acc[u] = pack_postop(fn, acc[u]);
    }
    const int64_t off = (h * hunkPacks + tid) * 16;
#pragma unroll
    for (int d = 0; d < ND; d++)
#pragma unroll
      for (int u = 0; u < UNROLL; u++) st16_dst<POLS>(a, d, off + u * ustride, acc[u]);
    if (!more) break;
#pragma unroll
    for (int s = 0; s < NS; s++)
#pragma unroll
      for (int u = 0; u < UNROLL; u++) cur[s][u] = nxt[s][u];
    h = hn;
  }
}

// Element-granular path (misaligned pointers and the < 16 B tail),
// reduceCopyPacks<BytePerPack=sizeof(T)> equivalent.
template <class Fn, int POLS>
__device__ __forceinline__ void rc_elems(const Fn& fn, const RCArgs& a, int64_t eBegin,
                                         int64_t eEnd, int64_t gtid, int64_t gthreads) {
  using T = typename Fn::EltType;
  for (int64_t i = eBegin + gtid; i < eEnd; i += gthreads) {
    T acc = ldT<src_pol(POLS, 0), T>(a.srcs[0], i);
    if (Fn::kPreOp && a.preOpSrcs > 0) acc = fn.preOp(acc);
    for (int s = 1; s < a.nSrcs; s++) {
      T v = ldT_src<POLS, T>(a, s, i);
      if (Fn::kPreOp && s < a.preOpSrcs) v = fn.preOp(v);
      acc = fn.reduce(acc, v);
    }
    if (Fn::kPostOp && a.postOp) acc = fn.postOp(acc);
    for (int d = 0; d < a.nDsts; d++) stT_dst<POLS, T>(a, d, i, acc);
  }
}

// ------------------------------------------------------------ misaligned
// Operands that are not 16-byte aligned (common_kernel.h:237-241 drops to
// element packs for ANY misalignment).  Here the body still moves in 16-byte
// packs when every destination shares one misalignment m (mod 16):
//   head  — the first (16 - m) / sizeof(T) elements, element path;
//   body  — packs aligned on the destinations; a source whose misalignment
//           differs by k is read as ALIGNED 16-byte packs and realigned in
//           registers: lane l funnel-shifts its pack with lane l+1's (a
//           wavefront shuffle, ds_bpermute), lane 63 loads its successor
//           pack itself, v_alignbyte_b32 extracts bytes [k, k+16);
//   tail  — the last < 16 bytes, element path.
// Aligned loads never cross a 16-byte boundary, so reading the bytes of the
// first / last pack that lie outside an operand cannot fault.  Destinations
// with different misalignments fall back to the element path.

// Bytes [k, k + 16) of the 32-byte concatenation lo:hi (k wave-uniform).
__device__ __forceinline__ u32x4 funnel16(u32x4 lo, u32x4 hi, int k) {
  const uint32_t r = (uint32_t)(k & 3);
  const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  u32x4 o;
  switch (k >> 2) {
#define VCCL_FUNNEL_CASE(Q)                                               \
  case Q:                                                                 \
    o.x = __builtin_amdgcn_alignbyte(w[Q + 1], w[Q + 0], r);              \
    o.y = __builtin_amdgcn_alignbyte(w[Q + 2], w[Q + 1], r);              \
    o.z = __builtin_amdgcn_alignbyte(w[Q + 3], w[Q + 2], r);              \
    o.w = __builtin_amdgcn_alignbyte(w[Q + 4], w[Q + 3], r);              \
    break;
    VCCL_FUNNEL_CASE(0)
    VCCL_FUNNEL_CASE(1)
    VCCL_FUNNEL_CASE(2)
    default:
    VCCL_FUNNEL_CASE(3)
#undef VCCL_FUNNEL_CASE
  }
  return o;
}

// Load of source s for the shifted body: an aligned source reads its own pack
// (clamped to the last body pack, never past the body); a source k bytes past
// a 16-byte boundary reads the aligned pack at or below (clamped to pack
// nPacks, which still holds body bytes, so it cannot fault).
template <int P>
__device__ __forceinline__ u32x4 ld16_body(const char* p, int k, int64_t pk, int64_t nPacks) {
  if (k == 0) return ld16<P>(p, (pk < nPacks ? pk : nPacks - 1) * 16);
  return ld16<P>(p - k, (pk < nPacks ? pk : nPacks) * 16);
}
template <int POLS>
__device__ __forceinline__ u32x4 ld16_body_src(const RCArgs& a, int s, int k, int64_t pk,
                                               int64_t nPacks) {
  switch (s) {
    case 0: return ld16_body<src_pol(POLS, 0)>(a.srcs[0], k, pk, nPacks);
    case 1: return ld16_body<src_pol(POLS, 1)>(a.srcs[1], k, pk, nPacks);
    case 2: return ld16_body<src_pol(POLS, 2)>(a.srcs[2], k, pk, nPacks);
    default: return ld16_body<src_pol(POLS, 3)>(src_ptr(a, s), k, pk, nPacks);
  }
}
// The aligned pack at byte offset `off` below source s's start (k bytes past
// a boundary): lane 63's successor pack.
template <int POLS>
__device__ __forceinline__ u32x4 ld16_succ_src(const RCArgs& a, int s, int k, int64_t off) {
  switch (s) {
    case 0: return ld16<src_pol(POLS, 0)>(a.srcs[0] - k, off);
    case 1: return ld16<src_pol(POLS, 1)>(a.srcs[1] - k, off);
    case 2: return ld16<src_pol(POLS, 2)>(a.srcs[2] - k, off);
    default: return ld16<src_pol(POLS, 3)>(src_ptr(a, s) - k, off);
  }
}
// The next lane's value (lane l gets lane l+1's), lane 63 gets `fill`: one
// DPP `wave_shl:1` move per dword (a VALU op; lanes whose source lies past
// the wave keep the old value), no LDS round trip as ds_bpermute would take.
// Every lane of the wave must be active.
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v, uint32_t fill) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x130 /* wave_shl:1 */, 0xf, 0xf,
                                               false);
}
__device__ __forceinline__ u32x4 from_next_lane(u32x4 v, u32x4 fill) {
  u32x4 o;
  o.x = from_next_lane(v.x, fill.x);
  o.y = from_next_lane(v.y, fill.y);
  o.z = from_next_lane(v.z, fill.z);
  o.w = from_next_lane(v.w, fill.w);
  return o;
}
// The previous lane's value (lane l gets lane l-1's), lane 0 gets `fill`
// (DPP `wave_shr:1`).
__device__ __forceinline__ u32x4 from_prev_lane(u32x4 v, u32x4 fill) {
  u32x4 o;
  o.x = (uint32_t)__builtin_amdgcn_update_dpp((int)fill.x, (int)v.x, 0x138, 0xf, 0xf, false);
  o.y = (uint32_t)__builtin_amdgcn_update_dpp((int)fill.y, (int)v.y, 0x138, 0xf, 0xf, false);
  o.z = (uint32_t)__builtin_amdgcn_update_dpp((int)fill.z, (int)v.z, 0x138, 0xf, 0xf, false);
  o.w = (uint32_t)__builtin_amdgcn_update_dpp((int)fill.w, (int)v.w, 0x138, 0xf, 0xf, false);
  return o;
}
// Lane 63's value in every lane.
__device__ __forceinline__ u32x4 lane63_of(u32x4 v) {
  u32x4 o;
  o.x = __builtin_amdgcn_readlane(v.x, 63);
  o.y = __builtin_amdgcn_readlane(v.y, 63);
  o.z = __builtin_amdgcn_readlane(v.z, 63);
  o.w = __builtin_amdgcn_readlane(v.w, 63);
  return o;
}
// Lane 0's value in every lane (v_readlane into scalar registers).
__device__ __forceinline__ u32x4 lane0_of(u32x4 v) {
  u32x4 o;
  o.x = __builtin_amdgcn_readlane(v.x, 0);
  o.y = __builtin_amdgcn_readlane(v.y, 0);
  o.z = __builtin_amdgcn_readlane(v.z, 0);
  o.w = __builtin_amdgcn_readlane(v.w, 0);
  return o;
}
// This lane's pack funnel-shifted with the next lane's; lane 63 supplies
// `ext`, the successor pack (its own load, or lane 0 of the wave's next pack
// row).
__device__ __forceinline__ u32x4 realign(u32x4 cur, u32x4 ext, int k) {
  return funnel16(cur, from_next_lane(cur, ext), k);
}

// ------------------------------------------------- misaligned destinations
// Destination d whose body starts k bytes past a 16-byte boundary A (where
// destination 0, the body's reference, is aligned): its aligned pack q
// (address A + 16q) holds body bytes [16q - k, 16q + 16 - k), i.e. the last
// k bytes of body pack q - 1 and the first 16 - k of pack q.  The lane
// holding pack p stores aligned pack q = p, funnelling the previous lane's
// result with its own (DPP lane shift + v_alignbyte, the source realignment
// run backwards), so a wave row of 64 packs stores 64 aligned packs — whole
// 64 B lines when A is line-aligned, as for a buffer offset by k.  Lane 0's
// previous pack is lane 63's of the wave's previous row (v_readlane); only a
// wave span's two ends store partial packs: its first lane the first
// 16 - k bytes of its result, its last valid lane the last k bytes, each as
// <= 4 naturally aligned 8/4/2/1-byte stores (the neighbouring span's ends
// fill the rest of those packs).  Every body byte is written exactly once.
// Measured (2 x 256 MiB f32 -> 2 x 256 MiB, profiles/r02l): destinations at
// +0 / +4 B 5.85 TB/s, +0 / +12 B 5.85, against 6.25 for the same operands
// all aligned (two destinations: half the traffic is writes) — 0.94 of the
// aligned rate.  Before: the element path 3.6 (round 1); pack q = p + 1 per
// lane (rows ending mid-line) with partial stores at every row's ends
// 5.0-5.55 (profiles/r02e, r02f); plain (write-back) partial stores 2.7 (two
// partial writes of one line meet in L2 and reach HBM as read-modify-writes,
// profiles/r02g); wave-boundary packs completed through LDS after a
// workgroup barrier 5.0 (profiles/r02h); 4-row spans 5.0 (fewer partials,
// half the waves in flight, profiles/r02l_r4).

// Bytes [from, from + 8) of the 16-byte value (lo | hi << 64), zero past 16.
__device__ __forceinline__ uint64_t bytes_at(uint64_t lo, uint64_t hi, int from) {
  if (from == 0) return lo;
  if (from < 8) return (lo >> (8 * from)) | (hi << (64 - 8 * from));
  if (from == 8) return hi;
  return hi >> (8 * (from - 8));
}
// Store bytes [from, to) of v to addr + from .. addr + to - 1.
template <int P>
__device__ __forceinline__ void st_partial(char* addr, u32x4 v, int from, int to) {
  const uint64_t lo = (uint64_t)v.x | ((uint64_t)v.y << 32);
  const uint64_t hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
  while (from < to) {
    const uintptr_t a = (uintptr_t)(addr + from);
    const uint64_t x = bytes_at(lo, hi, from);
    if ((a & 7) == 0 && to - from >= 8) {
      stT<P, uint64_t>(addr + from, 0, x);
      from += 8;
    } else if ((a & 3) == 0 && to - from >= 4) {
      stT<P, uint32_t>(addr + from, 0, (uint32_t)x);
      from += 4;
    } else if ((a & 1) == 0 && to - from >= 2) {
      stT<P, uint16_t>(addr + from, 0, (uint16_t)x);
      from += 2;
    } else {
      stT<P, uint8_t>(addr + from, 0, (uint8_t)x);
      from += 1;
    }
  }
}
// Store body pack p (value v) to destination `dst` (the body start of that
// destination, k bytes past alignment).  Every lane of the wave must call it
// (the lane shift); `valid` = p < nPacks, `nextValid` = p + 1 < nPacks.
// `prevOk`: `prev` is pack p - 1 (lane 63 of the wave's previous row), so
// lane 0 stores a whole pack instead of its first 16 - k bytes; `lastRow`:
// lane 63's last k bytes are not stored by a next row's lane 0.
template <int P>
__device__ __forceinline__ void st16_realigned(char* dst, int k, int64_t p, u32x4 v, u32x4 prev,
                                               bool prevOk, bool lastRow, bool valid,
                                               bool nextValid) {
  if (k == 0) {
    if (valid) st16<P>(dst, p * 16, v);
    return;
  }
  const u32x4 pv = from_prev_lane(v, prev);
  if (!valid) return;
  char* at = dst + p * 16;
  if (prevOk || __lane_id() != 0) st16<P>(dst - k, p * 16, funnel16(pv, v, 16 - k));
  else st_partial<P>(at, v, 0, 16 - k);
  if (!nextValid || (lastRow && __lane_id() == 63)) st_partial<P>(at, v, 16 - k, 16);
}
template <int POLS>
__device__ __forceinline__ void st16_dst_realigned(const RCArgs& a, int d, int k, int64_t p, u32x4 v,
                                                   u32x4 prev, bool prevOk, bool lastRow,
                                                   bool valid, bool nextValid) {
  switch (d) {
#define VCCL_ST_CASE(D, PTR)                                                                     \
  case D:                                                                                        \
    st16_realigned<dst_pol(POLS, D)>(PTR, k, p, v, prev, prevOk, lastRow, valid, nextValid);     \
    return;
    VCCL_ST_CASE(0, a.dsts[0])
    VCCL_ST_CASE(1, a.dsts[1])
    VCCL_ST_CASE(2, a.dsts[2])
    default:
    VCCL_ST_CASE(3, dst_ptr(a, d))
#undef VCCL_ST_CASE
  }
}

// Body packs [0, nPacks) when some operand is not 16-byte aligned on the
// body (source s k_s bytes past a boundary, destination d k_d bytes).  A hunk
// gives every wave UNROLL consecutive rows of 64 packs (row u = packs
// [64u, 64u + 64) of the wave's span), so lane 63's successor pack in row u
// is lane 0's pack of row u + 1 (a v_readlane): only the span's last row
// loads lane 63's successor itself, and only the span's two ends store
// partial destination packs.  Whole waves run (the lane shift needs every
// lane); a lane past the end loads clamped packs and stores nothing.  NS / ND
// compile-time (NS > 0): every load of a hunk is issued before the first
// lane shift, so their latencies overlap.  nthreads is a multiple of 64.
template <class Fn, int NS, int ND, int UNROLL, int POLS, bool DSTR>
__device__ __forceinline__ void rc_hunks_shifted(const Fn& fn, const RCArgs& a, int64_t nPacks,
                                                 int64_t worker, int64_t nWorkers, int tid,
                                                 int nthreads) {
  static_assert(NS >= 1 && NS <= kMaxSrcs, "compile-time source count");
  const int64_t hunkPacks = (int64_t)nthreads * UNROLL;
  const int64_t nHunks = (nPacks + hunkPacks - 1) / hunkPacks;
  const int lane = __lane_id();
  const bool last = lane == 63;
  int k[NS], kd[ND];
#pragma unroll
  for (int s = 0; s < NS; s++) k[s] = (int)((uintptr_t)src_ptr(a, s) & 15);
#pragma unroll
  for (int d = 0; d < ND; d++) kd[d] = DSTR ? (int)((uintptr_t)dst_ptr(a, d) & 15) : 0;
  for (int64_t h = worker; h < nHunks; h += nWorkers) {
    // this wave's span: UNROLL rows of 64 consecutive packs
    const int64_t p0 = h * hunkPacks + (int64_t)(tid - lane) * UNROLL + lane;
    if (p0 - lane >= nPacks) continue;  // the whole wave is past the end
    u32x4 cur[NS][UNROLL];
#pragma unroll
    for (int s = 0; s < NS; s++)
#pragma unroll
      for (int u = 0; u < UNROLL; u++)
        cur[s][u] = ld16_body_src<POLS>(a, s, k[s], p0 + 64 * u, nPacks);
    u32x4 extLast[NS];  // lane 63's successor of the span's last row
#pragma unroll
    for (int s = 0; s < NS; s++) {
      extLast[s] = cur[s][UNROLL - 1];
      const int64_t pn = p0 + 64 * (UNROLL - 1) + 1;
      if (k[s] != 0 && last)
        extLast[s] = ld16_succ_src<POLS>(a, s, k[s], (pn < nPacks ? pn : nPacks) * 16);
    }
    u32x4 acc[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      auto src = [&](int s) __attribute__((always_inline)) -> u32x4 {
        if (!k[s]) return cur[s][u];
        return realign(cur[s][u], u + 1 < UNROLL ? lane0_of(cur[s][u + 1]) : extLast[s], k[s]);
      };
      acc[u] = src(0);
      if (Fn::kPreOp && a.preOpSrcs > 0) acc[u] = pack_preop(fn, acc[u]);
#pragma unroll
      for (int s = 1; s < NS; s++) {
        u32x4 v = src(s);
        if (Fn::kPreOp && s < a.preOpSrcs) v = pack_preop(fn, v);
        acc[u] = pack_reduce(fn, acc[u], v);
      }
      if (Fn::kPostOp && a.postOp) acc[u] = pack_postop(fn, acc[u]);
    }
    // Halo: the previous span's last pack (pw - 1), recomputed here — the
    // same loads and fold, so the same bits — lets lane 0 store the aligned
    // destination pack that straddles the span boundary in ONE full 16-byte
    // store; the previous span then stores no tail piece.  Only the body's
    // first span (pw == 0) and the last pack keep partial pieces.
    u32x4 halo = acc[0];
    bool useHalo = false;
    if constexpr (DSTR) {
      bool anyKd = false;
#pragma unroll
      for (int d = 0; d < ND; d++) anyKd = anyKd || kd[d] != 0;
      const int64_t pw = p0 - lane;  // first pack of this wave's span
      if (anyKd && pw > 0) {
        auto hsrc = [&](int s) __attribute__((always_inline)) -> u32x4 {
          const u32x4 raw = ld16_body_src<POLS>(a, s, k[s], pw - 1, nPacks);
          return k[s] ? funnel16(raw, lane0_of(cur[s][0]), k[s]) : raw;
        };
        halo = hsrc(0);
        if (Fn::kPreOp && a.preOpSrcs > 0) halo = pack_preop(fn, halo);
#pragma unroll
        for (int s = 1; s < NS; s++) {
          u32x4 v = hsrc(s);
          if (Fn::kPreOp && s < a.preOpSrcs) v = pack_preop(fn, v);
          halo = pack_reduce(fn, halo, v);
        }
        if (Fn::kPostOp && a.postOp) halo = pack_postop(fn, halo);
        useHalo = true;
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      const int64_t p = p0 + 64 * u;
#pragma unroll
      for (int d = 0; d < ND; d++) {
        if constexpr (DSTR)
          st16_dst_realigned<POLS>(a, d, kd[d], p, acc[u], u > 0 ? lane63_of(acc[u > 0 ? u - 1 : 0]) : halo,
                                   u > 0 || useHalo, false, p < nPacks, p + 1 < nPacks);
        else if (p < nPacks)
          st16_dst<POLS>(a, d, p * 16, acc[u]);
      }
    }
  }
}

// Runtime operand counts (any nSrcs / nDsts up to the maxima), one pack per
// thread per step.
template <class Fn, int POLS, bool DSTR>
__device__ __forceinline__ void rc_hunks_shifted_rt(const Fn& fn, const RCArgs& a, int64_t nPacks,
                                                    int64_t worker, int64_t nWorkers, int tid,
                                                    int nthreads) {
  const int64_t nSteps = (nPacks + nthreads - 1) / nthreads;
  for (int64_t h = worker; h < nSteps; h += nWorkers) {
    const int64_t p = h * nthreads + tid;
    if (p - __lane_id() >= nPacks) continue;
    auto load = [&](int s) __attribute__((always_inline)) -> u32x4 {
      const int k = (int)((uintptr_t)src_ptr(a, s) & 15);
      const u32x4 cur = ld16_body_src<POLS>(a, s, k, p, nPacks);
      if (k == 0) return cur;
      u32x4 ext = cur;
      if (__lane_id() == 63) ext = ld16_succ_src<POLS>(a, s, k, (p + 1 < nPacks ? p + 1 : nPacks) * 16);
      return realign(cur, ext, k);
    };
    u32x4 acc = load(0);
    if (Fn::kPreOp && a.preOpSrcs > 0) acc = pack_preop(fn, acc);
    for (int s = 1; s < a.nSrcs; s++) {
      u32x4 v = load(s);
      if (Fn::kPreOp && s < a.preOpSrcs) v = pack_preop(fn, v);
      acc = pack_reduce(fn, acc, v);
    }
    if (Fn::kPostOp && a.postOp) acc = pack_postop(fn, acc);
    for (int d = 0; d < a.nDsts; d++) {
      if constexpr (DSTR)
        st16_dst_realigned<POLS>(a, d, (int)((uintptr_t)dst_ptr(a, d) & 15), p, acc, acc, false,
                                 true, p < nPacks, p + 1 < nPacks);
      else if (p < nPacks)
        st16_dst<POLS>(a, d, p * 16, acc);
    }
  }
}

__device__ __forceinline__ bool rc_all_aligned16(const RCArgs& a) {
  uintptr_t bits = 0;
  for (int s = 0; s < a.nSrcs; s++) bits |= (uintptr_t)src_ptr(a, s);
  for (int d = 0; d < a.nDsts; d++) bits |= (uintptr_t)dst_ptr(a, d);
  return (bits & 15) == 0;
}

// Aligned operands: full hunks, then < one hunk of packs, then < 16 bytes.
template <class Fn, int NS, int ND, int UNROLL, int POLS, int ORDER, bool PIPE, class Hook = NoHook>
__device__ __forceinline__ void reduce_copy_aligned(const Fn& fn, const RCArgs& a, int64_t nElts,
                                                    int64_t worker, int64_t nWorkers, int tid,
                                                    int nthreads, Hook&& hook = Hook{}) {
  using T = typename Fn::EltType;
  const int64_t gtid = worker * nthreads + tid, gthreads = nWorkers * nthreads;
  const int64_t nPacks = nElts * (int64_t)sizeof(T) / 16;
  const int64_t hunkPacks = (int64_t)nthreads * UNROLL;
  const int64_t fullPacks = (nPacks / hunkPacks) * hunkPacks;
  if constexpr (PIPE && NS >= 1 && ND >= 1)
    rc_hunks_pipelined<Fn, NS, ND, UNROLL, POLS>(fn, a, fullPacks, worker, nWorkers, tid, nthreads, hook);
  else
    rc_hunks<Fn, NS, ND, UNROLL, POLS, ORDER>(fn, a, fullPacks, worker, nWorkers, tid, nthreads);
  // Remaining packs (< one hunk): one pack per thread, grid-strided.
  for (int64_t p = fullPacks + gtid; p < nPacks; p += gthreads) {
    const int64_t off = p * 16;
    u32x4 acc = ld16<src_pol(POLS, 0)>(a.srcs[0], off);
    if (Fn::kPreOp && a.preOpSrcs > 0) acc = pack_preop(fn, acc);
    for (int s = 1; s < a.nSrcs; s++) {
      u32x4 v = ld16_src<POLS>(a, s, off);
      if (Fn::kPreOp && s < a.preOpSrcs) v = pack_preop(fn, v);
      acc = pack_reduce(fn, acc, v);
    }
    if (Fn::kPostOp && a.postOp) acc = pack_postop(fn, acc);
    for (int d = 0; d < a.nDsts; d++) st16_dst<POLS>(a, d, off, acc);
  }
  // Element tail (< 16 bytes).
  const int64_t eDone = nPacks * 16 / (int64_t)sizeof(T);
  if (eDone < nElts) rc_elems<Fn, POLS>(fn, a, eDone, nElts, gtid, gthreads);
}

// Full reduce-copy of nElts elements by `nWorkers` cooperating workgroups of
// `nthreads` threads (this workgroup = `worker`).  Pointers in `a` are the
// element-0 addresses.  Wave-uniform control flow throughout (every branch
// below depends on pointers and counts only).
//
// DSTR (destination realignment): destinations at different misalignments
// are realigned in registers (true), or — for callers that never pass them
// and need the registers (the direct kernels stage a misaligned output
// through their aligned inbox) — sent to the element path (false).
#ifndef VCCL_SHIFT_ROWS
#define VCCL_SHIFT_ROWS 2
#endif
// Rows of 64 packs per wave span on the grid kernels' misaligned path (2:
// 4 measured slower, see above).
constexpr int kShiftRows = VCCL_SHIFT_ROWS;
template <class Fn, int NS, int ND, int UNROLL, int POLS, int ORDER = 0, bool PIPE = false,
          bool DSTR = true, class Hook = NoHook>
__device__ __forceinline__ void reduce_copy(const Fn& fn, const RCArgs& a, int64_t nElts,
                                            int64_t worker, int64_t nWorkers, int tid,
                                            int nthreads, Hook&& hook = Hook{}) {
  using T = typename Fn::EltType;
  constexpr int esz = (int)sizeof(T);
  const int64_t gtid = worker * nthreads + tid, gthreads = nWorkers * nthreads;
  if (nElts <= 0) return;
  if (rc_all_aligned16(a)) {
    reduce_copy_aligned<Fn, NS, ND, UNROLL, POLS, ORDER, PIPE>(fn, a, nElts, worker, nWorkers, tid,
                                                               nthreads, hook);
    return;
  }
  // Misaligned (see above): the body is aligned on destination 0; sources
  // and the other destinations at other offsets are realigned in registers.
  const int m = (int)((uintptr_t)a.dsts[0] & 15);
  bool ok = m % esz == 0;
  for (int d = 1; d < a.nDsts; d++)
    ok = ok && ((uintptr_t)dst_ptr(a, d) & (DSTR ? esz - 1 : 15)) == (DSTR ? 0u : (uintptr_t)m);
  for (int s = 0; s < a.nSrcs; s++) ok = ok && ((uintptr_t)src_ptr(a, s) & (esz - 1)) == 0;
  if (!ok) {
    rc_elems<Fn, POLS>(fn, a, 0, nElts, gtid, gthreads);
    return;
  }
  int64_t he = ((16 - m) & 15) / esz;
  if (he > nElts) he = nElts;
  if (he > 0) rc_elems<Fn, POLS>(fn, a, 0, he, gtid, gthreads);
  if (he == nElts) return;
  RCArgs b = a;
#pragma unroll
  for (int s = 0; s < kMaxSrcs; s++) b.srcs[s] = a.srcs[s] + he * esz;
#pragma unroll
  for (int d = 0; d < kMaxDsts; d++) b.dsts[d] = a.dsts[d] + he * esz;
  if (rc_all_aligned16(b)) {  // one common misalignment: the aligned engine past the head
    reduce_copy_aligned<Fn, NS, ND, UNROLL, POLS, ORDER, PIPE>(fn, b, nElts - he, worker, nWorkers,
                                                               tid, nthreads);
    return;
  }
  const int64_t nPacks = (nElts - he) * esz / 16;
  if (nPacks > 0) {
    // batched loads for the grid kernels; the in-ring copy (PIPE, a 1024-thread
    // workgroup with a 128-VGPR budget) keeps the lean one-pack loop
    if constexpr (NS >= 1 && ND >= 1 && !PIPE)
      rc_hunks_shifted<Fn, NS, ND, (DSTR ? kShiftRows : (UNROLL < 2 ? UNROLL : 2)), POLS, DSTR>(
          fn, b, nPacks, worker, nWorkers, tid, nthreads);
    else
      rc_hunks_shifted_rt<Fn, POLS, DSTR>(fn, b, nPacks, worker, nWorkers, tid, nthreads);
  }
  const int64_t eDone = he + nPacks * 16 / esz;
  if (eDone < nElts) rc_elems<Fn, POLS>(fn, a, eDone, nElts, gtid, gthreads);
}

}  // namespace vccl
