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
#pragma once
#include "ops.hpp"

namespace vccl {

constexpr int kMaxSrcs = 8;
constexpr int kMaxDsts = 8;

// Memory flavours for the pack path.
enum : int { kLdPlain = 0, kLdNT = 1 };
enum : int { kStPlain = 0, kStNT = 1 };

template <int LD>
__device__ __forceinline__ u32x4 ld16(const char* p) {
  if constexpr (LD == kLdNT) return __builtin_nontemporal_load((const u32x4*)p);
  else return *(const u32x4*)p;
}
template <int ST>
__device__ __forceinline__ void st16(char* p, u32x4 v) {
  if constexpr (ST == kStNT) __builtin_nontemporal_store(v, (u32x4*)p);
  else *(u32x4*)p = v;
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

// One pass over `nPacks` 16-byte packs starting at byte offset `base`.
// NS/ND: compile-time source/destination counts (0 = runtime, <= kMax*).
template <class Fn, int NS, int ND, int UNROLL, int LD, int ST>
__device__ __forceinline__ void rc_hunks(const Fn& fn, const RCArgs& a, int64_t base,
                                         int64_t nPacks, int64_t worker, int64_t nWorkers,
                                         int tid, int nthreads) {
  const int nS = NS ? NS : a.nSrcs;
  const int nD = ND ? ND : a.nDsts;
  const int64_t hunkPacks = (int64_t)nthreads * UNROLL;
  const int64_t nHunks = nPacks / hunkPacks;
  for (int64_t h = worker; h < nHunks; h += nWorkers) {
    const int64_t off = base + (h * hunkPacks + tid) * 16;
    u32x4 acc[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) acc[u] = ld16<LD>(a.srcs[0] + off + (int64_t)u * nthreads * 16);
    if (Fn::kPreOp && a.preOpSrcs > 0) {
#pragma unroll
      for (int u = 0; u < UNROLL; u++) acc[u] = pack_preop(fn, acc[u]);
    }
    auto fold_src = [&](int s) __attribute__((always_inline)) {
      u32x4 tmp[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; u++) tmp[u] = ld16<LD>(a.srcs[s] + off + (int64_t)u * nthreads * 16);
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
      for (int u = 0; u < UNROLL; u++) st16<ST>(a.dsts[d] + off + (int64_t)u * nthreads * 16, acc[u]);
    };
    if constexpr (ND > 0) {
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

// Element-granular path (misaligned pointers and the < 16 B tail),
// reduceCopyPacks<BytePerPack=sizeof(T)> equivalent.
template <class Fn>
__device__ __forceinline__ void rc_elems(const Fn& fn, const RCArgs& a, int64_t eBegin,
                                         int64_t eEnd, int64_t gtid, int64_t gthreads) {
  using T = typename Fn::EltType;
  for (int64_t i = eBegin + gtid; i < eEnd; i += gthreads) {
    T acc = ((const T*)a.srcs[0])[i];
    if (Fn::kPreOp && a.preOpSrcs > 0) acc = fn.preOp(acc);
    for (int s = 1; s < a.nSrcs; s++) {
      T v = ((const T*)a.srcs[s])[i];
      if (Fn::kPreOp && s < a.preOpSrcs) v = fn.preOp(v);
      acc = fn.reduce(acc, v);
    }
    if (Fn::kPostOp && a.postOp) acc = fn.postOp(acc);
    for (int d = 0; d < a.nDsts; d++) ((T*)a.dsts[d])[i] = acc;
  }
}

__device__ __forceinline__ bool rc_all_aligned16(const RCArgs& a) {
  uintptr_t bits = 0;
  for (int s = 0; s < a.nSrcs; s++) bits |= (uintptr_t)a.srcs[s];
  for (int d = 0; d < a.nDsts; d++) bits |= (uintptr_t)a.dsts[d];
  return (bits & 15) == 0;
}

// Full reduce-copy of nElts elements by `nWorkers` cooperating workgroups of
// `nthreads` threads (this workgroup = `worker`).  Pointers in `a` are the
// element-0 addresses.  Wave-uniform control flow throughout.
template <class Fn, int NS, int ND, int UNROLL, int LD, int ST>
__device__ __forceinline__ void reduce_copy(const Fn& fn, const RCArgs& a, int64_t nElts,
                                            int64_t worker, int64_t nWorkers, int tid,
                                            int nthreads) {
  using T = typename Fn::EltType;
  const int64_t gtid = worker * nthreads + tid, gthreads = nWorkers * nthreads;
  if (nElts <= 0) return;
  if (!rc_all_aligned16(a)) {
    rc_elems(fn, a, 0, nElts, gtid, gthreads);
    return;
  }
  const int64_t nBytes = nElts * (int64_t)sizeof(T);
  const int64_t nPacks = nBytes / 16;
  const int64_t hunkPacks = (int64_t)nthreads * UNROLL;
  const int64_t fullPacks = (nPacks / hunkPacks) * hunkPacks;
  rc_hunks<Fn, NS, ND, UNROLL, LD, ST>(fn, a, 0, fullPacks, worker, nWorkers, tid, nthreads);
  // Remaining packs (< one hunk): one pack per thread, grid-strided.
  for (int64_t p = fullPacks + gtid; p < nPacks; p += gthreads) {
    const int64_t off = p * 16;
    u32x4 acc = ld16<LD>(a.srcs[0] + off);
    if (Fn::kPreOp && a.preOpSrcs > 0) acc = pack_preop(fn, acc);
    for (int s = 1; s < a.nSrcs; s++) {
      u32x4 v = ld16<LD>(a.srcs[s] + off);
      if (Fn::kPreOp && s < a.preOpSrcs) v = pack_preop(fn, v);
      acc = pack_reduce(fn, acc, v);
    }
    if (Fn::kPostOp && a.postOp) acc = pack_postop(fn, acc);
    for (int d = 0; d < a.nDsts; d++) st16<ST>(a.dsts[d] + off, acc);
  }
  // Element tail (< 16 bytes).
  const int64_t eDone = nPacks * 16 / (int64_t)sizeof(T);
  if (eDone < nElts) rc_elems(fn, a, eDone, nElts, gtid, gthreads);
}

}  // namespace vccl
