// Grid-wide reduce-copy kernels for ONE kernel element type (VCCL_KT), so the
// build compiles the 7 element types in parallel.  Semantics: reduceCopy()
// (common_kernel.h:208-285) and oneRankReduce (onerank.cu:13-44).
#include <hip/hip_runtime.h>

#include "dispatch.hpp"
#include "launch.hpp"
#include "reduce_copy.hpp"

#ifndef VCCL_KT
#error "compile with -DVCCL_KT=<kernel element type>"
#endif

namespace vccl {

// POLS: per-operand memory policies (mkpol); ORDER 4 = the software-pipelined
// hunk loop (next hunk's loads issued before this hunk's stores).
template <class Fn, int NS, int ND, int UNROLL, int POLS, int ORDER>
__global__ __launch_bounds__(1024) void k_reduce_copy(RCArgs a, int64_t nElts, uint64_t redArg) {
  Fn fn(load_op_arg(a.argPtr, a.argBytes, redArg));
  reduce_copy<Fn, NS, ND, UNROLL, POLS, ORDER == 4 ? 0 : ORDER, ORDER == 4>(
      fn, a, nElts, blockIdx.x, gridDim.x, threadIdx.x, blockDim.x);
}

// LDS-staged variant (benchmark sweep only, `order` 2): the north-star's
// "LDS double-buffered staging" measured against the register path.  Each
// wave moves its sources HBM -> LDS with global_load_lds_dwordx4 (LDS-DMA,
// no VGPR destination) two tiles deep: while tile t+1's DMA is in flight the
// wave reads tile t back (ds_read_b128, each lane its own 16 bytes, so no
// workgroup barrier is needed), reduces and stores.  A lane's LDS slot is
// wave base + lane x 16 (the DMA's fixed destination pattern).  Full tiles
// only (the launcher falls back to the register path otherwise).
constexpr int kLdsU = 2;  // packs per lane per source per tile
template <class Fn, int NS, int ST>
__global__ __launch_bounds__(256) void k_reduce_copy_lds(RCArgs a, int64_t nTiles, uint64_t redArg) {
  using T = typename Fn::EltType;
  (void)sizeof(T);
  __shared__ __attribute__((aligned(16))) char lds[2][NS][kLdsU][256 * 16];
  Fn fn(load_op_arg(a.argPtr, a.argBytes, redArg));
  const int tid = threadIdx.x, wbase = (tid >> 6) * 64 * 16;
  constexpr int64_t kTilePacks = 256 * kLdsU;
  auto issue = [&](int64_t tile, int buf) {
#pragma unroll
    for (int s = 0; s < NS; s++)
#pragma unroll
      for (int u = 0; u < kLdsU; u++) {
        const int64_t pack = tile * kTilePacks + u * 256 + tid;
        __builtin_amdgcn_global_load_lds(
            (const void*)(a.srcs[s] + pack * 16),
            (__attribute__((address_space(3))) void*)(&lds[buf][s][u][wbase]), 16, 0, 2 /*nt*/);
      }
  };
  int64_t t = blockIdx.x;
  if (t >= nTiles) return;
  issue(t, 0);
  for (int buf = 0; t < nTiles; t += gridDim.x, buf ^= 1) {
    const bool more = t + gridDim.x < nTiles;
    if (more) issue(t + gridDim.x, buf ^ 1);
    // tile t's DMA (and everything issued before it) complete; the next
    // tile's NS x kLdsU DMAs stay in flight
    if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS * kLdsU) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < kLdsU; u++) {
      u32x4 acc = *(const u32x4*)(&lds[buf][0][u][wbase + (tid & 63) * 16]);
      if constexpr (Fn::kPreOp) {
        if (a.preOpSrcs > 0) acc = pack_preop(fn, acc);
      }
#pragma unroll
      for (int s = 1; s < NS; s++) {
        u32x4 v = *(const u32x4*)(&lds[buf][s][u][wbase + (tid & 63) * 16]);
        acc = pack_reduce(fn, acc, v);
      }
      if constexpr (Fn::kPostOp) {
        if (a.postOp) acc = pack_postop(fn, acc);
      }
      const int64_t pack = t * kTilePacks + u * 256 + tid;
      st16<ST>(a.dsts[0], pack * 16, acc);
    }
    // this wave's ds_reads of `buf` must finish before its DMA refills it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// Launch one instantiation (uniform load policy L, store policy S).
template <class Fn, int NS, int ND, int U, int L, int S, int O>
static hipError_t launch_one(const RCArgs& a, int64_t nElts, uint64_t redArg, const LaunchGeom& lg,
                             hipStream_t s) {
  hipLaunchKernelGGL((k_reduce_copy<Fn, NS, ND, U, uniform_pol(L, S), O>), dim3(lg.grid),
                     dim3(lg.block), 0, s, a, nElts, redArg);
  return hipGetLastError();
}

// Two-destination sweep (the ring's final-reduce / recv-copy-send shape,
// 2 sources -> 2 destinations, measurement only): nt loads, unroll {2, 4},
// a store policy PER destination (ntStores = 16 | d0 | d1 << 2; below 16 the
// uniform encoding), store order {0 destination-major, 1 XCD-contiguous
// hunks, 3 interleaved, 4 pipelined}.
template <class Fn, int U, int D0, int D1>
static hipError_t launch_2dst_pol(const RCArgs& a, int64_t n, uint64_t r, const LaunchGeom& lg,
                                  hipStream_t s) {
  constexpr int P = mkpol(kNT, kNT, kNT, kNT, D0, D1, D1, D1);
  auto go = [&]<int O>() {
    hipLaunchKernelGGL((k_reduce_copy<Fn, 2, 2, U, P, O>), dim3(lg.grid), dim3(lg.block), 0, s, a,
                       n, r);
    return hipGetLastError();
  };
  if (lg.order == 1) return go.template operator()<1>();
  if (lg.order == 3) return go.template operator()<3>();
  if (lg.order == 4) return go.template operator()<4>();
  return go.template operator()<0>();
}
template <class Fn, int U>
static hipError_t sweep_2dst(const RCArgs& a, int64_t n, uint64_t r, const LaunchGeom& lg,
                             hipStream_t s) {
  const int d0 = lg.ntStores >= 16 ? (lg.ntStores & 3) : lg.ntStores;
  const int d1 = lg.ntStores >= 16 ? ((lg.ntStores >> 2) & 3) : lg.ntStores;
  auto by_d1 = [&]<int D0>() -> hipError_t {
    switch (d1) {
      case kNT: return launch_2dst_pol<Fn, U, D0, kNT>(a, n, r, lg, s);
      case kSys: return launch_2dst_pol<Fn, U, D0, kSys>(a, n, r, lg, s);
      case kSc1NT: return launch_2dst_pol<Fn, U, D0, kSc1NT>(a, n, r, lg, s);
      default: return launch_2dst_pol<Fn, U, D0, kPlain>(a, n, r, lg, s);
    }
  };
  switch (d0) {
    case kNT: return by_d1.template operator()<kNT>();
    case kSys: return by_d1.template operator()<kSys>();
    case kSc1NT: return by_d1.template operator()<kSc1NT>();
    default: return by_d1.template operator()<kPlain>();
  }
}

// Sweep dispatch (benchmark shape only): unroll {1,2,4,8} x load policy
// {plain, nt, sys, sc1nt} x store policy {plain, nt, sys, sc1nt} x order {0,1}.
template <class Fn, int NS, int ND, int U>
static hipError_t sweep_ls(const RCArgs& a, int64_t n, uint64_t r, const LaunchGeom& lg,
                           hipStream_t s) {
  if constexpr (NS >= 1 && ND == 1) {
    using T = typename Fn::EltType;
    const int64_t bytes = n * (int64_t)sizeof(T);
    const int64_t tileBytes = 256 * kLdsU * 16;
    bool aligned = true;
    for (int i = 0; i < NS; i++) aligned &= ((uintptr_t)a.srcs[i] & 15) == 0;
    aligned &= ((uintptr_t)a.dsts[0] & 15) == 0;
    if (lg.order == 2 && aligned && bytes % tileBytes == 0) {
      const int64_t nTiles = bytes / tileBytes;
      const int grid = (int)std::min<int64_t>(nTiles, lg.grid);  // persistent: pass gridBlocks
      if (lg.ntStores == 2)
        hipLaunchKernelGGL((k_reduce_copy_lds<Fn, NS, kSys>), dim3(grid), dim3(256), 0, s, a, nTiles, r);
      else
        hipLaunchKernelGGL((k_reduce_copy_lds<Fn, NS, kNT>), dim3(grid), dim3(256), 0, s, a, nTiles, r);
      return hipGetLastError();
    }
  }
  auto by_order = [&]<int L, int S>() -> hipError_t {
    if (lg.order == 1) return launch_one<Fn, NS, ND, U, L, S, 1>(a, n, r, lg, s);
    return launch_one<Fn, NS, ND, U, L, S, 0>(a, n, r, lg, s);
  };
  auto by_store = [&]<int L>() -> hipError_t {
    switch (lg.ntStores) {
      case 1: return by_order.template operator()<L, kNT>();
      case 2: return by_order.template operator()<L, kSys>();
      case 3: return by_order.template operator()<L, kSc1NT>();
      default: return by_order.template operator()<L, kPlain>();
    }
  };
  switch (lg.ntLoads) {
    case 1: return by_store.template operator()<kNT>();
    case 2: return by_store.template operator()<kSys>();
    case 3: return by_store.template operator()<kSc1NT>();
    default: return by_store.template operator()<kPlain>();
  }
}

template <class Fn, int NS, int ND>
static hipError_t launch_nsnd(const RCArgs& a, int64_t nElts, uint64_t redArg,
                              const LaunchGeom& lg, hipStream_t s) {
  // Only the benchmark shape (2-src f32 sum) carries the full sweep set; every
  // other functor gets the tuned default (keeps the code object small).
  constexpr bool kSweep = std::is_same<Fn, FnSum<float>>::value && NS == 2 && ND == 1;
  constexpr bool kSweep2 = std::is_same<Fn, FnSum<float>>::value && NS == 2 && ND == 2;
  if constexpr (kSweep2) {
    if (lg.unroll == 4) return sweep_2dst<Fn, 4>(a, nElts, redArg, lg, s);
    return sweep_2dst<Fn, 2>(a, nElts, redArg, lg, s);
  } else if constexpr (std::is_same<Fn, FnSum<float>>::value && NS == 1 && ND == 1) {
    // the copy shape (1 -> 1): the read/write-mix reference for the above
    if (lg.unroll == 4) return sweep_ls<Fn, NS, ND, 4>(a, nElts, redArg, lg, s);
    return sweep_ls<Fn, NS, ND, 2>(a, nElts, redArg, lg, s);
  } else if constexpr (!kSweep) {
    hipLaunchKernelGGL((k_reduce_copy<Fn, NS, ND, kRcDefUnroll, rc_def_pols(ND), kRcDefOrder>),
                       dim3(lg.grid), dim3(lg.block), 0, s, a, nElts, redArg);
    return hipGetLastError();
  } else {
    if (lg.unroll == 8) return sweep_ls<Fn, NS, ND, 8>(a, nElts, redArg, lg, s);
    if (lg.unroll == 2) return sweep_ls<Fn, NS, ND, 2>(a, nElts, redArg, lg, s);
    if (lg.unroll == 1) return sweep_ls<Fn, NS, ND, 1>(a, nElts, redArg, lg, s);
    return sweep_ls<Fn, NS, ND, 4>(a, nElts, redArg, lg, s);
  }
}

template <>
hipError_t rc_launch<VCCL_KT>(int devOp, const RCArgs& a, int64_t nElts, uint64_t redArg,
                              const LaunchGeom& lg, hipStream_t stream) {
  using T = typename KTypeOf<VCCL_KT>::T;
  hipError_t err = hipErrorInvalidValue;
  dispatch_op<T>(devOp, [&]<class Fn>() {
    if (a.nSrcs == 2 && a.nDsts == 1) err = launch_nsnd<Fn, 2, 1>(a, nElts, redArg, lg, stream);
    else if (a.nSrcs == 1 && a.nDsts == 1) err = launch_nsnd<Fn, 1, 1>(a, nElts, redArg, lg, stream);
    // reduce + copy to two places (the ring all-reduce's final step shape)
    else if (a.nSrcs == 2 && a.nDsts == 2) err = launch_nsnd<Fn, 2, 2>(a, nElts, redArg, lg, stream);
    else err = launch_nsnd<Fn, 0, 0>(a, nElts, redArg, lg, stream);
  });
  return err;
}

}  // namespace vccl
