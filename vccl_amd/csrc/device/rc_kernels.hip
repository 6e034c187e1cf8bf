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

template <class Fn, int NS, int ND, int UNROLL, int LD, int ST, int ORDER>
__global__ __launch_bounds__(1024) void k_reduce_copy(RCArgs a, int64_t nElts, uint64_t redArg) {
  Fn fn(load_op_arg(a.argPtr, a.argBytes, redArg));
  reduce_copy<Fn, NS, ND, UNROLL, uniform_pol(LD, ST), ORDER>(fn, a, nElts, blockIdx.x, gridDim.x,
                                                           threadIdx.x, blockDim.x);
}

// Launch one instantiation.
template <class Fn, int NS, int ND, int U, int L, int S, int O>
static hipError_t launch_one(const RCArgs& a, int64_t nElts, uint64_t redArg, const LaunchGeom& lg,
                             hipStream_t s) {
  hipLaunchKernelGGL((k_reduce_copy<Fn, NS, ND, U, L, S, O>), dim3(lg.grid), dim3(lg.block), 0, s,
                     a, nElts, redArg);
  return hipGetLastError();
}

// Sweep dispatch (benchmark shape only): unroll {1,2,4,8} x load policy
// {plain, nt, sys, sc1nt} x store policy {plain, nt, sys, sc1nt} x order {0,1}.
template <class Fn, int NS, int ND, int U>
static hipError_t sweep_ls(const RCArgs& a, int64_t n, uint64_t r, const LaunchGeom& lg,
                           hipStream_t s) {
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
  if constexpr (!kSweep) {
    return launch_one<Fn, NS, ND, kRcDefUnroll, kRcDefLd, kRcDefSt, kRcDefOrder>(a, nElts, redArg,
                                                                                 lg, s);
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
    else err = launch_nsnd<Fn, 0, 0>(a, nElts, redArg, lg, stream);
  });
  return err;
}

}  // namespace vccl
