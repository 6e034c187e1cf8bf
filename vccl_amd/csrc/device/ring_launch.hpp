// Host-side declarations for the ring kernels (one specialisation per kernel
// element type, compiled in parallel).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "coll_types.hpp"
#include "dispatch.hpp"
#include "ring_types.hpp"

namespace vccl {

enum : int { kCollAllReduce = 0, kCollReduceScatter = 1, kCollAllGather = 2, kCollBroadcast = 3, kCollReduce = 4 };
// 16-byte packs per thread per operand in flight in a ring step: 4 (2 for
// the fp8 types, whose per-element prod / min / max / PreMulSum kernels
// spill at 4).  Twice round 1's 2 keeps twice the write-through stores in
// flight per channel: the 2-rank rehearsal's all-gather 1 GiB 2614 ->
// 1714 us, all-reduce -2 %, reduce-scatter -1 % (profiles/r02w).
#ifndef VCCL_RING_UNROLL
#define VCCL_RING_UNROLL 4
#endif
constexpr int kRingUnroll = VCCL_RING_UNROLL;
constexpr int kRingMaxThreads = 512;  // k_ring launch bound (ring_kernels.hip)

// Every launcher takes `stop`: an event the kernel's own completion signal
// records (hipExtLaunchKernel's stopEvent) — the comm's ordering event,
// recorded without a separate marker packet; nullptr = none.
//
// w.w.nChannels workgroups (the largest part's channelHi + 1); the SIMPLE
// ring, or the same schedules over LL128 FIFOs (separate objects).
template <int K>
hipError_t ring_launch(int coll, int devOp, const RingBatch& w, int nthreads, hipStream_t stream,
                       hipEvent_t stop);
template <int K>
hipError_t ring_launch_ll128(int coll, int devOp, const RingBatch& w, int nthreads, hipStream_t stream,
                             hipEvent_t stop);
// The SIMPLE ring with the per-wave slot hand-off (ring.hpp prim_ws): only
// the bandwidth-regime kernels — sum over f32 / f16 / bf16 (all-reduce,
// reduce-scatter, reduce) and the byte-copy all-gather / broadcast — see
// ring_wave_kernel(); every other call takes ring_launch.
template <int K>
hipError_t ring_launch_wave(int coll, int devOp, const RingBatch& w, int nthreads, hipStream_t stream,
                            hipEvent_t stop);
enum : int { kRingVariantSimple = 0, kRingVariantLL128 = 1, kRingVariantWave = 2 };
template <int K>
inline hipError_t ring_launch_any(int variant, int coll, int devOp, const RingBatch& w, int nthreads,
                                  hipStream_t stream, hipEvent_t stop) {
  if (variant == kRingVariantLL128) return ring_launch_ll128<K>(coll, devOp, w, nthreads, stream, stop);
  if constexpr (K == K_U8 || K == K_F32 || K == K_F16 || K == K_BF16)
    if (variant == kRingVariantWave) return ring_launch_wave<K>(coll, devOp, w, nthreads, stream, stop);
  return ring_launch<K>(coll, devOp, w, nthreads, stream, stop);
}

// One-hop LL collectives (ll.hpp): 256-thread workgroups, `grid` of them.
// All-gather only in the K_U8 unit (byte copies).
template <int K>
hipError_t ll_launch(int coll, int devOp, const LLWork& w, int grid, hipStream_t stream, hipEvent_t stop);

// Direct collectives over the full mesh (direct.hpp): two-shot all-reduce,
// one-hop reduce-scatter / all-gather, 1 .. kDirectMaxWorks calls per launch;
// b.w.nBlocks workgroups (the largest part's) of kDirectThreads threads.
// All-gather only in the K_U8 unit.
template <int K>
hipError_t direct_launch(int coll, int devOp, const DirectBatch& b, hipStream_t stream, hipEvent_t stop);

// hipLaunchKernelGGL, or with `stop` bound to the kernel's completion.
template <class F, class... A>
inline hipError_t launch_k(F kernel, dim3 grid, dim3 block, hipStream_t stream, hipEvent_t stop, A... args) {
  if (stop) hipExtLaunchKernelGGL(kernel, grid, block, 0, stream, nullptr, stop, 0, args...);
  else hipLaunchKernelGGL(kernel, grid, block, 0, stream, args...);
  return hipGetLastError();
}

}  // namespace vccl
