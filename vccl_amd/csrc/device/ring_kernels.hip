// Collective kernels for ONE kernel element type (VCCL_KT) and ONE family
// (VCCL_PART: 0 ring, 1 LL, 2 direct, 3 LL128 ring, 4 ring with the per-wave
// hand-off — separate objects, built in parallel):
// per reduction functor the ring all-reduce / reduce-scatter / reduce (one workgroup
// per channel, enqueue.cc:1576-1666), the one-shot LL and the direct
// (two-shot all-reduce, one-hop reduce-scatter) kernels; in the K_U8 unit
// also the type-agnostic all-gathers (ring, LL, direct).
#include <hip/hip_runtime.h>

#include "dispatch.hpp"
#include "ring_launch.hpp"
#if VCCL_PART == 0 || VCCL_PART == 3 || VCCL_PART == 4
#include "ring.hpp"
#elif VCCL_PART == 1
#include "ll.hpp"
#else
#include "direct.hpp"
#endif

#ifndef VCCL_KT
#error "compile with -DVCCL_KT=<kernel element type>"
#endif
#ifndef VCCL_PART
#error "compile with -DVCCL_PART=<0 ring | 1 LL | 2 direct | 3 LL128 ring | 4 per-wave ring>"
#endif

namespace vccl {

#if VCCL_PART == 0 || VCCL_PART == 3 || VCCL_PART == 4
// PART 0: the SIMPLE ring; PART 3: the same schedules over LL128 FIFOs;
// PART 4: the SIMPLE ring with the per-wave hand-off, for the bandwidth
// kernels only (sum over f32 / f16 / bf16, the byte-copy all-gather and
// broadcast; Makefile WAVE_KTS), chosen per comm (VCCL_RING_WAVE).
constexpr int kPartProto = VCCL_PART == 3 ? kProtoLL128 : VCCL_PART == 4 ? kProtoSimpleWave : kProtoSimple;
#if VCCL_PART == 3
#define VCCL_RING_LAUNCH ring_launch_ll128
#elif VCCL_PART == 4
#define VCCL_RING_LAUNCH ring_launch_wave
#else
#define VCCL_RING_LAUNCH ring_launch
#endif

// 512 threads per channel: the ring primitive (pipelined aligned copy +
// realigning misaligned path, inlined per (recv, send, src, dst) shape) needs
// ~137 VGPRs, above the 128 a 1024-thread workgroup allows (that spilled in
// the hot loop).  Channel count, not threads per channel, sets ring
// bandwidth.
template <class Fn>
constexpr int ring_unroll() { return IsF8<typename Fn::EltType>::value ? 2 : kRingUnroll; }
#ifndef VCCL_AG_UNROLL
#define VCCL_AG_UNROLL kRingUnroll
#endif

// PROTO is a template parameter of every function below, so the SIMPLE and
// LL128 objects never define the same symbol differently.
template <int COLL, class Fn, int UNROLL, int PROTO>
__device__ __forceinline__ void ring_run(RingCtx& r, const Fn& fn, const RingWork& w) {
  if constexpr (COLL == kCollAllReduce) ring_allreduce<Fn, UNROLL, PROTO>(r, fn, w, blockIdx.x);
  else if constexpr (COLL == kCollReduceScatter)
    ring_reducescatter<Fn, UNROLL, PROTO>(r, fn, w, blockIdx.x);
  else if constexpr (COLL == kCollReduce) ring_reduce<Fn, UNROLL, PROTO>(r, fn, w, blockIdx.x);
  else if constexpr (COLL == kCollAllGather) ring_allgather<UNROLL, PROTO>(r, w, blockIdx.x);
  else ring_broadcast<UNROLL, PROTO>(r, w, blockIdx.x);
}

// One launch = 1 .. kRingMaxWorks calls (RingBatch, group aggregation): the
// channel workgroup runs them in order.  The kernel argument is read through
// scalar loads at any part index (no private copy).
template <int COLL, class Fn, int UNROLL, int PROTO>
__global__ __launch_bounds__(kRingMaxThreads) void k_ring(RingBatch b) {
  const RingWork& w = b.w;
  __shared__ WaveSync ws;
  __shared__ int shRing[kMaxRanks];
  if (threadIdx.x == 0) {
    for (int i = 0; i < kSyncDepth; i++) ws.done[i] = 0;
    ws.tail = ws.head = 0;
    ws.abort = 0;
    ws.poller = 0;
  }
  DevChannel* ch = &w.channels[blockIdx.x];
  RingCtx r;
  r.tid = threadIdx.x;
  r.nthreads = blockDim.x;
  r.load(ch, w.comm, w.nRanks, (VCCL_LDS int*)shRing);
  __syncthreads();
  r.slotBytes = w.slotBytes;
  r.ll128Slot = w.ll128SlotBytes;
  r.ws = (VCCL_LDS WaveSync*)&ws;
  r.shAbort = &r.ws->abort;
  r.lane = threadIdx.x & 63;
  r.nWaves = (int)(blockDim.x >> 6);
  r.seq = 0;
  r.pend = false;
  r.trace = w.comm->trace ? (VCCL_GLOBAL RingTraceRec*)((RingTraceRec*)w.comm->trace + (int64_t)blockIdx.x * w.comm->traceCap)
                          : nullptr;
  r.traceN = 0;
  const Fn fn(load_op_arg(w.redArgPtr, w.redArgBytes, w.redArg));
  const uint64_t recv0 = r.recvStep, send0 = r.sendStep;
  ring_run<COLL, Fn, UNROLL, PROTO>(r, fn, w);
  for (int i = 1; i < b.nParts; i++)
    ring_run<COLL, Fn, UNROLL, PROTO>(r, fn, ring_work_with(w, b.more[i - 1]));
  r.finish();  // this wave's last prim: drained, counted, posted by the last wave
  __syncthreads();
  // a channel none of the parts touched (below every part's channelLo) keeps
  // its counters untouched
  if (threadIdx.x == 0 && (r.recvStep != recv0 || r.sendStep != send0)) {
    ch->recvStep = r.recvStep;
    ch->sendStep = r.sendStep;
  }
}

template <>
hipError_t VCCL_RING_LAUNCH<VCCL_KT>(int coll, int devOp, const RingBatch& w, int nthreads,
                                     hipStream_t stream, hipEvent_t stop) {
  using T = typename KTypeOf<VCCL_KT>::T;
  hipError_t err = hipErrorInvalidValue;
  dim3 grid(w.w.nChannels), block(nthreads);
  if (coll == kCollAllGather || coll == kCollBroadcast) {  // byte copies: the K_U8 unit only
    if constexpr (VCCL_KT == K_U8) {
      if (coll == kCollBroadcast)
        return launch_k(k_ring<kCollBroadcast, FnCopy<uint8_t>, VCCL_AG_UNROLL, kPartProto>, grid, block, stream,
                        stop, w);
      return launch_k(k_ring<kCollAllGather, FnCopy<uint8_t>, VCCL_AG_UNROLL, kPartProto>, grid, block, stream,
                      stop, w);
    }
    return hipErrorInvalidValue;
  }
#if VCCL_PART == 4
  if (devOp != OP_SUM) return hipErrorInvalidValue;  // ring_wave_kernel() never asks
#endif
  dispatch_op<T>(devOp, [&]<class Fn>() {
    if constexpr (std::is_same<Fn, FnCopy<T>>::value) {
      err = hipErrorInvalidValue;
#if VCCL_PART == 4
    } else if constexpr (!std::is_same<Fn, FnSum<T>>::value || VCCL_KT == K_U8) {
      err = hipErrorInvalidValue;
#endif
    } else if (coll == kCollAllReduce) {
      err = launch_k(k_ring<kCollAllReduce, Fn, ring_unroll<Fn>(), kPartProto>, grid, block, stream, stop, w);
    } else if (coll == kCollReduceScatter) {
      err = launch_k(k_ring<kCollReduceScatter, Fn, ring_unroll<Fn>(), kPartProto>, grid, block, stream, stop,
                     w);
    } else if (coll == kCollReduce) {
      err = launch_k(k_ring<kCollReduce, Fn, ring_unroll<Fn>(), kPartProto>, grid, block, stream, stop, w);
    }
  });
  return err;
}

#elif VCCL_PART == 1
template <class Fn>
__global__ __launch_bounds__(256) void k_ll_allreduce(LLWork w) {
  ll_allreduce<Fn>(w);
}
template <class Fn>
__global__ __launch_bounds__(256) void k_ll_reducescatter(LLWork w) {
  ll_reducescatter<Fn>(w);
}
template <int K>  // instantiated in the K_U8 unit only (byte copies)
__global__ __launch_bounds__(256) void k_ll_allgather(LLWork w) { ll_allgather(w); }

template <>
hipError_t ll_launch<VCCL_KT>(int coll, int devOp, const LLWork& w, int grid, hipStream_t stream,
                              hipEvent_t stop) {
  using T = typename KTypeOf<VCCL_KT>::T;
  if (coll == kCollAllGather) {
    if constexpr (VCCL_KT == K_U8) {
      return launch_k(k_ll_allgather<K_U8>, dim3(grid), dim3(256), stream, stop, w);
    }
    return hipErrorInvalidValue;
  }
  hipError_t err = hipErrorInvalidValue;
  dispatch_op<T>(devOp, [&]<class Fn>() {
    if constexpr (!std::is_same<Fn, FnCopy<T>>::value) {
      err = coll == kCollAllReduce ? launch_k(k_ll_allreduce<Fn>, dim3(grid), dim3(256), stream, stop, w)
                                   : launch_k(k_ll_reducescatter<Fn>, dim3(grid), dim3(256), stream, stop, w);
    }
  });
  return err;
}

#elif VCCL_PART == 2
template <class Fn>
__global__ __launch_bounds__(kDirectThreads) void k_direct_allreduce(DirectBatch b) {
  direct_batch(b, [](const DirectWork& w, uint32_t& e, int& f) { direct_allreduce_part<Fn>(w, e, f); });
}
template <class Fn>
__global__ __launch_bounds__(kDirectThreads) void k_direct_reducescatter(DirectBatch b) {
  direct_batch(b, [](const DirectWork& w, uint32_t& e, int& f) { direct_reducescatter_part<Fn>(w, e, f); });
}
template <int K>  // instantiated in the K_U8 unit only (byte copies)
__global__ __launch_bounds__(kDirectThreads) void k_direct_allgather(DirectBatch b) {
  direct_batch(b, [](const DirectWork& w, uint32_t& e, int& f) { direct_allgather_part(w, e, f); });
}

template <>
hipError_t direct_launch<VCCL_KT>(int coll, int devOp, const DirectBatch& b, hipStream_t stream,
                                  hipEvent_t stop) {
  using T = typename KTypeOf<VCCL_KT>::T;
  const dim3 grid(b.w.nBlocks), block(kDirectThreads);
  if (coll == kCollAllGather) {
    if constexpr (VCCL_KT == K_U8) {
      return launch_k(k_direct_allgather<K_U8>, grid, block, stream, stop, b);
    }
    return hipErrorInvalidValue;
  }
  hipError_t err = hipErrorInvalidValue;
  dispatch_op<T>(devOp, [&]<class Fn>() {
    if constexpr (!std::is_same<Fn, FnCopy<T>>::value) {
      err = coll == kCollAllReduce ? launch_k(k_direct_allreduce<Fn>, grid, block, stream, stop, b)
                                   : launch_k(k_direct_reducescatter<Fn>, grid, block, stream, stop, b);
    }
  });
  return err;
}

#endif

}  // namespace vccl
