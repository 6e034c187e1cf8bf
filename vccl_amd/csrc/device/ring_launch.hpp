// Host-side declarations for the ring kernels (one specialisation per kernel
// element type, compiled in parallel).
#pragma once
#include <hip/hip_runtime.h>

#include "direct.hpp"
#include "ll.hpp"
#include "ring_types.hpp"

namespace vccl {

enum : int { kCollAllReduce = 0, kCollReduceScatter = 1, kCollAllGather = 2 };
constexpr int kRingUnroll = 2;

template <int K>
hipError_t ring_launch(int coll, int devOp, const RingWork& w, int nthreads, hipStream_t stream);

// One-shot LL all-reduce (ll.hpp): 256-thread workgroups, `grid` of them.
template <int K>
hipError_t ll_launch(int devOp, const LLWork& w, int grid, hipStream_t stream);

// Two-shot direct all-reduce (direct.hpp): w.nBlocks workgroups of
// kDirectThreads threads.
template <int K>
hipError_t direct_launch(int devOp, const DirectWork& w, hipStream_t stream);

}  // namespace vccl
