// Host-side declarations for the ring kernels (one specialisation per kernel
// element type, compiled in parallel).
#pragma once
#include <hip/hip_runtime.h>

#include "coll_types.hpp"
#include "ring_types.hpp"

namespace vccl {

enum : int { kCollAllReduce = 0, kCollReduceScatter = 1, kCollAllGather = 2 };
constexpr int kRingUnroll = 2;
constexpr int kRingMaxThreads = 512;  // k_ring launch bound (ring_kernels.hip)

template <int K>
hipError_t ring_launch(int coll, int devOp, const RingWork& w, int nthreads, hipStream_t stream);

// One-hop LL collectives (ll.hpp): 256-thread workgroups, `grid` of them.
// All-gather only in the K_U8 unit (byte copies).
template <int K>
hipError_t ll_launch(int coll, int devOp, const LLWork& w, int grid, hipStream_t stream);

// Direct collectives over the full mesh (direct.hpp): two-shot all-reduce,
// one-hop reduce-scatter / all-gather; w.nBlocks workgroups of
// kDirectThreads threads.  All-gather only in the K_U8 unit.
template <int K>
hipError_t direct_launch(int coll, int devOp, const DirectWork& w, hipStream_t stream);

}  // namespace vccl
