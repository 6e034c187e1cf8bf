// Host-side launcher declarations shared by the per-type kernel TUs and the
// C-ABI layer (one explicit specialisation per kernel element type).
#pragma once
#include <hip/hip_runtime.h>

#include "dispatch.hpp"
#include "reduce_copy.hpp"

namespace vccl {

// Library defaults for the grid-wide reduce-copy, from the interleaved sweeps
// of tools/sweep_rc.py on MI355X (profiles/r01_sweep_rc*.log):
// 256 threads, 2 x 16 B per thread per source, one hunk per workgroup (no
// grid-stride below kRcMaxGrid), nontemporal loads, sc0 sc1 write-through
// stores (the destination line is not kept in L2: +6.6 % over plain stores).
constexpr int kRcDefBlock = 256;
constexpr int kRcDefUnroll = 2;
constexpr int kRcMaxGrid = 65536;
constexpr int kRcDefLd = kLdNT;
constexpr int kRcDefSt = kSys;
constexpr int kRcDefOrder = 0;
// With two or more destinations their stores alternate write-through (sc0
// sc1) and nt: 2 -> 2 f32 runs at 7.13 TB/s so, 6.0 with every destination
// write-through (tools/sweep_rc.py twodst, profiles/r03a).  ND = 0: runtime
// destination count.
constexpr int rc_def_pols(int nd) {
  return nd == 1 ? uniform_pol(kRcDefLd, kRcDefSt)
                 : mkpol(kRcDefLd, kRcDefLd, kRcDefLd, kRcDefLd, kSys, kNT, kSys, kNT);
}
constexpr int kRcDefSt2 = 16 | kSys | kNT << 2;  // the same, in vcclLaunchConfig's encoding

// Internal entry used by both the C ABI and the one-rank path.  `a` holds the
// pointers; geometry from cfg (nullptr = defaults).
struct vcclLaunchConfigLite {
  int blockSize, unroll, gridBlocks, ntLoads, ntStores, order;
};
hipError_t reduce_copy_launch(int devOp, int datatype, uint64_t redArg, RCArgs a, int64_t nElts,
                              const vcclLaunchConfigLite* cfg, hipStream_t stream);

template <int K>
hipError_t rc_launch(int devOp, const RCArgs& a, int64_t nElts, uint64_t redArg,
                     const LaunchGeom& lg, hipStream_t stream);

}  // namespace vccl
