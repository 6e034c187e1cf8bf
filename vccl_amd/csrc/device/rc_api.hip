// C-ABI layer of the reduce-copy engine (include/vccl_device.h).  Argument
// checks mirror ArgsCheck (misc/argcheck.cc:45-86) for what applies here.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../../include/vccl_device.h"
#include "launch.hpp"

using namespace vccl;

static int elt_size_of_kt(int k) {
  switch (k) {
    case K_U8: case K_F8E4M3: case K_F8E5M2: return 1;
    case K_F16: case K_BF16: return 2;
    case K_U32: case K_F32: return 4;
    default: return 8;
  }
}

namespace vccl {
hipError_t reduce_copy_launch(int devOp, int datatype, uint64_t redArg, RCArgs a, int64_t nElts,
                              const vcclLaunchConfigLite* cfg, hipStream_t stream) {
  const int k = kernel_type_of(devOp, datatype);
  if (k < 0) return hipErrorInvalidValue;
  LaunchGeom lg;
  lg.block = (cfg && cfg->blockSize) ? cfg->blockSize : kRcDefBlock;
  lg.unroll = (cfg && cfg->unroll) ? cfg->unroll : kRcDefUnroll;
  if (lg.block != 64 && lg.block != 128 && lg.block != 256 && lg.block != 512 && lg.block != 1024)
    return hipErrorInvalidValue;
  if (lg.unroll != 1 && lg.unroll != 2 && lg.unroll != 4 && lg.unroll != 8) return hipErrorInvalidValue;
  lg.ntLoads = cfg ? cfg->ntLoads : kRcDefLd;
  lg.ntStores = cfg ? cfg->ntStores : (a.nDsts >= 2 ? kRcDefSt2 : kRcDefSt);
  lg.order = cfg ? cfg->order : kRcDefOrder;
  // ntStores 16..31: per-destination policies (two-destination sweep only)
  if (lg.ntLoads < 0 || lg.ntLoads > 3 || lg.ntStores < 0 || lg.ntStores > 31 ||
      (lg.ntStores > 3 && lg.ntStores < 16))
    return hipErrorInvalidValue;
  const int64_t bytes = nElts * elt_size_of_kt(k);
  const int64_t hunk = (int64_t)lg.block * lg.unroll * 16;
  const int64_t want = (bytes + hunk - 1) / hunk;
  lg.grid = (cfg && cfg->gridBlocks)
                ? cfg->gridBlocks
                : (int)std::min<int64_t>(want, (int64_t)kRcMaxGrid);
  if (lg.grid < 1) lg.grid = 1;
  a.argBytes = elt_size_of_kt(k);
  switch (k) {
    case K_U8: return rc_launch<K_U8>(devOp, a, nElts, redArg, lg, stream);
    case K_U32: return rc_launch<K_U32>(devOp, a, nElts, redArg, lg, stream);
    case K_U64: return rc_launch<K_U64>(devOp, a, nElts, redArg, lg, stream);
    case K_F16: return rc_launch<K_F16>(devOp, a, nElts, redArg, lg, stream);
    case K_F32: return rc_launch<K_F32>(devOp, a, nElts, redArg, lg, stream);
    case K_F64: return rc_launch<K_F64>(devOp, a, nElts, redArg, lg, stream);
    case K_BF16: return rc_launch<K_BF16>(devOp, a, nElts, redArg, lg, stream);
    case K_F8E4M3: return rc_launch<K_F8E4M3>(devOp, a, nElts, redArg, lg, stream);
    case K_F8E5M2: return rc_launch<K_F8E5M2>(devOp, a, nElts, redArg, lg, stream);
  }
  return hipErrorInvalidValue;
}
}  // namespace vccl

extern "C" ncclResult_t vcclReduceCopyEx(vcclDevRedOp_t devOp, ncclDataType_t datatype,
                                         uint64_t redArg, int preOpSrcs, int postOp, int nSrcs,
                                         const void* const* srcs, int nDsts, void* const* dsts,
                                         size_t nElts, hipStream_t stream,
                                         const vcclLaunchConfig* cfg) {
  if (nSrcs < 1 || nSrcs > kMaxSrcs || nDsts < 1 || nDsts > kMaxDsts) return ncclInvalidArgument;
  if (kernel_type_of((int)devOp, (int)datatype) < 0) return ncclInvalidArgument;
  if (nElts == 0) return ncclSuccess;
  if (srcs == nullptr || dsts == nullptr) return ncclInvalidArgument;
  RCArgs a = {};
  for (int s = 0; s < nSrcs; s++) {
    if (!srcs[s]) return ncclInvalidArgument;
    a.srcs[s] = (const char*)srcs[s];
  }
  for (int d = 0; d < nDsts; d++) {
    if (!dsts[d]) return ncclInvalidArgument;
    a.dsts[d] = (char*)dsts[d];
  }
  a.nSrcs = nSrcs;
  a.nDsts = nDsts;
  a.preOpSrcs = preOpSrcs < 0 ? 0 : preOpSrcs;
  a.postOp = postOp ? 1 : 0;
  a.argPtr = nullptr;
  vcclLaunchConfigLite lite;
  if (cfg) lite = {cfg->blockSize, cfg->unroll, cfg->gridBlocks, cfg->ntLoads, cfg->ntStores,
                   cfg->order};
  hipError_t err = reduce_copy_launch((int)devOp, (int)datatype, redArg, a, (int64_t)nElts,
                                      cfg ? &lite : nullptr, stream);
  if (err == hipErrorInvalidValue) return ncclInvalidArgument;
  return err == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

extern "C" ncclResult_t vcclReduceCopy(vcclDevRedOp_t devOp, ncclDataType_t datatype,
                                       uint64_t redArg, int preOpSrcs, int postOp, int nSrcs,
                                       const void* const* srcs, int nDsts, void* const* dsts,
                                       size_t nElts, hipStream_t stream) {
  return vcclReduceCopyEx(devOp, datatype, redArg, preOpSrcs, postOp, nSrcs, srcs, nDsts, dsts,
                          nElts, stream, nullptr);
}

extern "C" int vcclKernelTypeOf(int devOp, ncclDataType_t datatype) {
  return kernel_type_of(devOp, (int)datatype);
}
