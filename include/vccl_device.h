/*
 * vccl-mi355x low-level C ABI: the reduce-copy engine and the op encoding,
 * callable without a communicator.  These are the entry points a maintainer
 * binds when wiring the MI355X engine under VCCL's own dispatch:
 *
 *   vcclReduceCopy        replaces reduceCopy<...>() as a launchable unit
 *                         (src/device/common_kernel.h:208-285; the one-rank
 *                         kernel onerank.cu:13-44 is its 1-src/1-dst case)
 *   vcclHostToDevRedOp    replaces hostToDevRedOp (src/enqueue.cc:2217-2310)
 *   vcclKernelTypeOf      replaces the generated function table's type
 *                         equivalence (src/device/generate.py:129-137)
 *
 * Plain pointers and sizes only; device pointers must be valid on the device
 * that is current when the call is made.  All calls are asynchronous on
 * `stream` and capture-safe (no allocation, no synchronisation).
 */
#ifndef VCCL_DEVICE_H_
#define VCCL_DEVICE_H_

#include <stddef.h>
#include <stdint.h>

#include "nccl.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ncclDevRedOp_t (src/include/device.h:34-38) plus a byte copy. */
typedef enum {
  vcclDevSum = 0,
  vcclDevProd = 1,
  vcclDevMinMax = 2,
  vcclDevPreMulSum = 3,
  vcclDevSumPostDiv = 4,
  vcclDevCopy = 15 /* FuncCopy: datatype must be ncclUint8/ncclInt8 */
} vcclDevRedOp_t;

#define VCCL_MAX_SRCS 8
#define VCCL_MAX_DSTS 8

/* dst_j[i] = postOp( preOp(src_0[i]) (+) preOp?(src_1[i]) (+) ... ), i < nElts,
 * preOp applied to sources s < preOpSrcs, all with the scalar `redArg`
 * (PreMulSum); postOp (SumPostDiv divide) applied when postOp != 0.
 * Returns ncclInvalidArgument for unsupported (op, type), nSrcs/nDsts out of
 * [1, 8], or NULL pointers with nElts > 0. */
ncclResult_t vcclReduceCopy(vcclDevRedOp_t devOp, ncclDataType_t datatype, uint64_t redArg,
                            int preOpSrcs, int postOp, int nSrcs, const void* const* srcs,
                            int nDsts, void* const* dsts, size_t nElts, hipStream_t stream);

/* Launch-geometry override for measurement sweeps (0 = library default). */
typedef struct {
  int blockSize;    /* threads per workgroup: 64, 128, 256, 512 or 1024 */
  int unroll;       /* 16-byte packs in flight per thread per source: 1, 2, 4 or 8 */
  int gridBlocks;   /* workgroups in the grid */
  int ntLoads;      /* load policy: 0 plain, 1 nontemporal, 2 sc0 sc1, 3 sc1 nt */
  int ntStores;     /* store policy: same encoding; 16 | d0 | d1 << 2 sets the
                       two destinations' policies separately */
  int order;        /* hunk order: 0 round-robin, 1 XCD-contiguous, 2 LDS-staged,
                       3 stores interleaved across destinations, 4 pipelined */
} vcclLaunchConfig;
/* Sweep variants other than the defaults exist only for the fp32 sum shapes
 * 2 -> 1 (every field), 2 -> 2 (unroll 2/4, per-destination store policies,
 * order 0/3/4) and 1 -> 1 (unroll 2/4); other shapes always run the tuned
 * default. */

ncclResult_t vcclReduceCopyEx(vcclDevRedOp_t devOp, ncclDataType_t datatype, uint64_t redArg,
                              int preOpSrcs, int postOp, int nSrcs, const void* const* srcs,
                              int nDsts, void* const* dsts, size_t nElts, hipStream_t stream,
                              const vcclLaunchConfig* config);

/* hostToDevRedOp for built-in ops: devOp + 64-bit opArg (xormask for
 * min/max, 1/nRanks bits for float avg, nRanks<<1|signed for integer avg). */
ncclResult_t vcclHostToDevRedOp(ncclRedOp_t op, ncclDataType_t datatype, int nRanks,
                                int* devOp, uint64_t* opArg);

/* Kernel element type a (devOp, datatype) pair runs on, or -1 when the pair
 * is unsupported.  Pairs with the same value share one kernel. */
int vcclKernelTypeOf(int devOp, ncclDataType_t datatype);

/* Library build description (arch, defaults), for logs and tests. */
const char* vcclBuildInfo(void);

#ifdef __cplusplus
}
#endif
#endif /* VCCL_DEVICE_H_ */
