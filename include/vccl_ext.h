/*
 * vccl-mi355x communicator extensions (host only, no GPU work).
 *
 *   vcclCommCollAlgo  which algorithm ncclAllReduce / ncclReduceScatter /
 *                     ncclAllGather would run for (count, datatype) on this
 *                     communicator — the outcome of the tuner step
 *                     topoGetAlgoInfo (src/enqueue.cc:1805-1945) that VCCL
 *                     only reports through NCCL_DEBUG=INFO logs.  For
 *                     benchmarks and tests; enqueues nothing.
 */
#ifndef VCCL_EXT_H_
#define VCCL_EXT_H_
#include <stddef.h>

#include "nccl.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef enum { vcclCollAllReduce = 0, vcclCollReduceScatter = 1, vcclCollAllGather = 2 } vcclColl_t;
typedef enum {
  vcclAlgoRing = 0,     /* SIMPLE ring over arc-balanced ring sets */
  vcclAlgoLL = 1,       /* one-shot LL all-reduce, chain-tree fold */
  vcclAlgoDirect = 2,   /* two-shot direct all-reduce over the full mesh */
  vcclAlgoOneRank = 3   /* nRanks == 1: copy / PreMulSum kernel */
} vcclAlgo_t;

ncclResult_t vcclCommCollAlgo(ncclComm_t comm, int coll, size_t count, ncclDataType_t datatype,
                              int* algo);

#ifdef __cplusplus
}
#endif
#endif /* VCCL_EXT_H_ */
