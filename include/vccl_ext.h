/*
 * vccl-mi355x communicator extensions (host only, no GPU work).
 *
 *   vcclCommCollAlgo  which algorithm ncclAllReduce / ncclReduceScatter /
 *                     ncclAllGather would run for (count, datatype) on this
 *                     communicator — the outcome of the tuner step
 *                     topoGetAlgoInfo (src/enqueue.cc:1805-1945) that VCCL
 *                     only reports through NCCL_DEBUG=INFO logs.  For
 *                     benchmarks and tests; enqueues nothing.
 *   vcclCommSetAlgo   per-communicator override of that choice (the
 *                     NCCL_ALGO / NCCL_PROTO environment, graph/tuning.cc:
 *                     354-373, read once at init): -1 = automatic, otherwise
 *                     a vcclAlgo_t; an algorithm that cannot carry a call
 *                     (bucket above its buffer, not an all-reduce) falls
 *                     through to the ring, as with the environment.
 *   vcclCommLaunchStats  collectives enqueued on this communicator so far and
 *                     how many launches carried more than one of them (group
 *                     aggregation of small all-reduces into one LL launch).
 *   vcclCommNetStats  payload bytes this rank's net proxy has sent / received
 *                     and its connection count (0 when every peer is reached
 *                     over xGMI).  The net transport carries ring connections
 *                     to peers on other nodes (or every connection with
 *                     VCCL_NET_FORCE=1) through host-pinned staging buffers
 *                     and TCP, as the reference's proxy + net transport
 *                     (src/proxy.cc:914-971, src/transport/net.cc:1293-1482).
 */
#ifndef VCCL_EXT_H_
#define VCCL_EXT_H_
#include <stddef.h>
#include <stdint.h>

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
ncclResult_t vcclCommSetAlgo(ncclComm_t comm, int algo);
ncclResult_t vcclCommLaunchStats(ncclComm_t comm, unsigned long long* collectives,
                                 unsigned long long* fusedLaunches);
ncclResult_t vcclCommNetStats(ncclComm_t comm, uint64_t* bytesSent, uint64_t* bytesReceived,
                              int* connections);

#ifdef __cplusplus
}
#endif
#endif /* VCCL_EXT_H_ */
