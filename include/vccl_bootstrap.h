/*
 * vccl-mi355x bootstrap diagnostic entry (host only, no GPU).
 *
 *   vcclBootstrapAllGather  one all-gather round over the communicator
 *                           rendezvous of ncclGetUniqueId / ncclCommInitRank;
 *                           replaces bootstrapAllGather
 *                           (src/include/bootstrap.h:19-33, src/bootstrap.cc:1037)
 *                           as a callable unit for multi-process host tests.
 *
 * `buf` holds nranks * bytesPerRank bytes; the caller fills its own slot
 * (rank * bytesPerRank) and receives every rank's slot.  Blocking.
 */
#ifndef VCCL_BOOTSTRAP_H_
#define VCCL_BOOTSTRAP_H_
#include <stddef.h>

#include "nccl.h"

#ifdef __cplusplus
extern "C" {
#endif

ncclResult_t vcclBootstrapAllGather(const ncclUniqueId* id, int rank, int nranks, void* buf,
                                    size_t bytesPerRank);

#ifdef __cplusplus
}
#endif
#endif /* VCCL_BOOTSTRAP_H_ */
