/*
 * vccl-mi355x public C ABI — drop-in for the bucket-reduction path of VCCL.
 *
 * Every declaration below replaces the identically named one in the
 * reference header /root/reference/src/nccl.h.in (file:line cited per item).
 * Enum values and argument order are identical; the only change is the stream
 * type (hipStream_t in place of cudaStream_t).  Every function is exported as
 * `ncclX` and as the profiling alias `pncclX` (reference: src/include/core.h:18-31).
 *
 * Scope: AllReduce / ReduceScatter / AllGather over the
 * repo's own transport (xGMI peer memory, no RCCL) and the comm lifecycle they
 * need, Broadcast / Bcast (the byte-copy ring), Reduce (the reduce ring),
 * CommSplit, MemAlloc / MemFree, Register / Deregister (a no-op) and
 * InitRankScalable.  The calls of the "out of scope" block at the end (Send, Recv,
 * GroupSimulateEnd, RCCL's AllToAll / AllToAllv) are declared and exported so a binary linked against
 * libnccl still loads; each logs a WARN and returns ncclInvalidUsage.
 */
#ifndef VCCL_NCCL_H_
#define VCCL_NCCL_H_

#include <hip/hip_runtime_api.h>
#include <limits.h>
#include <stddef.h>

#define NCCL_MAJOR 2
#define NCCL_MINOR 26
#define NCCL_PATCH 62
#define NCCL_SUFFIX ""
/* nccl.h.in:24 */
#define NCCL_VERSION(X, Y, Z) \
  (((X) <= 2 && (Y) <= 8) ? (X)*1000 + (Y)*100 + (Z) : (X)*10000 + (Y)*100 + (Z))
#define NCCL_VERSION_CODE NCCL_VERSION(NCCL_MAJOR, NCCL_MINOR, NCCL_PATCH)

#ifdef __cplusplus
extern "C" {
#endif

/* nccl.h.in:31-36 */
typedef struct ncclComm* ncclComm_t;
#define NCCL_COMM_NULL NULL
#define NCCL_UNIQUE_ID_BYTES 128
typedef struct { char internal[NCCL_UNIQUE_ID_BYTES]; } ncclUniqueId;

/* The enums below are int-sized as in the reference; C++ translation units
 * see that as a fixed underlying type, so a caller's out-of-range value (an
 * invalid datatype or op, which the library must reject with
 * ncclInvalidArgument) is a well-defined int there, not undefined behaviour
 * (found by `make sanitize`, UBSan's enum check). */
#ifdef __cplusplus
#define VCCL_ENUM_INT : int
#else
#define VCCL_ENUM_INT
#endif

/* nccl.h.in:40-48 */
typedef enum VCCL_ENUM_INT {
  ncclSuccess = 0,
  ncclUnhandledCudaError = 1, /* a HIP runtime call failed */
  ncclSystemError = 2,
  ncclInternalError = 3,
  ncclInvalidArgument = 4,
  ncclInvalidUsage = 5,
  ncclRemoteError = 6,
  ncclInProgress = 7,
  ncclNumResults = 8
} ncclResult_t;

#define NCCL_CONFIG_UNDEF_INT INT_MIN
#define NCCL_CONFIG_UNDEF_PTR NULL
#define NCCL_SPLIT_NOCOLOR -1
#define NCCL_UNDEF_FLOAT -1.0f

/* nccl.h.in:57-85 — same layout and magic. */
typedef struct ncclConfig_v21700 {
  size_t size;
  unsigned int magic;
  unsigned int version;
  int blocking;
  int cgaClusterSize;
  int minCTAs;
  int maxCTAs;
  const char* netName;
  int splitShare;
  int trafficClass;
} ncclConfig_t;

#define NCCL_CONFIG_INITIALIZER {                                   \
    sizeof(ncclConfig_t), 0xcafebeef,                               \
    NCCL_VERSION(NCCL_MAJOR, NCCL_MINOR, NCCL_PATCH),               \
    NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_INT,                   \
    NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_INT,                   \
    NCCL_CONFIG_UNDEF_PTR, NCCL_CONFIG_UNDEF_INT,                   \
    NCCL_CONFIG_UNDEF_INT }

/* nccl.h.in:220-236 */
typedef enum { ncclNumOps_dummy = 5 } ncclRedOp_dummy_t;
typedef enum VCCL_ENUM_INT {
  ncclSum = 0,
  ncclProd = 1,
  ncclMax = 2,
  ncclMin = 3,
  ncclAvg = 4,
  ncclNumOps = 5,
  ncclMaxRedOp = 0x7fffffff >> (32 - 8 * sizeof(ncclRedOp_dummy_t))
} ncclRedOp_t;

/* nccl.h.in:239-252 */
typedef enum VCCL_ENUM_INT {
  ncclInt8 = 0, ncclChar = 0,
  ncclUint8 = 1,
  ncclInt32 = 2, ncclInt = 2,
  ncclUint32 = 3,
  ncclInt64 = 4,
  ncclUint64 = 5,
  ncclFloat16 = 6, ncclHalf = 6,
  ncclFloat32 = 7, ncclFloat = 7,
  ncclFloat64 = 8, ncclDouble = 8,
  ncclBfloat16 = 9,
  ncclFloat8e4m3 = 10,
  ncclFloat8e5m2 = 11,
  ncclNumTypes = 12
} ncclDataType_t;

/* nccl.h.in:255-262 */
typedef enum VCCL_ENUM_INT {
  ncclScalarDevice = 0,
  ncclScalarHostImmediate = 1
} ncclScalarResidence_t;

/* ---- version / ids / lifecycle (nccl.h.in:117-217) ---- */
ncclResult_t  ncclGetVersion(int* version);
ncclResult_t pncclGetVersion(int* version);
ncclResult_t  ncclGetUniqueId(ncclUniqueId* uniqueId);
ncclResult_t pncclGetUniqueId(ncclUniqueId* uniqueId);
ncclResult_t  ncclCommInitRankConfig(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank, ncclConfig_t* config);
ncclResult_t pncclCommInitRankConfig(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank, ncclConfig_t* config);
ncclResult_t  ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank);
ncclResult_t pncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank);
ncclResult_t  ncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist);
ncclResult_t pncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist);
ncclResult_t  ncclCommFinalize(ncclComm_t comm);
ncclResult_t pncclCommFinalize(ncclComm_t comm);
ncclResult_t  ncclCommDestroy(ncclComm_t comm);
ncclResult_t pncclCommDestroy(ncclComm_t comm);
ncclResult_t  ncclCommAbort(ncclComm_t comm);
ncclResult_t pncclCommAbort(ncclComm_t comm);
const char*  ncclGetErrorString(ncclResult_t result);
const char* pncclGetErrorString(ncclResult_t result);
const char*  ncclGetLastError(ncclComm_t comm);
const char* pncclGetLastError(ncclComm_t comm);
/* nccl.h.in:191-193: reload the environment variables that set logging */
void  ncclResetDebugInit(void);
void pncclResetDebugInit(void);
ncclResult_t  ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError);
ncclResult_t pncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError);
ncclResult_t  ncclCommCount(const ncclComm_t comm, int* count);
ncclResult_t pncclCommCount(const ncclComm_t comm, int* count);
ncclResult_t  ncclCommCuDevice(const ncclComm_t comm, int* device);
ncclResult_t pncclCommCuDevice(const ncclComm_t comm, int* device);
ncclResult_t  ncclCommUserRank(const ncclComm_t comm, int* rank);
ncclResult_t pncclCommUserRank(const ncclComm_t comm, int* rank);

/* ---- user reduction ops (nccl.h.in:264-283; enqueue.cc:2528-2598) ---- */
ncclResult_t  ncclRedOpCreatePreMulSum(ncclRedOp_t* op, void* scalar, ncclDataType_t datatype, ncclScalarResidence_t residence, ncclComm_t comm);
ncclResult_t pncclRedOpCreatePreMulSum(ncclRedOp_t* op, void* scalar, ncclDataType_t datatype, ncclScalarResidence_t residence, ncclComm_t comm);
ncclResult_t  ncclRedOpDestroy(ncclRedOp_t op, ncclComm_t comm);
ncclResult_t pncclRedOpDestroy(ncclRedOp_t op, ncclComm_t comm);

/* ---- collectives on the hot path ---- */
/* nccl.h.in:353-356; collectives.cc:93-106 */
ncclResult_t  ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count,
    ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm, hipStream_t stream);
ncclResult_t pncclAllReduce(const void* sendbuff, void* recvbuff, size_t count,
    ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm, hipStream_t stream);
/* nccl.h.in:369-374; collectives.cc:145-158 */
ncclResult_t  ncclReduceScatter(const void* sendbuff, void* recvbuff, size_t recvcount,
    ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm, hipStream_t stream);
ncclResult_t pncclReduceScatter(const void* sendbuff, void* recvbuff, size_t recvcount,
    ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm, hipStream_t stream);
/* nccl.h.in:386-389; collectives.cc:77-91 */
ncclResult_t  ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount,
    ncclDataType_t datatype, ncclComm_t comm, hipStream_t stream);
ncclResult_t pncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount,
    ncclDataType_t datatype, ncclComm_t comm, hipStream_t stream);

/* ---- group semantics (nccl.h.in:425-465; group.cc:92-110) ---- */
ncclResult_t  ncclGroupStart(void);
ncclResult_t pncclGroupStart(void);
ncclResult_t  ncclGroupEnd(void);
ncclResult_t pncclGroupEnd(void);

/* ---- broadcast: the ring broadcast (src/device/broadcast.h), the byte-copy
 * ring of the all-gather from one root (torch's DDP broadcasts its module
 * state with it) ---- */
/* nccl.h.in:326-329 (in place) */
ncclResult_t  ncclBcast(void* buff, size_t count, ncclDataType_t datatype, int root,
    ncclComm_t comm, hipStream_t stream);
ncclResult_t pncclBcast(void* buff, size_t count, ncclDataType_t datatype, int root,
    ncclComm_t comm, hipStream_t stream);
/* nccl.h.in:340-343 */
ncclResult_t  ncclBroadcast(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
    int root, ncclComm_t comm, hipStream_t stream);
ncclResult_t pncclBroadcast(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
    int root, ncclComm_t comm, hipStream_t stream);
/* nccl.h.in:312-315: the ring reduce (reduce.h) into root's recvbuff; a
 * non-root's recvbuff is never written and may be NULL */
ncclResult_t  ncclReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
    ncclRedOp_t op, int root, ncclComm_t comm, hipStream_t stream);
ncclResult_t pncclReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
    ncclRedOp_t op, int root, ncclComm_t comm, hipStream_t stream);

/* ---- memory, registration and scalable init (nccl.h.in:104-111, :178-181,
 * :208-217): exported so a caller linked against libnccl (PyTorch's nccl
 * backend imports all of them) never reaches another library with this
 * library's communicator.  ncclMemAlloc / Free = hipMalloc / hipFree;
 * registration is a no-op (zero-copy registration is out of scope, buffers
 * work unregistered; *handle = buff); ncclCommInitRankScalable = InitRankConfig
 * on commIds[0]'s root. ---- */
ncclResult_t  ncclMemAlloc(void** ptr, size_t size);
ncclResult_t pncclMemAlloc(void** ptr, size_t size);
ncclResult_t  ncclMemFree(void* ptr);
ncclResult_t pncclMemFree(void* ptr);
ncclResult_t  ncclCommInitRankScalable(ncclComm_t* newcomm, int nranks, int myrank, int nId,
    ncclUniqueId* commIds, ncclConfig_t* config);
ncclResult_t pncclCommInitRankScalable(ncclComm_t* newcomm, int nranks, int myrank, int nId,
    ncclUniqueId* commIds, ncclConfig_t* config);
ncclResult_t  ncclCommRegister(const ncclComm_t comm, void* buff, size_t size, void** handle);
ncclResult_t pncclCommRegister(const ncclComm_t comm, void* buff, size_t size, void** handle);
ncclResult_t  ncclCommDeregister(const ncclComm_t comm, void* handle);
ncclResult_t pncclCommDeregister(const ncclComm_t comm, void* handle);
/* nccl.h.in:173-174: ranks of one color form a new communicator ordered by
 * (key, parent rank); NCCL_SPLIT_NOCOLOR joins none (*newcomm = NULL).
 * Collective over `comm`; config NULL = defaults. */
ncclResult_t  ncclCommSplit(ncclComm_t comm, int color, int key, ncclComm_t* newcomm, ncclConfig_t* config);
ncclResult_t pncclCommSplit(ncclComm_t comm, int color, int key, ncclComm_t* newcomm, ncclConfig_t* config);

/* nccl.h.in:87-102 */
typedef struct ncclSimInfo_v22200 {
  size_t size;
  unsigned int magic;
  unsigned int version;
  float estimatedTime;
} ncclSimInfo_t;
#define NCCL_SIM_INFO_INITIALIZER {                                         \
  sizeof(ncclSimInfo_t), 0x74685283,                                        \
  NCCL_VERSION(NCCL_MAJOR, NCCL_MINOR, NCCL_PATCH), NCCL_UNDEF_FLOAT }

/* ---- out of scope: WARN + ncclInvalidUsage ---- */
/* nccl.h.in:472-473: ends the group (nothing launched) without an estimate
 * (the tuner's cost model is out of scope) */
ncclResult_t  ncclGroupSimulateEnd(ncclSimInfo_t* simInfo);
ncclResult_t pncclGroupSimulateEnd(ncclSimInfo_t* simInfo);
/* nccl.h.in:403-406 */
ncclResult_t  ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer,
    ncclComm_t comm, hipStream_t stream);
ncclResult_t pncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer,
    ncclComm_t comm, hipStream_t stream);
/* nccl.h.in:420-423 */
ncclResult_t  ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer,
    ncclComm_t comm, hipStream_t stream);
ncclResult_t pncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer,
    ncclComm_t comm, hipStream_t stream);
/* RCCL's all-to-all extensions (not VCCL API; PyTorch's ROCm build imports
 * them): out of scope too */
ncclResult_t  ncclAllToAll(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
    ncclComm_t comm, hipStream_t stream);
ncclResult_t pncclAllToAll(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
    ncclComm_t comm, hipStream_t stream);
ncclResult_t  ncclAllToAllv(const void* sendbuff, const size_t sendcounts[], const size_t sdispls[],
    void* recvbuff, const size_t recvcounts[], const size_t rdispls[], ncclDataType_t datatype,
    ncclComm_t comm, hipStream_t stream);
ncclResult_t pncclAllToAllv(const void* sendbuff, const size_t sendcounts[], const size_t sdispls[],
    void* recvbuff, const size_t recvcounts[], const size_t rdispls[], ncclDataType_t datatype,
    ncclComm_t comm, hipStream_t stream);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* VCCL_NCCL_H_ */
