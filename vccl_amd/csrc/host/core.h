// Internal host-side structures of libvccl (not part of the ABI).
//
// The communicator keeps only what the MI355X ring needs; its fields map to
// the reference's ncclComm (src/include/comm.h) where one exists.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/nccl.h"
#include "../device/ring_types.hpp"

namespace vccl {
struct DirectPeers;  // direct.hpp
}

namespace vccl {

// ----------------------------------------------------------------- logging
// NCCL_DEBUG=WARN|INFO|TRACE (debug.h:22-34); VCCL_DEBUG is an alias.
enum LogLevel { kLogNone = 0, kLogWarn = 1, kLogInfo = 2, kLogTrace = 3 };
int log_level();
void reset_log_level();
// The last WARN's text (ncclGetLastError), kept whatever the log level.
const char* last_error();
void log_msg(int level, const char* file, int line, const char* fmt, ...)
    __attribute__((format(printf, 4, 5)));
#define VWARN(...) ::vccl::log_msg(::vccl::kLogWarn, __FILE__, __LINE__, __VA_ARGS__)
#define VINFO(...)                                                                   \
  do {                                                                               \
    if (::vccl::log_level() >= ::vccl::kLogInfo)                                     \
      ::vccl::log_msg(::vccl::kLogInfo, __FILE__, __LINE__, __VA_ARGS__);            \
  } while (0)

#define HIPCHECK(cmd)                                                                \
  do {                                                                               \
    hipError_t e_ = (cmd);                                                           \
    if (e_ != hipSuccess) {                                                          \
      VWARN("HIP failure '%s' in %s", hipGetErrorString(e_), #cmd);                 \
      return ncclUnhandledCudaError;                                                 \
    }                                                                                \
  } while (0)
#define NCCLCHECK(cmd)                                                               \
  do {                                                                               \
    ncclResult_t r_ = (cmd);                                                         \
    if (r_ != ncclSuccess) return r_;                                                \
  } while (0)

// ----------------------------------------------------------------- params
// NCCL_PARAM idiom (param.h:17-25): env NCCL_<name> (or VCCL_<name>), cached.
int64_t param_int(const char* name, int64_t deflt);

// ----------------------------------------------------------------- bootstrap
struct Bootstrap;  // opaque (bootstrap.cc)
ncclResult_t bootstrap_get_unique_id(ncclUniqueId* id);
// The socket to the root (ncclCommAbort shuts it to end a pending init).
int bootstrap_fd(const Bootstrap* b);
// `abortReq` (optional): stop retrying the root when it is raised.
ncclResult_t bootstrap_init(const ncclUniqueId* id, int rank, int nranks, Bootstrap** out,
                            const std::atomic<bool>* abortReq = nullptr);
// allgather of `bytes` per rank: buf holds nranks*bytes, own slot filled in.
ncclResult_t bootstrap_allgather(Bootstrap* b, void* buf, size_t bytes);
ncclResult_t bootstrap_barrier(Bootstrap* b);
void bootstrap_close(Bootstrap* b);
uint32_t bootstrap_local_ip(Bootstrap* b);

// ----------------------------------------------------------------- net proxy
// Inter-node ring connections through host-pinned staging buffers moved by a
// proxy thread pair over TCP (proxy.cc).  Opaque here.
struct NetProxy;

// ----------------------------------------------------------------- rings
// Ring orders for one node: for n in {2,4,8} the
// arc-balanced ring sets over the fully connected xGMI mesh; otherwise the
// identity ring.  Returns the list of rings (each a permutation of 0..n-1).
std::vector<std::vector<int>> ring_orders(int nranks);

// ----------------------------------------------------------------- comm
struct PeerMap {               // what one rank published about itself
  int pid;
  int device;
  uint64_t hostHash;
  int64_t busId;               // PCI domain/bus/device: the GPU's identity across processes
  uint32_t netIp;              // net proxy listener (network order), see proxy.cc
  uint16_t netPort;
  uint16_t cuCount;            // compute units of the device (co-residency cap of shared GPUs)
  hipIpcMemHandle_t fifoHandle;
  hipIpcMemHandle_t flagHandle;
  hipIpcMemHandle_t llHandle;
  hipIpcMemHandle_t dBufHandle;
  hipIpcMemHandle_t dFlagHandle;
  hipIpcMemHandle_t ll128Handle;
  char* fifoPtr;               // raw pointers (valid only in the owner process)
  char* flagPtr;
  char* llPtr;
  char* dBufPtr;
  char* dFlagPtr;
  char* ll128Ptr;
};

struct UserRedOp {             // ncclRedOpCreatePreMulSum state (enqueue.cc:2528-2567)
  int freeNext;                // -1 = allocated
  ncclDataType_t datatype;
  int devOp;
  bool argIsPtr;
  uint64_t arg;
};

}  // namespace vccl

struct ncclComm {
  uint64_t magic;
  int rank = 0, nRanks = 1, device = 0;
  int nChannels = 0, slotBytes = 0, nThreads = 0;
  int stepBytes = 0;  // VCCL's FIFO step: the partition / chunk unit (slotBytes = the FIFO slot)
  uint64_t* ringTrace = nullptr;  // VCCL_RING_TRACE: nChannels x ringTraceCap RingTraceRec
  int ringTraceCap = 0;
  int shareBlockCap = 0;  // ranks sharing a GPU: workgroups per launch that stay co-resident (0 = no cap)
  vccl::Bootstrap* bootstrap = nullptr;
  // device resources
  char* fifoBuf = nullptr;     // nChannels * kSteps * slotBytes, uncached
  char* flagBuf = nullptr;     // nChannels * 2 flags * kFlagStride, uncached
  // one-shot LL all-reduce (ll.hpp): [2 parities][nRanks][llLines] 16 B lines
  char* llBuf = nullptr;
  int llLines = 0;             // lines per (parity, source) slot = llMaxBytes / 8
  size_t llMaxBytes = 0;       // largest all-reduce carried by LL
  std::vector<char*> llPeer;   // every rank's LL buffer mapped into this process
  // LL128 ring (ring.hpp prim_ll128): nChannels x kSteps slots of
  // ll128SlotBytes, uncached; VCCL's LL128 partition and chunk
  // (ll128ChunkBytes of data per step, enqueue.cc:2027-2032) and thread count
  // (NCCL_LL128_NTHREADS, tuning.cc:198-211) for the channel tuning.
  char* ll128Buf = nullptr;
  int64_t ll128SlotBytes = 0;
  int64_t ll128StepBytes = 0;  // NCCL_LL128_BUFFSIZE / NCCL_STEPS (init.cc:617-633)
  int ll128Threads = 640;
  size_t ll128MinBytes = 0, ll128MaxBytes = 0;  // automatic LL128 window (0 = off)
  // two-shot direct all-reduce (direct.hpp): inbox [2 phases][nRanks][dRegionBytes]
  char* dBuf = nullptr;
  char* dFlags = nullptr;      // kDirectFlagBytes of epoch flags
  size_t directMaxBytes = 0;   // largest all-reduce carried by the direct path
  size_t llRsAgMaxBytes = 0;   // largest RS / AG bucket (n blocks) on the one-hop LL path
  size_t directRsAgMaxBytes = 0;  // ... and on the one-hop direct path
  int64_t dRegionBytes = 0;
  int directMaxBlocks = 0;
  vccl::DirectPeers* dPeers = nullptr;  // device-resident peer table
  vccl::NetProxy* net = nullptr;  // inter-node ring connections (proxy.cc)
  int netListenFd = -1;        // proxy listener, open from init until connections are made
  int algoForce = 0;           // NCCL_ALGO/NCCL_PROTO: 0 auto, 1 ring/SIMPLE, 2 tree/LL, 3 direct, 4 LL128 ring
  int algoAllowed = 15;        // paths the NCCL_ALGO / NCCL_PROTO lists leave (init.cc algo_proto_select)
  vccl::DevComm* devComm = nullptr;
  vccl::DevChannel* devChannels = nullptr;
  volatile int* abortFlag = nullptr;  // host pinned, mapped
  int* errorFlag = nullptr;           // host pinned, mapped
  std::vector<void*> ipcOpened;       // peer mappings to close
  std::vector<vccl::PeerMap> peers;
  // ordering of launches on this comm across user streams
  hipEvent_t lastLaunch = nullptr;
  hipEvent_t joinEvent = nullptr;     // joins other streams into a fused group launch
  hipStream_t lastStream = nullptr;
  bool hasLastLaunch = false;         // lastLaunch/lastStream are valid
  // VCCL_DEBUG_NO_MARK=1 with no stop event bound: the last launch left no
  // event, so waiting for the comm's work polls lastStream instead
  bool lastUnmarked = false;
  // the same ordering inside each stream capture, keyed by capture id (two
  // captures on one comm may interleave): events recorded in the
  // graph, a small pool reused least-recently-used first (never destroyed
  // while the comm lives — a graph may still reference one)
  struct CapOrder {
    unsigned long long id = 0;
    bool used = false;
    hipEvent_t ev = nullptr;
    hipStream_t last = nullptr;
    bool has = false;
  };
  static constexpr int kMaxCaptures = 16;
  std::vector<CapOrder> caps;         // most recently used first
  uint64_t fusedLaunches = 0;         // group launches that carried > 1 collective
  int ringWave = 0;                   // SIMPLE ring launches take the per-wave hand-off (VCCL_RING_WAVE)
  uint64_t waveLaunches = 0;          // ring launches that ran the per-wave kernel
  // CTA (workgroup) bounds of every collective launch: ncclConfig_t
  // minCTAs / maxCTAs or NCCL_MIN_CTAS / NCCL_MAX_CTAS (init.cc:1478-1540)
  int minCTAs = 1, maxCTAs = 64;
  // Non-blocking communicator (ncclConfig_t.blocking = 0 / NCCL_COMM_BLOCKING=0,
  // group.cc:553-576): ncclCommInitRank* returns ncclInProgress and the
  // initialisation runs on initThread; ncclCommGetAsyncError reports
  // ncclInProgress until it ends, then its result.  Every other call on the
  // comm waits for it first (comm_check).
  int blocking = 1;
  std::atomic<bool> initPending{false};
  // ncclCommAbort of a pending non-blocking init: raise initAbort, shut the
  // bootstrap socket (initFd, published once connected) so a wait on peers
  // that never come ends at once
  std::atomic<bool> initAbort{false};
  std::atomic<int> initFd{-1};
  ncclResult_t initResult = ncclSuccess;
  std::thread initThread;
  std::mutex initMutex;
  // state
  std::atomic<int> asyncError{0};
  std::vector<vccl::UserRedOp> userOps;
  int userOpFreeHead = 0;
  uint64_t opCount = 0;
  bool destroyed = false;
};

namespace vccl {
constexpr uint64_t kCommMagic = 0x76636363'6c6d6933ull;  // "vccclmi3"
// A valid, live comm whose initialisation has ended (a non-blocking one is
// waited for); its result unless allowFailedInit (destroy / abort).
ncclResult_t comm_check(const ncclComm* comm, const char* api, bool allowFailedInit = false);
// The same without waiting for a non-blocking initialisation (GetAsyncError).
ncclResult_t comm_check_live(const ncclComm* comm, const char* api);
// Waits until every eager launch of `comm` has completed (init.cc).
ncclResult_t comm_wait_own_launches(ncclComm* comm);
// The comm's device error word as a result code (init.cc).
ncclResult_t error_word_result(ncclComm* comm);

// Net proxy (proxy.cc).  net_listen opens this rank's listener before the
// peer exchange (address published in `me`); net_connect builds the
// connections of every channel whose prev / next is flagged in netPeer,
// points those channel ends at host-pinned staging memory and starts the
// proxy threads; net_stop joins them and frees everything (idempotent).
ncclResult_t net_listen(ncclComm* c, PeerMap* me);
ncclResult_t net_connect(ncclComm* c, const std::vector<std::vector<int>>& rings,
                         std::vector<DevChannel>& chans, const std::vector<char>& netPeer);
void net_stop(ncclComm* c);
}  // namespace vccl
