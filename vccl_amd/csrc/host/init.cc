// Communicator lifecycle: unique id, init (rank / all), destroy, abort, queries.
//
// Reference: src/init.cc (ncclCommInitRankDev :1651-1730, ncclCommInitAll
// :1750-1814, initTransportsRank :672-1276, setupChannel :599-615) and the
// P2P transport (src/transport/p2p.cc:209-560).  MI355X design: no topology
// search — one node, fully connected xGMI mesh, fixed arc-balanced ring sets
// (SURVEY.md Appendix D); each channel's FIFO and flags live in the receiver's
// HBM (uncached) and are mapped into the sender by hipIpc* (multi-process) or
// peer access (single process).
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstring>
#include <string>
#include <thread>

#include "../../../include/vccl_ext.h"
#include "../device/coll_types.hpp"
#include "../device/ring_launch.hpp"
#include "core.h"

namespace vccl {

ncclResult_t comm_check_live(const ncclComm* comm, const char* api) {
  if (comm == nullptr) {
    VWARN("%s : comm argument is NULL", api);
    return ncclInvalidArgument;
  }
  if (comm->magic != kCommMagic || comm->destroyed) {
    VWARN("%s : comm argument is invalid or destroyed", api);
    return ncclInvalidArgument;
  }
  return ncclSuccess;
}

// Joins a non-blocking comm's initialisation thread (once, whichever caller
// gets there first).
static void wait_init(ncclComm* c) {
  if (c->blocking) return;
  std::lock_guard<std::mutex> g(c->initMutex);
  if (c->initThread.joinable()) c->initThread.join();
}

// ncclCommEnsureReady (init.cc:300-317): a comm whose non-blocking
// initialisation has not ended is not usable yet — every call but
// ncclCommGetAsyncError and ncclCommAbort fails with ncclInvalidArgument
// (ncclCommDestroy too, init.cc:2066), it does not wait.
ncclResult_t comm_check(const ncclComm* comm, const char* api, bool allowFailedInit) {
  NCCLCHECK(comm_check_live(comm, api));
  ncclComm* c = const_cast<ncclComm*>(comm);
  if (!c->blocking && c->initPending.load(std::memory_order_acquire)) {
    VWARN("%s : Attempt to use communicator before the previous operation returned ncclSuccess", api);
    return ncclInvalidArgument;
  }
  wait_init(c);
  if (!allowFailedInit && c->initResult != ncclSuccess) {
    VWARN("%s : the communicator's initialisation failed (%d)", api, (int)c->initResult);
    return c->initResult;
  }
  return ncclSuccess;
}

// Walecki's decomposition of the complete graph on an odd number of vertices
// n = 2m + 1 into m edge-disjoint Hamiltonian cycles: vertex n-1 (the hub)
// followed by the zigzag k, k+1, k-1, k+2, k-2, ... over 0..2m-1 (mod 2m),
// k = 0..m-1.  Each cycle run in both directions gives n-1 arc-disjoint
// directed rings that use every xGMI link once per direction.
static std::vector<std::vector<int>> walecki_rings(int n) {
  const int m = (n - 1) / 2, h = 2 * m;
  std::vector<std::vector<int>> out;
  for (int k = 0; k < m; k++) {
    std::vector<int> cyc{n - 1, k};
    for (int j = 1; (int)cyc.size() < n; j++) {
      cyc.push_back(((k + j) % h + h) % h);
      if ((int)cyc.size() < n) cyc.push_back(((k - j) % h + h) % h);
    }
    out.push_back(cyc);
    std::vector<int> rev{cyc[0]};
    for (int i = n - 1; i >= 1; i--) rev.push_back(cyc[i]);
    out.push_back(rev);
  }
  // rotate each ring to start at rank 0 (cosmetic: a ring is a cycle)
  for (auto& r : out) std::rotate(r.begin(), std::find(r.begin(), r.end(), 0), r.end());
  return out;
}

// Ring sets over the fully connected xGMI mesh (SURVEY.md Appendix D,
// verified by tests/test_ring_schedule.py):
//   8 GPUs: 7 arc-disjoint directed Hamiltonian cycles (every link carries
//           one ring per direction);
//   4 GPUs: all 6 directed Hamiltonian cycles (every arc in exactly 2: no
//           arc-disjoint decomposition exists);
//   odd n (3, 5, 7): Walecki's n-1 arc-disjoint directed rings;
//   6 GPUs: two edge-disjoint Hamiltonian cycles, both directions (4 of each
//           rank's 5 links; K6 has no directed Hamiltonian decomposition);
//   2 GPUs: the single ring.
std::vector<std::vector<int>> ring_orders(int n) {
  if (n == 8)
    return {{0, 1, 2, 3, 4, 5, 6, 7}, {0, 2, 1, 3, 5, 4, 7, 6}, {0, 3, 1, 4, 6, 2, 7, 5},
            {0, 4, 1, 5, 7, 2, 6, 3}, {0, 5, 3, 6, 1, 7, 4, 2}, {0, 6, 5, 2, 4, 3, 7, 1},
            {0, 7, 3, 2, 5, 1, 6, 4}};
  if (n == 4)
    return {{0, 1, 2, 3}, {0, 1, 3, 2}, {0, 2, 1, 3}, {0, 2, 3, 1}, {0, 3, 1, 2}, {0, 3, 2, 1}};
  if (n == 6)
    return {{0, 1, 2, 3, 4, 5}, {0, 5, 4, 3, 2, 1}, {0, 2, 4, 1, 5, 3}, {0, 3, 5, 1, 4, 2}};
  if (n >= 3 && n % 2 == 1 && n - 1 <= kOrderMaxRings) return walecki_rings(n);
  std::vector<int> id(n);
  for (int i = 0; i < n; i++) id[i] = i;
  return {id};
}

// NCCL_ALGO / NCCL_PROTO (read once at init): the reference's parseList
// (graph/tuning.cc:53-116) — a comma list of names, case-insensitive, a
// leading '^' enables everything but the listed ones; per-collective
// "func:list" entries after a ';' are not supported here (WARNed and
// ignored).  Unknown names, or lists that leave no protocol or no algorithm
// at all, fail init with ncclInvalidUsage.  Paths: the one-hop LL
// all-reduce (protocol LL, algorithm Tree: it restates VCCL's chain-tree LL
// fold), the one-hop LL reduce-scatter / all-gather (protocol LL, algorithm
// Tree or Ring: they restate VCCL's ring-LL fold), the LL128 ring, the SIMPLE
// ring, and the direct path (algorithm "Direct", an extension; allowed only
// while NCCL_ALGO is unset or lists it).  A path is forced when it is the
// only one the lists leave; otherwise the excluded ones are dropped from the
// automatic choice.  A pair the reference accepts but no path here serves
// (e.g. Tree with Simple: VCCL's SIMPLE tree is out of scope) falls back to
// the SIMPLE ring, or the LL128 ring when Simple is excluded, with a WARN
// (ADVICE r4, r5); with neither allowed it fails (ncclInvalidUsage).
enum { kAllowLL = 1, kAllowLL128 = 2, kAllowSimple = 4, kAllowDirect = 8, kAllowLLRsAg = 16 };
static ncclResult_t parse_name_list(const char* env, const char* str, const char* const* names, int nNames,
                                    unsigned* mask) {
  *mask = (1u << nNames) - 1;
  if (!str || !*str) return ncclSuccess;
  std::string s(str);
  const size_t semi = s.find(';');
  if (semi != std::string::npos) {
    VWARN("%s=%s: per-collective entries are not supported, using \"%s\"", env, str, s.substr(0, semi).c_str());
    s = s.substr(0, semi);
  }
  if (s.find(':') != std::string::npos) {
    VWARN("%s=%s: per-collective entries are not supported, ignored", env, str);
    return ncclSuccess;
  }
  bool exclude = false;
  if (!s.empty() && s[0] == '^') {
    exclude = true;
    s = s.substr(1);
  }
  unsigned listed = 0;
  size_t pos = 0;
  while (pos <= s.size()) {
    size_t comma = s.find(',', pos);
    if (comma == std::string::npos) comma = s.size();
    const std::string tok = s.substr(pos, comma - pos);
    pos = comma + 1;
    if (tok.empty()) continue;
    int k = 0;
    while (k < nNames && strcasecmp(tok.c_str(), names[k]) != 0) k++;
    if (k == nNames) {
      VWARN("Unrecognized element token \"%s\" when parsing %s=\"%s\"", tok.c_str(), env, str);
      return ncclInvalidUsage;
    }
    listed |= 1u << k;
  }
  *mask = exclude ? ((1u << nNames) - 1) & ~listed : listed;
  return ncclSuccess;
}
ncclResult_t algo_proto_select(const char* algo, const char* proto, int* force, int* allowed) {
  static const char* const kProtos[] = {"LL", "LL128", "Simple"};
  static const char* const kAlgos[] = {"Tree", "Ring", "CollnetDirect", "CollnetChain", "NVLS", "NVLSTree",
                                       "PAT", "Direct"};
  unsigned p = 0, a = 0;
  NCCLCHECK(parse_name_list("NCCL_PROTO", proto, kProtos, 3, &p));
  NCCLCHECK(parse_name_list("NCCL_ALGO", algo, kAlgos, 8, &a));
  if (p == 0 || a == 0) {
    VWARN("NCCL_ALGO=%s / NCCL_PROTO=%s leave no %s", algo ? algo : "", proto ? proto : "",
          p == 0 ? "protocol" : "algorithm");
    return ncclInvalidUsage;
  }
  const bool tree = a & 1, ring = a & 2, direct = a & 0x80;
  // the one-hop LL all-reduce restates VCCL's chain-tree LL fold (Tree), the
  // one-hop LL reduce-scatter / all-gather its ring-LL one (Tree or Ring, as
  // before: VCCL's tree carries no RS / AG); the direct path moves
  // SIMPLE-style bulk copies
  int m = 0;
  if ((p & 1) && tree) m |= kAllowLL | kAllowLLRsAg;
  if ((p & 1) && ring) m |= kAllowLLRsAg;
  if ((p & 2) && ring) m |= kAllowLL128;
  if ((p & 4) && ring) m |= kAllowSimple;
  if ((p & 4) && direct) m |= kAllowDirect;
  if (m == 0) {
    // No path here serves the pair (e.g. Tree + Simple: VCCL's SIMPLE tree is
    // out of scope).  Fall back only to a ring whose protocol the user still
    // allows: the SIMPLE ring, else the LL128 ring; a list that
    // leaves only LL with no LL path for its algorithms is refused.
    const int fb = (p & 4) ? kAllowSimple : (p & 2) ? kAllowLL128 : 0;
    if (!fb) {
      VWARN("NCCL_ALGO=%s / NCCL_PROTO=%s: no path of this library serves that pair with an allowed protocol",
            algo ? algo : "", proto ? proto : "");
      return ncclInvalidUsage;
    }
    VWARN("NCCL_ALGO=%s / NCCL_PROTO=%s: no path of this library serves that pair; using the %s ring",
          algo ? algo : "", proto ? proto : "", fb == kAllowSimple ? "SIMPLE" : "LL128");
    m = fb;
  }
  const int f = m == kAllowDirect ? 3 : m == kAllowLL128 ? 4 : m == kAllowSimple ? 1
                : (m & ~(kAllowLL | kAllowLLRsAg)) == 0 ? 2 : 0;
  *force = f;
  *allowed = m;
  return ncclSuccess;
}

static uint64_t host_hash() {
  char name[256] = {0};
  gethostname(name, sizeof(name) - 1);
  uint64_t h = 1469598103934665603ull;
  for (char* p = name; *p; p++) h = (h ^ (uint8_t)*p) * 1099511628211ull;
  return h;
}

static ncclResult_t alloc_uncached(void** p, size_t bytes) {
  // NCCL_FIFO_ALLOC: 0 = uncached (default), 1 = fine-grained, 2 = coarse (hipMalloc)
  int mode = (int)param_int("FIFO_ALLOC", 0);
  hipError_t e;
  if (mode == 2) e = hipMalloc(p, bytes);
  else e = hipExtMallocWithFlags(p, bytes, mode == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached);
  if (e != hipSuccess) {
    VWARN("FIFO allocation of %zu bytes failed: %s", bytes, hipGetErrorString(e));
    return ncclUnhandledCudaError;
  }
  return ncclSuccess;
}

static void free_resources(ncclComm* c) {
  net_stop(c);  // first: its threads read the host staging memory and flags
  for (void* p : c->ipcOpened) (void)hipIpcCloseMemHandle(p);
  c->ipcOpened.clear();
  if (c->fifoBuf) (void)hipFree(c->fifoBuf);
  if (c->flagBuf) (void)hipFree(c->flagBuf);
  if (c->llBuf) (void)hipFree(c->llBuf);
  c->llBuf = nullptr;
  if (c->ll128Buf) (void)hipFree(c->ll128Buf);
  c->ll128Buf = nullptr;
  if (c->dBuf) (void)hipFree(c->dBuf);
  if (c->dFlags) (void)hipFree(c->dFlags);
  if (c->dPeers) (void)hipFree(c->dPeers);
  c->dBuf = c->dFlags = nullptr;
  c->dPeers = nullptr;
  if (c->devComm) (void)hipFree(c->devComm);
  if (c->ringTrace) (void)hipFree(c->ringTrace);
  c->ringTrace = nullptr;
  if (c->devChannels) (void)hipFree(c->devChannels);
  if (c->abortFlag) (void)hipHostFree((void*)c->abortFlag);
  if (c->errorFlag) (void)hipHostFree(c->errorFlag);
  if (c->lastLaunch) (void)hipEventDestroy(c->lastLaunch);
  if (c->joinEvent) (void)hipEventDestroy(c->joinEvent);
  for (auto& cap : c->caps)
    if (cap.ev) (void)hipEventDestroy(cap.ev);
  c->caps.clear();
  c->joinEvent = nullptr;
  c->fifoBuf = c->flagBuf = nullptr;
  c->devComm = nullptr;
  c->devChannels = nullptr;
  c->abortFlag = nullptr;
  c->errorFlag = nullptr;
  c->lastLaunch = nullptr;
}

// Map a peer's buffer into this process/device.
enum { kMapFifo = 0, kMapFlag = 1, kMapLL = 2, kMapDirect = 3, kMapDirectFlag = 4, kMapLL128 = 5 };
static ncclResult_t map_peer(ncclComm* c, const PeerMap& me, const PeerMap& p, int which,
                             char** out) {
  char* const raws[] = {p.fifoPtr, p.flagPtr, p.llPtr, p.dBufPtr, p.dFlagPtr, p.ll128Ptr};
  const hipIpcMemHandle_t* const handles[] = {&p.fifoHandle, &p.flagHandle, &p.llHandle,
                                              &p.dBufHandle, &p.dFlagHandle, &p.ll128Handle};
  char* raw = raws[which];
  const hipIpcMemHandle_t& handle = *handles[which];
  if (p.pid == me.pid && p.hostHash == me.hostHash) {
    if (p.device != c->device) {
      hipError_t e = hipDeviceEnablePeerAccess(p.device, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
        VWARN("hipDeviceEnablePeerAccess(%d -> %d) failed: %s", c->device, p.device,
              hipGetErrorString(e));
        return ncclUnhandledCudaError;
      }
      (void)hipGetLastError();
    }
    *out = raw;
    return ncclSuccess;
  }
  void* ptr = nullptr;
  hipError_t e = hipIpcOpenMemHandle(&ptr, handle, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) {
    VWARN("hipIpcOpenMemHandle failed: %s", hipGetErrorString(e));
    return ncclUnhandledCudaError;
  }
  c->ipcOpened.push_back(ptr);
  *out = (char*)ptr;
  return ncclSuccess;
}

static ncclResult_t init_rank(ncclComm* c, const ncclUniqueId* id) {
  VINFO("rank %d/%d dev %d: bootstrap", c->rank, c->nRanks, c->device);
  NCCLCHECK(bootstrap_init(id, c->rank, c->nRanks, &c->bootstrap, &c->initAbort));
  // an abort of a pending non-blocking init shuts this socket (ncclCommAbort);
  // publish first, then look at the flag, so one of the two sides sees the other
  c->initFd.store(bootstrap_fd(c->bootstrap));
  if (c->initAbort.load()) {
    VWARN("rank %d: communicator initialisation aborted", c->rank);
    return ncclRemoteError;
  }
  const int n = c->nRanks;
  const auto rings = ring_orders(n);
  const int nRings = (int)rings.size();
  // Channel count: NCCL_NCHANNELS total, else VCCL_CHANNELS_PER_RING x rings,
  // by default from a link-bound model, within VCCL's
  // MAXCHANNELS of 64 (device.h:62) so that VCCL can run the same geometry:
  //   channels per ring = ceil(H * L / (k * R)), at most 64 / rings in all,
  // L = 76.8 GB/s per xGMI link and direction (MI355X spec), k = rings
  // sharing an arc (2 for the 4-GPU set of all 6 Hamiltonian cycles, else 1),
  // R = 40 GB/s, the per-channel rate of the ring step shapes that read the
  // own input from HBM (tools/step_probe, profiles/r03l: 36-44 GB/s at 96
  // concurrent channels), H = 8 headroom for remote-store latency that no
  // single-GPU run can measure (a channel then carries <= 1/8 of its local
  // rate at link peak).  2 GPUs: 16; 3: 2 x 16; 4: 6 x 8 = 48; 5, 6: 4 x 16
  // = 64; 7: 6 x 10 = 60; 8: 7 x 9 = 63.  The shared-GPU rehearsals, which
  // are bound by CUs rather than links, set their counts with the knobs.
  const int arcShare = n == 4 ? 2 : 1;
  const int perRingModel = (int)((8 * 768 + 10 * 40 * arcShare - 1) / (10 * 40 * arcShare));  // ceil(8*76.8/(40k))
  int perRing = (int)param_int("CHANNELS_PER_RING",
                               std::max(1, std::min(perRingModel, kVcclMaxChannels / nRings)));
  int nch = (int)param_int("NCHANNELS", (int64_t)perRing * nRings);
  // minCTAs / maxCTAs bound the channel count (graph/connect.cc:486-490), and
  // so do NCCL_MIN_NCHANNELS / NCCL_MAX_NCHANNELS (legacy MIN_NRINGS /
  // MAX_NRINGS, connect.cc:326-360)
  nch = std::max(c->minCTAs, std::min(nch, c->maxCTAs));
  int64_t minNch = param_int("MIN_NRINGS", -2), maxNch = param_int("MAX_NRINGS", -2);
  if (param_int("MIN_NCHANNELS", -2) != -2) minNch = param_int("MIN_NCHANNELS", -2);
  if (param_int("MAX_NCHANNELS", -2) != -2) maxNch = param_int("MAX_NCHANNELS", -2);
  if (maxNch != -2) nch = std::min<int64_t>(nch, std::max<int64_t>(1, maxNch));
  if (minNch > 0) nch = std::max<int64_t>(nch, minNch);
  nch = std::max(1, std::min(nch, kMaxChannels));
  c->nChannels = n > 1 ? nch : 0;
  // Step = VCCL's FIFO step: NCCL_BUFFSIZE / NCCL_STEPS (init.cc:619-633,
  // 4 MiB -> 512 KiB), or VCCL_SLOT_BYTES directly.  It sets VCCL's
  // partition and ring chunk (4 steps, cbd_schedule), hence the fold order.
  // The FIFO slot (the unit a chunk crosses the FIFO in, one flag hand-off
  // each) is the step unless VCCL_SLICE_BYTES sets it apart without touching
  // the fold order.  A chunk may span at most kSteps / 2 slots: a recv-send
  // step needs free slots while its successor still holds the previous
  // step's (the reference's chunkSteps 4 of NCCL_STEPS 8); 8 slots of 256 KiB
  // for a 2 MiB chunk deadlock the n = 2 all-reduce (profiles/r03n).
  const int64_t buffSize = param_int("BUFFSIZE", -2);
  c->stepBytes = (int)param_int("SLOT_BYTES", buffSize > 0 ? buffSize / kSteps : 512 << 10);
  if (c->stepBytes < 4096 || c->stepBytes % 4096 || c->stepBytes > (64 << 20)) {
    VWARN("slot size (NCCL_BUFFSIZE / 8 or VCCL_SLOT_BYTES) must be a multiple of 4096 up to "
          "64 MiB, using 524288");
    c->stepBytes = 512 << 10;
  }
  c->slotBytes = (int)param_int("SLICE_BYTES", c->stepBytes);
  if (c->slotBytes < 4096 || c->slotBytes % 4096 || c->slotBytes > (64 << 20) ||
      (int64_t)c->slotBytes * (kSteps / 2) < (int64_t)c->stepBytes * 4) {
    VWARN("VCCL_SLICE_BYTES must be a multiple of 4096 up to 64 MiB and hold a ring chunk (4 steps of %d B) "
          "in %d slots, using the step", c->stepBytes, kSteps / 2);
    c->slotBytes = c->stepBytes;
  }
  NCCLCHECK(algo_proto_select(getenv("NCCL_ALGO"), getenv("NCCL_PROTO"), &c->algoForce, &c->algoAllowed));
  // Threads per ring channel (NCCL_NTHREADS, tuning.cc:198-200): 256 or 512
  // (the ring kernel's launch bound, ring_launch.hpp kRingMaxThreads).
  c->nThreads = (int)param_int("NTHREADS", kRingMaxThreads);
  if (c->nThreads != 256 && c->nThreads != 512) {
    if (c->nThreads != kRingMaxThreads)
      VINFO("NCCL_NTHREADS=%d not supported by the ring kernel, using %d", c->nThreads, kRingMaxThreads);
    c->nThreads = kRingMaxThreads;
  }

  HIPCHECK(hipHostMalloc((void**)&c->abortFlag, sizeof(int), hipHostMallocMapped));
  HIPCHECK(hipHostMalloc((void**)&c->errorFlag, sizeof(int), hipHostMallocMapped));
  *c->abortFlag = 0;
  *c->errorFlag = 0;
  // Ordering events (stream_order / stream_mark): only ever waited on by
  // other streams of this device, never by the host.  VCCL_EVENT_FENCE: 0 =
  // HIP's default system-scope release when the event is recorded, 1 =
  // device-scope release (hipEventReleaseToDevice), 2 = no system fence
  // (hipEventDisableSystemFence).
  const int64_t evMode = param_int("EVENT_FENCE", 0);
  const unsigned evFlags = hipEventDisableTiming | (evMode == 1   ? hipEventReleaseToDevice
                                                    : evMode == 2 ? hipEventDisableSystemFence
                                                                  : 0u);
  HIPCHECK(hipEventCreateWithFlags(&c->lastLaunch, evFlags));
  HIPCHECK(hipEventCreateWithFlags(&c->joinEvent, evFlags));
  c->caps.resize(ncclComm::kMaxCaptures);
  for (auto& cap : c->caps) HIPCHECK(hipEventCreateWithFlags(&cap.ev, evFlags));

  PeerMap me{};
  me.pid = (int)getpid();
  me.device = c->device;
  me.hostHash = host_hash();
  {
    int dom = 0, bus = 0, dev = 0;
    HIPCHECK(hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, c->device));
    HIPCHECK(hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, c->device));
    HIPCHECK(hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, c->device));
    me.busId = ((int64_t)dom << 16) | (bus << 8) | dev;
    int cus = 0;
    HIPCHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
    me.cuCount = (uint16_t)std::max(1, std::min(cus, 65535));
  }
  if (n > 1) {
    const size_t fifoBytes = (size_t)c->nChannels * kSteps * slot_stride(c->slotBytes);
    const size_t flagBytes = (size_t)c->nChannels * 2 * kFlagStride;
    VINFO("rank %d: alloc fifo %zu B", c->rank, fifoBytes);
    NCCLCHECK(alloc_uncached((void**)&c->fifoBuf, fifoBytes));
    NCCLCHECK(alloc_uncached((void**)&c->flagBuf, flagBytes));
    HIPCHECK(hipMemset(c->flagBuf, 0, flagBytes));
    HIPCHECK(hipIpcGetMemHandle(&me.fifoHandle, c->fifoBuf));
    HIPCHECK(hipIpcGetMemHandle(&me.flagHandle, c->flagBuf));
    me.fifoPtr = c->fifoBuf;
    me.flagPtr = c->flagBuf;
    // LL buffers for the one-shot small-bucket all-reduce.
    // LL vs direct crossover (profiles/r01_sweep_algos_*.log): LL pays one
    // hop but moves 2(n-1)x the bucket per rank, the direct path two hops
    // and 2(n-1)/n x; LL wins up to ~64 KiB (2 ranks) / ~128 KiB (more).
    c->llMaxBytes = (size_t)param_int("LL_THRESHOLD", n <= 2 ? (64 << 10) : (128 << 10));
    c->llMaxBytes = (c->llMaxBytes + 7) / 8 * 8;
    if (c->llMaxBytes > 0) {
      // Slot capacity: the single-call threshold, or more for group
      // aggregation (VCCL_LL_GROUP_BYTES): a group's run of small all-reduces
      // fills one slot even when their sum is above the single-call
      // threshold — one LL launch still beats one launch per bucket there.
      const int64_t groupBytes = std::max<int64_t>(param_int("LL_GROUP_BYTES", 1 << 20), 0);
      c->llLines = (int)((std::max<int64_t>((int64_t)c->llMaxBytes, groupBytes) + 7) / 8);
      const size_t llBytes = (size_t)2 * n * c->llLines * 16;
      NCCLCHECK(alloc_uncached((void**)&c->llBuf, llBytes));
      HIPCHECK(hipMemset(c->llBuf, 0, llBytes));
      HIPCHECK(hipIpcGetMemHandle(&me.llHandle, c->llBuf));
      me.llPtr = c->llBuf;
    }
    // Inbox of the direct collectives (direct.hpp): 2 phases x n regions of
    // one shard of a VCCL_DIRECT_CHUNK_BYTES chunk each, plus the epoch
    // flags.  Larger buckets stream through the inbox chunk by chunk.
    // Two-shot direct all-reduce up to VCCL_DIRECT_THRESHOLD (8 MiB from 4
    // ranks), the SIMPLE ring above: the ring, with VCCL's own partition, is
    // the north-star path and keeps VCCL's fold order for large buckets; the
    // direct path's two hops (vs 2(n-1)) matter where the per-hop latency
    // does, i.e. small and mid buckets at n >= 4 (profiles/r02e/lat_n4.log,
    // lat_n8.log).  Above 8 MiB the ring's continuous pipeline wins (4 ranks:
    // 16 MiB 111 vs 121 us, 64 MiB 330 vs 504 us, profiles/r03g/lat_n4.log).
    // At n = 2 the ring IS two hops and its channels beat the direct path at
    // every size above LL (profiles/r02/lat_n2.log, r03r: 1 GiB ring 655 vs
    // direct ~220 GB/s).
    c->directMaxBytes = n <= kDirectMaxRanks
                            ? (size_t)param_int("DIRECT_THRESHOLD", n >= 4 ? (int64_t)8 << 20 : 0)
                            : 0;
    c->directMaxBlocks = (int)std::max<int64_t>(
        1, std::min<int64_t>(param_int("DIRECT_MAX_BLOCKS", 64), kDirectMaxBlocks));
    // Reduce-scatter / all-gather (the whole bucket, n blocks): one-hop LL
    // while one rank's block fits a slot and the bucket is at most n x the
    // all-reduce LL threshold (each rank sends 2(n-1)/n x the bucket as LL
    // lines, vs 2(n-1) x for the LL all-reduce), the one-hop direct path up
    // to VCCL_DIRECT_RSAG_THRESHOLD, the SIMPLE ring above.
    c->llRsAgMaxBytes = n <= kOrderMaxRanks && c->llMaxBytes > 0
                            ? (size_t)param_int("LL_RSAG_THRESHOLD", (int64_t)n * c->llMaxBytes)
                            : 0;
    // (The one-hop path saves n-2 hops over the ring: nothing at n = 2, and
    // the 2-rank rehearsal has the ring ahead at 1-8 MiB, profiles/r02h; at
    // n = 8 the one-hop paths lead at <= 1 MiB, profiles/r02e/lat_n8.log.)
    c->directRsAgMaxBytes =
        n <= kDirectMaxRanks
            ? (size_t)param_int("DIRECT_RSAG_THRESHOLD", n >= 4 ? (int64_t)8 << 20 : 0) : 0;
    // The inbox exists whenever the mesh allows the direct path, so that
    // NCCL_ALGO=Direct can take any bucket even where no size defaults to it.
    if (n <= kDirectMaxRanks) {
      const int64_t chunk = std::max<int64_t>(param_int("DIRECT_CHUNK_BYTES", 16 << 20), 64 << 10);
      c->dRegionBytes = (chunk + n - 1) / n / 256 * 256 + 256;
      const size_t bytes = (size_t)kDirectInboxRegions * n * c->dRegionBytes;
      NCCLCHECK(alloc_uncached((void**)&c->dBuf, bytes));
      NCCLCHECK(alloc_uncached((void**)&c->dFlags, kDirectFlagBytes));
      HIPCHECK(hipMemset(c->dFlags, 0, kDirectFlagBytes));
      HIPCHECK(hipIpcGetMemHandle(&me.dBufHandle, c->dBuf));
      HIPCHECK(hipIpcGetMemHandle(&me.dFlagHandle, c->dFlags));
      me.dBufPtr = c->dBuf;
      me.dFlagPtr = c->dFlags;
    } else {
      c->directMaxBytes = c->directRsAgMaxBytes = 0;
    }
  }
  if (n > 1) {
    // LL128 ring buffers: with NCCL_PROTO=LL128, or VCCL_LL128=1 (the
    // automatic window VCCL_LL128_MIN..MAX, default 64 KiB - 1 MiB, inside
    // the range VCCL's tuner gives LL128, enqueue.cc:2032).  VCCL's LL128 step
    // (NCCL_LL128_BUFFSIZE / 8, default 120 x 640 x 8 x 8 B / 8 = 614,400 B)
    // carries 15/16 of it as data, rounded to the 1,920 B grain: 576,000 B per
    // chunk; the slot holds that many data bytes in lines of kLL128LineBytes
    // (600 rounds of 1 KiB with the default 128-byte line).
    // (VCCL_LL128_ALLOC=1: the buffers only — vcclCommSetAlgo may pick the
    // LL128 ring per call, the automatic choice is unchanged)
    // NCCL_PROTO without SIMPLE but with LL128 (e.g. "LL,LL128"): the LL128
    // ring carries every call LL does not
    const bool ll128Only = (c->algoAllowed & kAllowLL128) && !(c->algoAllowed & kAllowSimple);
    const bool want = c->algoForce == 4 || ll128Only || param_int("LL128", 0) != 0 ||
                      param_int("LL128_ALLOC", 0) != 0;
    if (want) {
      c->ll128StepBytes = std::max<int64_t>(param_int("LL128_BUFFSIZE", 120 * 640 * kSteps * 8) / kSteps, 1920 * 16);
      c->ll128Threads = (int)std::max<int64_t>(param_int("LL128_NTHREADS", 640), 64);
      const int64_t chunk = c->ll128StepBytes / 16 * 15 / 1920 * 1920;
      c->ll128SlotBytes = (chunk + kLL128RoundData - 1) / kLL128RoundData * kLL128RoundWire;
      const size_t bytes = (size_t)c->nChannels * kSteps * c->ll128SlotBytes;
      NCCLCHECK(alloc_uncached((void**)&c->ll128Buf, bytes));
      HIPCHECK(hipMemset(c->ll128Buf, 0, bytes));
      HIPCHECK(hipIpcGetMemHandle(&me.ll128Handle, c->ll128Buf));
      me.ll128Ptr = c->ll128Buf;
      if (ll128Only) {
        c->ll128MinBytes = 0;
        c->ll128MaxBytes = ~(size_t)0;
      } else if (param_int("LL128", 0) != 0 && (c->algoAllowed & kAllowLL128)) {
        c->ll128MinBytes = (size_t)param_int("LL128_MIN", 64 << 10);
        // 1 MiB: the rehearsals have the LL128 ring ahead of the SIMPLE ring
        // up to 256 KiB - 1 MiB and behind at 8 MiB, inside
        // VCCL's own 64 KiB - 8 MiB LL128 range (enqueue.cc:2032)
        c->ll128MaxBytes = (size_t)param_int("LL128_MAX", 1 << 20);
      }
    }
  }
  // paths NCCL_ALGO / NCCL_PROTO exclude drop out of the automatic choice
  if (!(c->algoAllowed & kAllowLL)) c->llMaxBytes = 0;
  if (!(c->algoAllowed & kAllowLLRsAg)) c->llRsAgMaxBytes = 0;
  if (!(c->algoAllowed & kAllowDirect)) c->directMaxBytes = c->directRsAgMaxBytes = 0;
  if (n > 1) NCCLCHECK(net_listen(c, &me));
  VINFO("rank %d: exchange peer info", c->rank);
  c->peers.assign(n, PeerMap{});
  c->peers[c->rank] = me;
  NCCLCHECK(bootstrap_allgather(c->bootstrap, c->peers.data(), sizeof(PeerMap)));
  // Transport per peer (the reference's selectTransport, transport.cc:
  // 37-68, reduced to two): xGMI peer memory within the node, the net proxy
  // (proxy.cc) to a peer on another node — or to every peer with
  // VCCL_NET_FORCE=1, which runs the inter-node path on one node.
  const bool netForce = param_int("NET_FORCE", 0) != 0;
  std::vector<char> netPeer(n, 0);
  bool anyNet = false;
  for (int r = 0; r < n; r++) {
    if (r == c->rank) continue;
    netPeer[r] = netForce || c->peers[r].hostHash != me.hostHash;
    anyNet |= netPeer[r] != 0;
  }
  if (anyNet) {
    // LL and the two-shot direct path need every peer's memory mapped
    // (full xGMI mesh): all-reduce takes the ring.  Net channels move
    // through the proxy, a few are enough (NCCL's net defaults use 2-4).
    c->llMaxBytes = c->llRsAgMaxBytes = 0;
    c->directMaxBytes = c->directRsAgMaxBytes = 0;
    c->ll128MinBytes = c->ll128MaxBytes = 0;
    if (c->algoForce == 4) c->algoForce = 1;  // LL128 lines need the xGMI mesh: SIMPLE
    // ... so no LL128 FIFO is mapped: drop the local one too, so that neither
    // the automatic choice nor vcclCommSetAlgo(LL128) can pick a ring whose
    // channels carry no LL128 slots
    if (c->ll128Buf) (void)hipFree(c->ll128Buf);
    c->ll128Buf = nullptr;
    c->nChannels = std::max(1, std::min(c->nChannels, (int)param_int("NET_NCHANNELS", 8)));
    VINFO("rank %d: inter-node ring through the net proxy, %d channels", c->rank, c->nChannels);
  }
  // init.cc:732-735: two ranks on one GPU is invalid usage.  The escape hatch
  // exists for protocol tests on a 1-GPU machine only.  Checked over every
  // pair, so every rank fails together.
  if (!param_int("ALLOW_SHARED_DEVICE", 0) && !netForce) {
    for (int q = 0; q < n; q++)
      for (int r = q + 1; r < n; r++)
        if (c->peers[r].hostHash == c->peers[q].hostHash && c->peers[r].busId == c->peers[q].busId) {
          VWARN("Duplicate GPU detected : rank %d and rank %d both on device %lx", q, r,
                (long)c->peers[q].busId);
          return ncclInvalidUsage;
        }
  }
  {
    // Ranks sharing a GPU (VCCL_ALLOW_SHARED_DEVICE: rehearsals on fewer GPUs
    // than ranks) spin on each other, so all their ring workgroups must be
    // resident at once: one 512-thread ring workgroup fills a CU (176-232
    // VGPRs), so k ranks on a device get at most 7/8 of its CUs / k channels
    // (e.g. 4 ranks on 256 CUs: 56), the rest left to the other kernels.
    // Computed from the shared peer table, so every rank picks the same
    // count (the partition depends on it); the FIFO was sized for the
    // uncapped count, its tail stays unused.  Real one-rank-per-GPU runs are
    // untouched.
    int share = 1, cus = 1 << 30;
    for (int q = 0; q < n; q++) {
      int k = 0;
      for (int r = 0; r < n; r++)
        k += c->peers[r].hostHash == c->peers[q].hostHash && c->peers[r].busId == c->peers[q].busId;
      share = std::max(share, k);
      cus = std::min(cus, (int)c->peers[q].cuCount);
    }
    if (share > 1) {
      const int cap = std::max(1, cus * 7 / 8 / share);
      c->shareBlockCap = cap;  // the LL and direct grids too (enqueue.cc)
      c->directMaxBlocks = std::min(c->directMaxBlocks, cap);
      if (c->nChannels > cap) {
        VINFO("rank %d: %d ranks share a GPU of %d CUs: %d -> %d ring channels", c->rank, share, cus,
              c->nChannels, cap);
        c->nChannels = cap;
      }
    }
  }
  {
    // Ranks of this comm that share ONE device inside ONE process (allowed
    // only through VCCL_ALLOW_SHARED_DEVICE) spin on each other, so their
    // kernels must be co-resident.  HIP gives a process GPU_MAX_HW_QUEUES
    // hardware queues (4 by default) and deals streams to them round-robin,
    // one of them taken by the process's first (null / runtime) stream: with
    // more sharing ranks than the remaining queues, two ranks' kernels
    // serialise on one queue and every peer spins until the timeout
    // (profiles/r01_diag_protocol.log).  Refuse that configuration up front.
    // Every rank evaluates every (process, device) group from the same peer
    // table, so all ranks fail together (none is left waiting at the final
    // barrier).
    const char* hq = getenv("GPU_MAX_HW_QUEUES");
    const int hwQueues = hq && atoi(hq) > 0 ? atoi(hq) : 4;
    for (int q = 0; q < n; q++) {
      int sameDev = 0;
      for (int r = 0; r < n; r++)
        sameDev += c->peers[r].pid == c->peers[q].pid &&
                   c->peers[r].hostHash == c->peers[q].hostHash &&
                   c->peers[r].busId == c->peers[q].busId;
      if (sameDev > 1 && sameDev > hwQueues - 1) {
        VWARN("%d ranks of this communicator share device %lx in one process, but only %d of the "
              "process's %d hardware queues can keep their kernels co-resident",
              sameDev, (long)c->peers[q].busId, hwQueues - 1, hwQueues);
        return ncclInvalidUsage;
      }
    }
  }

  DevComm dc{};
  dc.rank = c->rank;
  dc.nRanks = n;
  dc.nChannels = c->nChannels;
  dc.slotBytes = c->slotBytes;
  HIPCHECK(hipHostGetDevicePointer((void**)&dc.abortFlag, (void*)c->abortFlag, 0));
  HIPCHECK(hipHostGetDevicePointer((void**)&dc.errorFlag, c->errorFlag, 0));
  dc.spinTimeoutTicks = (uint64_t)param_int("SPIN_TIMEOUT_S", 60) * 100000000ull;
  // FIFO payload moves with sc0 sc1 write-through accesses, so no L2
  // writeback / invalidate is needed per slot; VCCL_FENCES=1 adds the
  // system-scope release/acquire fences back (A/B and safety valve).
  dc.useFences = (int)param_int("FENCES", 0);
  if (anyNet) dc.useFences = 1;  // slots and flags in host memory: full system-scope fences
  dc.pollMode = (int)param_int("POLL_MODE", 0);
  // The per-wave SIMPLE ring (ring_kernels.hip PART 4) for this comm's
  // launches (VCCL_RING_WAVE=1 or vcclCommSetRingWave; default off: no gain
  // on a shared GPU).  Inside it, slots below
  // VCCL_RING_WAVE_MIN (a full default slot) still take the workgroup
  // hand-off (latency-bound slots, profiles/r05k); 0 = always per wave.
  c->ringWave = param_int("RING_WAVE", 0) != 0;
  dc.ringWaveMin = std::max<int64_t>(0, param_int("RING_WAVE_MIN", 512 << 10));
  // Opt-in slot timeline of the SIMPLE ring (vcclCommRingTrace)
  c->ringTraceCap = n > 1 ? (int)std::max<int64_t>(0, std::min<int64_t>(param_int("RING_TRACE", 0), 1 << 16)) : 0;
  if (c->ringTraceCap > 0) {
    const size_t tb = (size_t)c->nChannels * c->ringTraceCap * sizeof(RingTraceRec);
    HIPCHECK(hipMalloc((void**)&c->ringTrace, tb));
    HIPCHECK(hipMemset(c->ringTrace, 0, tb));
  }
  dc.trace = c->ringTrace;
  dc.traceCap = c->ringTraceCap;
  // reduce-scatter fold order of this rank on each ring (ring_types.hpp)
  dc.nRings = std::min(nRings, kOrderMaxRings);
  for (int k = 0; k < dc.nRings && n <= kOrderMaxRanks; k++) {
    const auto& ring = rings[k];
    const int pos = (int)(std::find(ring.begin(), ring.end(), c->rank) - ring.begin());
    for (int j = 0; j < n; j++) dc.rsOrder[k][j] = (int8_t)ring[(pos + 1 + j) % n];
    for (int j = 0; j < n; j++) dc.ringAt[k][j] = (int8_t)ring[j];
  }
  // LL chain (DevComm::llChain): VCCL_LL_CHAIN="r0,r1,..." (root first), a
  // permutation of the ranks, else the identity.  Every rank must pass the
  // same order.
  for (int j = 0; j < n && j < kOrderMaxRanks; j++) dc.llChain[j] = (int8_t)j;
  if (const char* chainEnv = getenv("VCCL_LL_CHAIN"); chainEnv && *chainEnv && n <= kOrderMaxRanks) {
    std::vector<int> order;
    for (const char* q = chainEnv; *q;) {
      char* end = nullptr;
      const long v = strtol(q, &end, 10);
      if (end == q) break;
      order.push_back((int)v);
      q = *end == ',' ? end + 1 : end;
    }
    std::vector<int> seen(n, 0);
    bool okChain = (int)order.size() == n;
    for (int v : order) okChain = okChain && v >= 0 && v < n && !seen[v]++;
    if (!okChain) {
      VWARN("VCCL_LL_CHAIN=%s is not a permutation of the %d ranks", chainEnv, n);
      return ncclInvalidUsage;
    }
    for (int j = 0; j < n; j++) dc.llChain[j] = (int8_t)order[j];
  }
  HIPCHECK(hipMalloc((void**)&c->devComm, sizeof(DevComm)));
  HIPCHECK(hipMemcpy(c->devComm, &dc, sizeof(dc), hipMemcpyHostToDevice));

  VINFO("rank %d: map peers", c->rank);
  if (n > 1) {
    std::vector<char*> fifoOf(n), flagOf(n);
    for (int r = 0; r < n; r++) {
      if (r == c->rank) {
        fifoOf[r] = c->fifoBuf;
        flagOf[r] = c->flagBuf;
        continue;
      }
      if (netPeer[r]) continue;  // reached through the net proxy
      NCCLCHECK(map_peer(c, me, c->peers[r], kMapFifo, &fifoOf[r]));
      NCCLCHECK(map_peer(c, me, c->peers[r], kMapFlag, &flagOf[r]));
    }
    if (c->dBuf && !anyNet) {
      DirectPeers dp{};
      for (int r = 0; r < n; r++) {
        if (r == c->rank) {
          dp.buf[r] = c->dBuf;
          dp.flags[r] = c->dFlags;
          continue;
        }
        NCCLCHECK(map_peer(c, me, c->peers[r], kMapDirect, &dp.buf[r]));
        NCCLCHECK(map_peer(c, me, c->peers[r], kMapDirectFlag, &dp.flags[r]));
      }
      HIPCHECK(hipMalloc((void**)&c->dPeers, sizeof(DirectPeers)));
      HIPCHECK(hipMemcpy(c->dPeers, &dp, sizeof(dp), hipMemcpyHostToDevice));
    }
    c->llPeer.assign(n, nullptr);
    if (c->llBuf && !anyNet) {
      for (int r = 0; r < n; r++) {
        if (r == c->rank) c->llPeer[r] = c->llBuf;
        else NCCLCHECK(map_peer(c, me, c->peers[r], kMapLL, &c->llPeer[r]));
      }
    }
    std::vector<char*> ll128Of(n, nullptr);
    if (c->ll128Buf && !anyNet) {
      for (int r = 0; r < n; r++) {
        if (r == c->rank) ll128Of[r] = c->ll128Buf;
        else NCCLCHECK(map_peer(c, me, c->peers[r], kMapLL128, &ll128Of[r]));
      }
    }
    std::vector<DevChannel> chans(c->nChannels);
    const size_t fifoPerCh = (size_t)kSteps * slot_stride(c->slotBytes);
    const size_t ll128PerCh = (size_t)kSteps * c->ll128SlotBytes;
    for (int ch = 0; ch < c->nChannels; ch++) {
      const auto& ring = rings[ch % nRings];
      int pos = (int)(std::find(ring.begin(), ring.end(), c->rank) - ring.begin());
      int next = ring[(pos + 1) % n], prev = ring[(pos + n - 1) % n];
      DevChannel& d = chans[ch];
      memset(&d, 0, sizeof(d));
      for (int k = 0; k < n; k++) d.ringRanks[k] = ring[(pos + k) % n];
      d.ringPos = pos;
      auto flag = [&](int r, int which) {
        return (uint64_t*)(flagOf[r] + ((size_t)ch * 2 + which) * kFlagStride);
      };
      d.recvFifo = c->fifoBuf + ch * fifoPerCh;
      d.recvTail = flag(c->rank, 0);
      d.prevSendHead = flag(prev, 1);
      d.sendFifo = fifoOf[next] + ch * fifoPerCh;
      d.nextRecvTail = flag(next, 0);
      d.sendHead = flag(c->rank, 1);
      d.recvStep = d.sendStep = 0;
      d.sendSizes = nullptr;
      d.recvSizes = nullptr;
      d.ll128Recv = ll128Of[c->rank] ? ll128Of[c->rank] + ch * ll128PerCh : nullptr;
      d.ll128Send = ll128Of[next] ? ll128Of[next] + ch * ll128PerCh : nullptr;
      // a net end's pointers are set by net_connect below
      if (netPeer[prev]) {
        d.recvFifo = nullptr;
        d.recvTail = d.prevSendHead = nullptr;
      }
      if (netPeer[next]) {
        d.sendFifo = nullptr;
        d.nextRecvTail = d.sendHead = nullptr;
      }
    }
    if (anyNet) NCCLCHECK(net_connect(c, rings, chans, netPeer));
    else net_stop(c);  // close the unused listener
    HIPCHECK(hipMalloc((void**)&c->devChannels, sizeof(DevChannel) * c->nChannels));
    HIPCHECK(hipMemcpy(c->devChannels, chans.data(), sizeof(DevChannel) * c->nChannels,
                       hipMemcpyHostToDevice));
  }
  VINFO("rank %d: final barrier", c->rank);
  NCCLCHECK(bootstrap_barrier(c->bootstrap));
  VINFO("comm %p rank %d/%d dev %d: %d channels x %d threads, step %d B, FIFO slot %d B", (void*)c, c->rank,
        n, c->device, c->nChannels, c->nThreads, c->stepBytes, c->slotBytes);
  VINFO("rank %d: thresholds LL %zu, LL RS/AG %zu, direct %zu, direct RS/AG %zu, LL128 [%zu, %zu]%s, "
        "algo force %d", c->rank, c->llMaxBytes, c->llRsAgMaxBytes, c->directMaxBytes,
        c->directRsAgMaxBytes, c->ll128MinBytes, c->ll128MaxBytes, c->ll128Buf ? " (buffers)" : "",
        c->algoForce);
  return ncclSuccess;
}

// ncclConfig_t + NCCL_* environment -> CTA bounds and blocking mode
// (envConfigOverride, init.cc:1472-1545: env wins, non-positive values are
// ignored, both capped at MAXCHANNELS, min > max sets min = max).
static ncclResult_t apply_config(ncclComm* c, const ncclConfig_t* config) {
  int minC = NCCL_CONFIG_UNDEF_INT, maxC = NCCL_CONFIG_UNDEF_INT;
  int blocking = NCCL_CONFIG_UNDEF_INT;
  if (config) {
    if (config->magic != 0xcafebeef) {
      VWARN("ncclCommInitRankConfig: config not initialised with NCCL_CONFIG_INITIALIZER");
      return ncclInvalidArgument;
    }
    if ((config->minCTAs != NCCL_CONFIG_UNDEF_INT && config->minCTAs <= 0) ||
        (config->maxCTAs != NCCL_CONFIG_UNDEF_INT && config->maxCTAs <= 0) ||
        (config->blocking != NCCL_CONFIG_UNDEF_INT && config->blocking != 0 &&
         config->blocking != 1)) {
      VWARN("ncclCommInitRankConfig: invalid config (blocking %d, minCTAs %d, maxCTAs %d)",
            config->blocking, config->minCTAs, config->maxCTAs);
      return ncclInvalidArgument;  // init.cc:1603-1612
    }
    minC = config->minCTAs;
    maxC = config->maxCTAs;
    blocking = config->blocking;
  }
  const int64_t envMin = param_int("MIN_CTAS", NCCL_CONFIG_UNDEF_INT);
  const int64_t envMax = param_int("MAX_CTAS", NCCL_CONFIG_UNDEF_INT);
  const int64_t envBlocking = param_int("COMM_BLOCKING", NCCL_CONFIG_UNDEF_INT);
  if (envMin != NCCL_CONFIG_UNDEF_INT && envMin > 0) minC = (int)envMin;
  if (envMax != NCCL_CONFIG_UNDEF_INT && envMax > 0) maxC = (int)envMax;
  if (envBlocking == 0 || envBlocking == 1) blocking = (int)envBlocking;
  c->minCTAs = minC == NCCL_CONFIG_UNDEF_INT ? 1 : std::min(minC, kMaxChannels);
  c->maxCTAs = maxC == NCCL_CONFIG_UNDEF_INT ? kMaxChannels : std::min(maxC, kMaxChannels);
  if (c->minCTAs > c->maxCTAs) c->minCTAs = c->maxCTAs;
  c->blocking = blocking == 0 ? 0 : 1;
  return ncclSuccess;
}

ncclResult_t comm_init_rank(ncclComm_t* out, int nranks, const ncclUniqueId* id, int rank,
                            int device, const ncclConfig_t* config) {
  if (!out) return ncclInvalidArgument;
  *out = nullptr;
  if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) {
    VWARN("ncclCommInitRank : invalid rank %d / nranks %d", rank, nranks);
    return ncclInvalidArgument;
  }
  auto* c = new ncclComm();
  c->magic = kCommMagic;
  c->rank = rank;
  c->nRanks = nranks;
  c->device = device;
  c->userOpFreeHead = 0;
  if (ncclResult_t cr = apply_config(c, config); cr != ncclSuccess) {
    c->magic = 0;
    delete c;
    return cr;
  }
  if (!c->blocking) {
    // Non-blocking (group.cc:553-576): the handle now, the initialisation on
    // a thread of its own; ncclCommGetAsyncError says when it has ended.  On
    // failure the comm keeps no resources and only destroy / abort accept it.
    c->initPending.store(true, std::memory_order_relaxed);
    c->asyncError.store(ncclInProgress, std::memory_order_relaxed);
    const ncclUniqueId idCopy = *id;
    *out = c;
    c->initThread = std::thread([c, idCopy]() {
      (void)hipSetDevice(c->device);
      const ncclResult_t r = init_rank(c, &idCopy);
      // on failure the bootstrap socket stays open until destroy / abort
      // closes it: an abort may still be shutting it down (initFd)
      if (r != ncclSuccess) free_resources(c);
      c->initResult = r;
      c->asyncError.store(r, std::memory_order_release);
      c->initPending.store(false, std::memory_order_release);
    });
    return ncclInProgress;
  }
  ncclResult_t r = init_rank(c, id);
  if (r != ncclSuccess) {
    free_resources(c);
    bootstrap_close(c->bootstrap);
    c->magic = 0;
    delete c;
    return r;
  }
  *out = c;
  return ncclSuccess;
}

// Wait for THIS comm's launches only — its ordering event, which every eager
// launch of the comm records (bound to the kernel's completion, or a marker
// behind it; enqueue.cc stream_mark), and the launches of one comm are
// serialised through it, so the last one done means all done.  The
// reference's commReclaim likewise waits on the comm's own strong stream
// (src/init.cc:2079-2111), never the whole device: a hipDeviceSynchronize
// here would also wait for other comms' kernels (possibly stuck on a lost
// peer of their own) and for unrelated user work.  timeoutS < 0: no bound.
// Captured launches belong to their graphs (the caller's to wait for).
static bool wait_own_launches(ncclComm* c, double timeoutS) {
  if (!c->hasLastLaunch || !c->lastLaunch) return true;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    // an unmarked launch (VCCL_DEBUG_NO_MARK without a bound stop event) is
    // done once its stream has drained
    const hipError_t e = c->lastUnmarked ? hipStreamQuery(c->lastStream) : hipEventQuery(c->lastLaunch);
    if (e != hipErrorNotReady) return true;  // done (or the event is unusable: nothing to wait for)
    if (timeoutS >= 0 &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeoutS)
      return false;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

ncclResult_t comm_wait_own_launches(ncclComm* c) { return wait_own_launches(c, -1) ? ncclSuccess : ncclInternalError; }

ncclResult_t comm_destroy(ncclComm* c, bool abort) {
  int old = -1;
  (void)hipGetDevice(&old);
  (void)hipSetDevice(c->device);
  // ncclCommAbort (init.cc:2079-2111): raise the abort word every spin of the
  // comm's kernels polls (ring.hpp / ll.hpp / direct.hpp, as checkAbort,
  // primitives.h:142-152), then wait for the comm's own work only.
  if (abort && c->abortFlag) __atomic_store_n((int*)c->abortFlag, 1, __ATOMIC_RELEASE);
  // An aborting kernel leaves within a few hundred spins; one still queued
  // behind other work on its stream will read the abort word when it starts,
  // so after the bound the comm's memory is left allocated (a kernel may
  // still touch it) rather than freed under it.
  const double bound = abort ? (double)param_int("ABORT_WAIT_S", 10) : -1.0;
  const bool drained = wait_own_launches(c, bound);
  // Peers in OTHER processes may still post a last credit into our flags:
  // rendezvous before freeing.  Not after an abort or an error: the peer that
  // failed may never come (the kernels have ended, so no credit is in
  // flight from this side either).  Comms of one process (ncclCommInitAll) are
  // legitimately destroyed one after another by a single thread (as with the
  // reference), so a barrier there would deadlock; their kernels are already
  // complete once their own launches are.
  bool remotePeers = false;
  for (const auto& p : c->peers) remotePeers |= p.pid != (int)getpid();
  const bool failed = c->asyncError.load() != 0 || (c->errorFlag && *(volatile int*)c->errorFlag);
  if (!abort && !failed && remotePeers && c->bootstrap && c->nRanks > 1) (void)bootstrap_barrier(c->bootstrap);
  if (!drained) {
    VWARN("comm %p rank %d: its last launch has not ended %.0f s after the abort; its device memory is left "
          "allocated", (void*)c, c->rank, bound);
    net_stop(c);
  } else {
    free_resources(c);
  }
  bootstrap_close(c->bootstrap);
  c->bootstrap = nullptr;
  c->destroyed = true;
  c->magic = 0;
  if (old >= 0) (void)hipSetDevice(old);
  delete c;
  return ncclSuccess;
}

}  // namespace vccl

using namespace vccl;

#define VCCL_EXPORT extern "C" __attribute__((visibility("default")))
#define VCCL_ALIAS(name) __attribute__((alias(#name), visibility("default")))

// vccl_ext.h: the ring set the library uses for nRanks ranks.
VCCL_EXPORT ncclResult_t vcclRingOrders(int nRanks, int maxRings, int* orders, int* nRings) {
  if (nRanks < 1 || nRanks > kMaxRanks || maxRings < 1 || !orders || !nRings) return ncclInvalidArgument;
  const auto rings = ring_orders(nRanks);
  *nRings = (int)rings.size();
  if ((int)rings.size() > maxRings) return ncclInvalidArgument;
  for (size_t k = 0; k < rings.size(); k++)
    for (int i = 0; i < nRanks; i++) orders[k * nRanks + i] = rings[k][i];
  return ncclSuccess;
}

VCCL_EXPORT ncclResult_t vcclAlgoSelection(const char* algo, const char* proto, int* force, int* allowed) {
  if (!force || !allowed) return ncclInvalidArgument;
  return algo_proto_select(algo, proto, force, allowed);
}

VCCL_EXPORT ncclResult_t ncclGetVersion(int* version) {
  if (!version) return ncclInvalidArgument;
  *version = NCCL_VERSION_CODE;
  return ncclSuccess;
}

VCCL_EXPORT ncclResult_t ncclGetUniqueId(ncclUniqueId* uniqueId) {
  return bootstrap_get_unique_id(uniqueId);
}

VCCL_EXPORT ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId commId,
                                          int rank) {
  int dev = 0;
  HIPCHECK(hipGetDevice(&dev));
  return comm_init_rank(comm, nranks, &commId, rank, dev, nullptr);
}

VCCL_EXPORT ncclResult_t ncclCommInitRankConfig(ncclComm_t* comm, int nranks,
                                                ncclUniqueId commId, int rank,
                                                ncclConfig_t* config) {
  int dev = 0;
  HIPCHECK(hipGetDevice(&dev));
  return comm_init_rank(comm, nranks, &commId, rank, dev, config);
}

// nccl.h.in:178-181: several roots spread the bootstrap of very large jobs;
// one node needs one, so every rank joins the root of commIds[0] (the same
// array on every rank).
VCCL_EXPORT ncclResult_t ncclCommInitRankScalable(ncclComm_t* newcomm, int nranks, int myrank, int nId,
                                                  ncclUniqueId* commIds, ncclConfig_t* config) {
  if (nId < 1 || !commIds) {
    VWARN("ncclCommInitRankScalable: nId %d, commIds %p", nId, (void*)commIds);
    return ncclInvalidArgument;
  }
  int dev = 0;
  HIPCHECK(hipGetDevice(&dev));
  return comm_init_rank(newcomm, nranks, &commIds[0], myrank, dev, config);
}

// nccl.h.in:104-111: device memory for any buffer the library is handed.
VCCL_EXPORT ncclResult_t ncclMemAlloc(void** ptr, size_t size) {
  if (!ptr) return ncclInvalidArgument;
  *ptr = nullptr;
  if (size == 0) return ncclSuccess;
  HIPCHECK(hipMalloc(ptr, size));
  return ncclSuccess;
}
VCCL_EXPORT ncclResult_t ncclMemFree(void* ptr) {
  if (ptr) HIPCHECK(hipFree(ptr));
  return ncclSuccess;
}

// nccl.h.in:208-217: buffer registration enables zero-copy in the reference;
// that is out of scope here and every collective works on
// unregistered buffers, so registration is accepted and does nothing.
VCCL_EXPORT ncclResult_t ncclCommRegister(const ncclComm_t comm, void* buff, size_t, void** handle) {
  NCCLCHECK(comm_check(comm, "ncclCommRegister"));
  if (!handle) return ncclInvalidArgument;
  *handle = buff;
  return ncclSuccess;
}
VCCL_EXPORT ncclResult_t ncclCommDeregister(const ncclComm_t comm, void*) {
  NCCLCHECK(comm_check(comm, "ncclCommDeregister"));
  return ncclSuccess;
}

// nccl.h.in:173-174 (src/init.cc ncclCommSplit): the ranks of `comm` with
// one color form a new communicator, ranked by (key, parent rank); color
// NCCL_SPLIT_NOCOLOR joins none (*newcomm = NULL).  Collective over the
// parent: its bootstrap carries every rank's (color, key), then the new
// roots' ids — the first member of each color hosts its group's root — and
// the members initialise as with ncclCommInitRankConfig on the parent's
// device (config NULL: the parent's CTA bounds).
VCCL_EXPORT ncclResult_t ncclCommSplit(ncclComm_t comm, int color, int key, ncclComm_t* newcomm,
                                       ncclConfig_t* config) {
  if (newcomm) *newcomm = nullptr;
  NCCLCHECK(comm_check(comm, "ncclCommSplit"));
  if (!newcomm) return ncclInvalidArgument;
  if (color < NCCL_SPLIT_NOCOLOR) {
    VWARN("ncclCommSplit: invalid color %d", color);
    return ncclInvalidArgument;
  }
  const int n = comm->nRanks, me = comm->rank;
  struct Entry {
    int color, key;
  };
  std::vector<Entry> ents((size_t)n);
  ents[me] = Entry{color, key};
  if (n > 1) NCCLCHECK(bootstrap_allgather(comm->bootstrap, ents.data(), sizeof(Entry)));
  std::vector<int> members;
  if (color != NCCL_SPLIT_NOCOLOR)
    for (int r = 0; r < n; r++)
      if (ents[r].color == color) members.push_back(r);
  std::stable_sort(members.begin(), members.end(),
                   [&](int a, int b) { return ents[a].key < ents[b].key; });  // ties: parent rank
  std::vector<ncclUniqueId> ids((size_t)n);
  memset(ids.data(), 0, ids.size() * sizeof(ncclUniqueId));
  if (!members.empty() && members[0] == me) NCCLCHECK(bootstrap_get_unique_id(&ids[me]));
  if (n > 1) NCCLCHECK(bootstrap_allgather(comm->bootstrap, ids.data(), sizeof(ncclUniqueId)));
  VINFO("ncclCommSplit: comm %p rank %d color %d key %d -> %zu ranks", (void*)comm, me, color, key,
        members.size());
  if (members.empty()) return ncclSuccess;
  const int newRank = (int)(std::find(members.begin(), members.end(), me) - members.begin());
  int old = -1;
  HIPCHECK(hipGetDevice(&old));
  if (old != comm->device) HIPCHECK(hipSetDevice(comm->device));
  // config NULL: the parent's (copyCommConfig, src/init.cc:2160-2161) — its
  // CTA bounds, so the child gets the parent's channel count
  ncclConfig_t inherit = NCCL_CONFIG_INITIALIZER;
  inherit.minCTAs = comm->minCTAs;
  inherit.maxCTAs = comm->maxCTAs;
  const ncclResult_t r = comm_init_rank(newcomm, (int)members.size(), &ids[members[0]], newRank, comm->device,
                                        config ? config : &inherit);
  if (old != comm->device) (void)hipSetDevice(old);
  return r;
}

VCCL_EXPORT ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist) {
  if (!comms || ndev < 1) return ncclInvalidArgument;
  int ndevices = 0;
  HIPCHECK(hipGetDeviceCount(&ndevices));
  std::vector<int> seen(ndevices, 0);
  for (int i = 0; i < ndev; i++) {
    int d = devlist ? devlist[i] : i;
    if (d < 0 || d >= ndevices) {
      VWARN("ncclCommInitAll : invalid device %d (totalnDev=%d)", d, ndevices);
      return ncclInvalidArgument;
    }
    if (seen[d]++ && !param_int("ALLOW_SHARED_DEVICE", 0)) return ncclInvalidUsage;  // init.cc:1782-1786
  }
  ncclUniqueId id;
  NCCLCHECK(bootstrap_get_unique_id(&id));
  std::vector<ncclResult_t> res(ndev, ncclSuccess);
  std::vector<std::thread> th;
  for (int i = 0; i < ndev; i++) {
    th.emplace_back([&, i] {
      int d = devlist ? devlist[i] : i;
      if (hipSetDevice(d) != hipSuccess) {
        res[i] = ncclUnhandledCudaError;
        return;
      }
      res[i] = comm_init_rank(&comms[i], ndev, &id, i, d, nullptr);
      if (res[i] == ncclInProgress) {  // NCCL_COMM_BLOCKING=0: InitAll still returns initialised comms
        wait_init(comms[i]);
        res[i] = comms[i]->initResult;
      }
    });
  }
  for (auto& t : th) t.join();
  for (int i = 0; i < ndev; i++) {
    if (res[i] != ncclSuccess) {
      for (int j = 0; j < ndev; j++)
        if (comms[j]) comm_destroy(comms[j], true), comms[j] = nullptr;
      return res[i];
    }
  }
  return ncclSuccess;
}

// ncclCommFinalize (init.cc commFinalize): every operation of the comm has
// completed when it returns — its own launches, not the whole device.
VCCL_EXPORT ncclResult_t ncclCommFinalize(ncclComm_t comm) {
  NCCLCHECK(comm_check(comm, "ncclCommFinalize"));
  int old = -1;
  (void)hipGetDevice(&old);
  (void)hipSetDevice(comm->device);
  const ncclResult_t r = comm_wait_own_launches(comm);
  if (old >= 0) (void)hipSetDevice(old);
  return r;
}

VCCL_EXPORT ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (comm == nullptr) return ncclSuccess;  // init.cc: destroying NULL is a no-op
  NCCLCHECK(comm_check(comm, "ncclCommDestroy", true));
  return comm_destroy(comm, false);
}

VCCL_EXPORT ncclResult_t ncclCommAbort(ncclComm_t comm) {
  if (comm == nullptr) return ncclSuccess;
  NCCLCHECK(comm_check_live(comm, "ncclCommAbort"));
  if (comm->initPending.load()) {
    // a non-blocking init still running (init.cc commAbort of an initialising
    // comm): stop it — no more root retries, and the bootstrap socket shut so
    // a wait on peers that never come returns at once
    comm->initAbort.store(true);
    const int fd = comm->initFd.load();
    if (fd >= 0) (void)shutdown(fd, SHUT_RDWR);
  }
  wait_init(comm);  // the init thread ends promptly once told to
  return comm_destroy(comm, true);
}

VCCL_EXPORT const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {  // src/init.cc ncclGetErrorString wording
    case ncclSuccess: return "no error";
    case ncclUnhandledCudaError: return "unhandled cuda error (run with NCCL_DEBUG=INFO for details)";
    case ncclSystemError: return "unhandled system error (run with NCCL_DEBUG=INFO for details)";
    case ncclInternalError: return "internal error - please report this issue to the NCCL developers";
    case ncclInvalidArgument: return "invalid argument (run with NCCL_DEBUG=WARN for details)";
    case ncclInvalidUsage: return "invalid usage (run with NCCL_DEBUG=WARN for details)";
    case ncclRemoteError: return "remote process exited or there was a network error";
    case ncclInProgress: return "NCCL operation in progress";
    default: return "unknown result code";
  }
}

// The comm's device error word as an ncclResult_t (ring_types.hpp): a spin
// that made no progress — a peer stopped — is ncclRemoteError; a net slot
// whose landed byte count is not its step's slice length is caught before
// it is reduced and reported as ncclInternalError.
ncclResult_t vccl::error_word_result(ncclComm* comm) {
  const int w = *(volatile int*)comm->errorFlag;
  if (w == kErrSlotSize) {
    VWARN("rank %d: a net slot landed with a byte count that is not its step's slice length; the call was "
          "stopped before reducing it", comm->rank);
    return ncclInternalError;
  }
  return w ? ncclRemoteError : ncclSuccess;
}

// The text of the last WARN, whatever NCCL_DEBUG filters (debug.cc:29,
// :265-272 ncclLastError; init.cc:2223-2225: comm unused, may be NULL).
VCCL_EXPORT const char* ncclGetLastError(ncclComm_t) { return last_error(); }

VCCL_EXPORT ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError) {
  NCCLCHECK(comm_check_live(comm, "ncclCommGetAsyncError"));
  if (!asyncError) return ncclInvalidArgument;
  if (comm->initPending.load(std::memory_order_acquire)) {  // non-blocking init still running
    *asyncError = ncclInProgress;
    return ncclSuccess;
  }
  wait_init(comm);  // ended: reap its thread
  int e = comm->asyncError.load();
  if (e == 0 && comm->errorFlag && *(volatile int*)comm->errorFlag) {
    e = error_word_result(comm);
    comm->asyncError = e;
  }
  *asyncError = (ncclResult_t)e;
  return ncclSuccess;
}

VCCL_EXPORT ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
  NCCLCHECK(comm_check(comm, "ncclCommCount"));
  if (!count) return ncclInvalidArgument;
  *count = comm->nRanks;
  return ncclSuccess;
}

VCCL_EXPORT ncclResult_t ncclCommCuDevice(const ncclComm_t comm, int* device) {
  NCCLCHECK(comm_check(comm, "ncclCommCuDevice"));
  if (!device) return ncclInvalidArgument;
  *device = comm->device;
  return ncclSuccess;
}

VCCL_EXPORT ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
  NCCLCHECK(comm_check(comm, "ncclCommUserRank"));
  if (!rank) return ncclInvalidArgument;
  *rank = comm->rank;
  return ncclSuccess;
}

// vccl_ext.h: run-time fence toggle and the epoch-wrap test hook.
VCCL_EXPORT ncclResult_t vcclCommSetFences(ncclComm_t comm, int useFences) {
  NCCLCHECK(comm_check(comm, "vcclCommSetFences"));
  if (useFences != 0 && useFences != 1) return ncclInvalidArgument;
  if (comm->nRanks < 2 || !comm->devComm) return ncclSuccess;
  int old = -1;
  (void)hipGetDevice(&old);
  HIPCHECK(hipSetDevice(comm->device));
  NCCLCHECK(comm_wait_own_launches(comm));
  HIPCHECK(hipMemcpy((char*)comm->devComm + offsetof(DevComm, useFences), &useFences, sizeof(int),
                     hipMemcpyHostToDevice));
  if (old >= 0) (void)hipSetDevice(old);
  return ncclSuccess;
}

// vccl_ext.h: the SIMPLE ring's slot hand-off for later launches (host
// only: the launcher picks the kernel; both leave the channel's FIFO state
// identical, so no wait is needed).
VCCL_EXPORT ncclResult_t vcclCommSetRingWave(ncclComm_t comm, int perWave, unsigned long long* waveLaunches) {
  NCCLCHECK(comm_check(comm, "vcclCommSetRingWave"));
  if (perWave != 0 && perWave != 1 && perWave != -1) return ncclInvalidArgument;
  if (perWave >= 0) comm->ringWave = perWave;
  if (waveLaunches) *waveLaunches = comm->waveLaunches;
  return ncclSuccess;
}

VCCL_EXPORT ncclResult_t vcclCommDebugSetEpochs(ncclComm_t comm, uint32_t llEpoch,
                                                uint32_t directEpoch) {
  NCCLCHECK(comm_check(comm, "vcclCommDebugSetEpochs"));
  if (comm->nRanks < 2 || !comm->devComm) return ncclSuccess;
  int old = -1;
  (void)hipGetDevice(&old);
  HIPCHECK(hipSetDevice(comm->device));
  NCCLCHECK(comm_wait_own_launches(comm));
  HIPCHECK(hipMemcpy((char*)comm->devComm + offsetof(DevComm, llEpoch), &llEpoch, sizeof(uint32_t),
                     hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy((char*)comm->devComm + offsetof(DevComm, dEpoch), &directEpoch,
                     sizeof(uint32_t), hipMemcpyHostToDevice));
  if (old >= 0) (void)hipSetDevice(old);
  return ncclSuccess;
}

// nccl.h.in:191-193: reload the logging level from NCCL_DEBUG / VCCL_DEBUG
VCCL_EXPORT void ncclResetDebugInit() { reset_log_level(); }

// pnccl* profiling aliases (src/include/core.h:18-31)
extern "C" {
void pncclResetDebugInit() VCCL_ALIAS(ncclResetDebugInit);
ncclResult_t pncclGetVersion(int*) VCCL_ALIAS(ncclGetVersion);
ncclResult_t pncclGetUniqueId(ncclUniqueId*) VCCL_ALIAS(ncclGetUniqueId);
ncclResult_t pncclCommInitRank(ncclComm_t*, int, ncclUniqueId, int) VCCL_ALIAS(ncclCommInitRank);
ncclResult_t pncclCommInitRankConfig(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*)
    VCCL_ALIAS(ncclCommInitRankConfig);
ncclResult_t pncclCommInitAll(ncclComm_t*, int, const int*) VCCL_ALIAS(ncclCommInitAll);
ncclResult_t pncclCommSplit(ncclComm_t, int, int, ncclComm_t*, ncclConfig_t*) VCCL_ALIAS(ncclCommSplit);
ncclResult_t pncclCommInitRankScalable(ncclComm_t*, int, int, int, ncclUniqueId*, ncclConfig_t*)
    VCCL_ALIAS(ncclCommInitRankScalable);
ncclResult_t pncclMemAlloc(void**, size_t) VCCL_ALIAS(ncclMemAlloc);
ncclResult_t pncclMemFree(void*) VCCL_ALIAS(ncclMemFree);
ncclResult_t pncclCommRegister(const ncclComm_t, void*, size_t, void**) VCCL_ALIAS(ncclCommRegister);
ncclResult_t pncclCommDeregister(const ncclComm_t, void*) VCCL_ALIAS(ncclCommDeregister);
ncclResult_t pncclCommFinalize(ncclComm_t) VCCL_ALIAS(ncclCommFinalize);
ncclResult_t pncclCommDestroy(ncclComm_t) VCCL_ALIAS(ncclCommDestroy);
ncclResult_t pncclCommAbort(ncclComm_t) VCCL_ALIAS(ncclCommAbort);
const char* pncclGetErrorString(ncclResult_t) VCCL_ALIAS(ncclGetErrorString);
const char* pncclGetLastError(ncclComm_t) VCCL_ALIAS(ncclGetLastError);
ncclResult_t pncclCommGetAsyncError(ncclComm_t, ncclResult_t*) VCCL_ALIAS(ncclCommGetAsyncError);
ncclResult_t pncclCommCount(const ncclComm_t, int*) VCCL_ALIAS(ncclCommCount);
ncclResult_t pncclCommCuDevice(const ncclComm_t, int*) VCCL_ALIAS(ncclCommCuDevice);
ncclResult_t pncclCommUserRank(const ncclComm_t, int*) VCCL_ALIAS(ncclCommUserRank);
}
