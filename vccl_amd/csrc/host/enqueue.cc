// Collective API -> argument check -> op encoding -> task -> launch.
//
// Keeps the observable semantics of the reference's dispatch surface
// (collectives.cc:77-158 -> ncclEnqueueCheck enqueue.cc:2448-2525 -> ArgsCheck
// misc/argcheck.cc:45-86 -> taskAppend enqueue.cc:2315-2442 with
// hostToDevRedOp :2217-2310 and the nRanks==1 shortcut ncclLaunchOneRank
// onerank.cu:47-83), re-implemented for one node: the planner picks a path
// per call (select_algo: one-shot LL, LL128 ring, two-shot direct, SIMPLE
// ring over xGMI); the ring's channel partition is VCCL's own cbd split
// (cbd_schedule below, ring.hpp cbd_part).  Group semantics (group.cc:92-110,
// :393-506): calls between ncclGroupStart/End are queued per thread and, at
// the outermost ncclGroupEnd, each comm's calls are laid out on VCCL's
// multi-task plan (group_plan: aggregation, a path per aggregate, the shared
// channel cursor) and launched in plan order, runs of one path fused into
// one launch (launch_group).
#include <algorithm>
#include <cstring>
#include <vector>

#include "../../../include/vccl_device.h"
#include "../../../include/vccl_ext.h"
#include "../device/dispatch.hpp"
#include "../device/launch.hpp"
#include "../device/ring_launch.hpp"
#include "core.h"

namespace vccl {

enum Coll { kAllReduce = 0, kReduceScatter = 1, kAllGather = 2, kBroadcast = 3, kReduce = 4 };
// Byte-copy collectives: the host rewrites them as int8 (enqueue.cc:2400-2404).
static inline bool is_copy_coll(int coll) { return coll == kAllGather || coll == kBroadcast; }

// One call's part of VCCL's channel partition (ncclDevWorkColl channelLo /
// channelHi + cbd, device.h:258-287): channels [channelLo, channelHi] carry
// parts of countLo / countMid... / countHi elements, moved in chunks of
// chunkLo / chunkMid / chunkHi elements.
struct CbdPlan {
  int channelLo, channelHi;
  int64_t countLo, countMid, countHi;
  int64_t chunkLo, chunkMid, chunkHi;  // elements
};

struct Task {
  int coll;
  const void* sendbuff;
  void* recvbuff;
  size_t count;
  ncclDataType_t datatype;
  int devOp;
  uint64_t arg;
  const void* argPtr;  // ncclScalarDevice PreMulSum scalar
  int root;            // broadcast / reduce
  ncclComm* comm;
  hipStream_t stream;
  // Set by the group planner (launch_planned): this call's partition inside
  // its group's VCCL plan, under the protocol of the path its aggregate took;
  // otherwise the call is planned alone (cbd_schedule).
  bool planned;
  CbdPlan plan;
};

// The paths a call can take (choose_algo / select_algo below).
enum { kAlgoRing = 0, kAlgoLL = 1, kAlgoDirect = 2, kAlgoRingLL128 = 3 };

static thread_local int tl_groupDepth = 0;
static thread_local std::vector<Task> tl_tasks;
static thread_local ncclResult_t tl_groupError = ncclSuccess;

static int type_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: case ncclFloat8e4m3: case ncclFloat8e5m2: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return -1;
  }
}

// __nv_cvt_float_to_fp8(f, __NV_SATFINITE, fmt) for the avg scalar
// (enqueue.cc:2265-2272): RN-even to `mbits` mantissa bits with exponent bias
// `bias`, magnitudes past max finite saturate, NaN -> 0x7f.
static uint8_t f32_to_fp8_satfinite(float f, int mbits, int bias, uint32_t maxCode) {
  uint32_t u;
  memcpy(&u, &f, 4);
  const uint32_t s = (u >> 24) & 0x80u, a = u & 0x7fffffffu;
  if (a > 0x7f800000u) return 0x7fu;
  const int e = (int)(a >> 23) - 127, emin = 1 - bias;
  if (a == 0) return (uint8_t)s;
  const uint64_t m = (a & 0x7fffffu) | 0x800000u;
  const int shift = (e >= emin ? e : emin) - mbits - e + 23;  // >= 23 - mbits
  uint64_t q = 0;
  if (shift < 40) {
    q = m >> shift;
    const uint64_t rem = m & ((1ull << shift) - 1), half = 1ull << (shift - 1);
    if (rem > half || (rem == half && (q & 1))) q++;
  }
  uint64_t code = e >= emin ? ((uint64_t)(e + bias) << mbits) + (q - (1ull << mbits)) : q;
  if (e > 15 + bias || code > maxCode) code = maxCode;
  return (uint8_t)(s | code);
}

// hostToDevRedOp (enqueue.cc:2217-2310) for built-in ops.
static ncclResult_t host_to_dev_redop(ncclRedOp_t op, ncclDataType_t dt, int nRanks, int* devOp,
                                      uint64_t* arg) {
  const int nbits = 8 * type_size(dt);
  if (nbits <= 0) return ncclInvalidArgument;
  const uint64_t allBits = ~0ull >> (64 - nbits);
  const uint64_t signBit = allBits ^ (allBits >> 1);
  const bool isSigned = dt == ncclInt8 || dt == ncclInt32 || dt == ncclInt64;
  *arg = 0;
  switch ((int)op) {
    case ncclSum: *devOp = OP_SUM; return ncclSuccess;
    case ncclProd: *devOp = OP_PROD; return ncclSuccess;
    case ncclMin:
    case ncclMax:
      *devOp = OP_MINMAX;
      if (isSigned) *arg ^= signBit;
      if (op == ncclMax) *arg ^= allBits;
      return ncclSuccess;
    case ncclAvg:
      switch ((int)dt) {
        case ncclInt8: case ncclInt32: case ncclInt64:
        case ncclUint8: case ncclUint32: case ncclUint64:
          *devOp = OP_SUMPOSTDIV;
          *arg = ((uint64_t)nRanks << 1) | (isSigned ? 1 : 0);
          return ncclSuccess;
        case ncclFloat16: {
          *devOp = OP_PREMULSUM;
          _Float16 h = (_Float16)(float)(1.0 / nRanks);
          uint16_t b;
          memcpy(&b, &h, 2);
          *arg = b;
          return ncclSuccess;
        }
        case ncclBfloat16: {
          *devOp = OP_PREMULSUM;
          __bf16 h = (__bf16)(float)(1.0 / nRanks);
          uint16_t b;
          memcpy(&b, &h, 2);
          *arg = b;
          return ncclSuccess;
        }
        case ncclFloat32: {
          *devOp = OP_PREMULSUM;
          float f = (float)(1.0 / nRanks);
          uint32_t b;
          memcpy(&b, &f, 4);
          *arg = b;
          return ncclSuccess;
        }
        case ncclFloat64: {
          *devOp = OP_PREMULSUM;
          double d = 1.0 / nRanks;
          memcpy(arg, &d, 8);
          return ncclSuccess;
        }
        case ncclFloat8e4m3:
          *devOp = OP_PREMULSUM;
          *arg = f32_to_fp8_satfinite((float)(1.0 / nRanks), 3, 7, 0x7eu);
          return ncclSuccess;
        case ncclFloat8e5m2:
          *devOp = OP_PREMULSUM;
          *arg = f32_to_fp8_satfinite((float)(1.0 / nRanks), 2, 15, 0x7bu);
          return ncclSuccess;
      }
      return ncclInvalidArgument;
  }
  return ncclInvalidArgument;
}

static ncclResult_t resolve_op(ncclComm* comm, ncclRedOp_t op, ncclDataType_t dt, int* devOp,
                               uint64_t* arg, const void** argPtr) {
  *argPtr = nullptr;
  if ((int)op < (int)ncclNumOps) return host_to_dev_redop(op, dt, comm->nRanks, devOp, arg);
  const int ix = (int)op - (int)ncclNumOps;
  if (ix >= (int)comm->userOps.size() || comm->userOps[ix].freeNext != -1) return ncclInvalidArgument;
  const UserRedOp& u = comm->userOps[ix];
  if (u.datatype != dt) {  // enqueue.cc:2301-2305
    VWARN("Data type supplied to user-created ncclRedOp_t does not match type given to reduction operation");
    return ncclInvalidArgument;
  }
  *devOp = u.devOp;
  *arg = u.argIsPtr ? 0 : u.arg;
  if (u.argIsPtr) *argPtr = (const void*)u.arg;
  return ncclSuccess;
}

// ArgsCheck (misc/argcheck.cc:45-86) minus the root check (no rooted colls).
static ncclResult_t args_check(ncclComm* comm, const char* name, ncclDataType_t dt, ncclRedOp_t op,
                               bool hasOp) {
  if ((int)dt < 0 || (int)dt >= (int)ncclNumTypes) {
    VWARN("%s : invalid type %d", name, (int)dt);
    return ncclInvalidArgument;
  }
  if (hasOp) {
    if ((int)op < 0 || (int)op > (int)ncclMaxRedOp) {
      VWARN("%s : invalid reduction operation %d", name, (int)op);
      return ncclInvalidArgument;
    }
    const int ix = (int)op - (int)ncclNumOps;
    if (ix >= 0 && (ix >= (int)comm->userOps.size() || comm->userOps[ix].freeNext != -1)) {
      VWARN("%s : reduction operation %d unknown to this communicator", name, (int)op);
      return ncclInvalidArgument;
    }
  }
  // fp8 (enqueue.cc:2379-2384 requires sm90 in the reference): native on gfx950
  return ncclSuccess;
}

// Order launches of one comm across different user streams (the reference
// serialises through its internal strong stream, enqueue.cc:1445-1548).
// The null stream (0) is a valid user stream, so "no launch yet" is a flag of
// its own, not a null lastStream.
//
// Graph capture (the reference's strong streams track capture the same way,
// misc/strongstream.cc): launches on a capturing stream are ordered only
// against earlier launches of the SAME capture, through an event recorded
// inside it (a fork/join inside the graph); they neither wait on the eager
// lastLaunch event (recorded outside the capture) nor overwrite it, so eager
// work before and after the capture keeps its own ordering.
struct CaptureState {
  bool active;
  unsigned long long id;
};
static ncclResult_t capture_state(hipStream_t s, CaptureState* cs) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  HIPCHECK(hipStreamGetCaptureInfo(s, &st, &id));
  cs->active = st == hipStreamCaptureStatusActive;
  cs->id = id;
  return ncclSuccess;
}
// The ordering state of capture `id`: comm->caps is a pool of kMaxCaptures
// entries created at init (no HIP object is created during a capture); a new
// id takes the least recently used entry whose capture has ended.  When every
// entry still belongs to a live capture, the call fails (ncclInvalidUsage)
// rather than silently dropping a live capture's ordering.
// A capture is live while its last stream still captures under its id; a
// stream destroyed since reads as ended (HIP validates the handle and fails
// the query — tests/mp_graph_worker.py captures_on_destroyed_streams).
static bool capture_live(const ncclComm::CapOrder& c) {
  if (!c.used || !c.has) return false;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  if (hipStreamGetCaptureInfo(c.last, &st, &id) != hipSuccess) return false;
  return st == hipStreamCaptureStatusActive && id == c.id;
}
static ncclResult_t capture_entry(ncclComm* comm, unsigned long long id, bool create,
                                  ncclComm::CapOrder** out) {
  *out = nullptr;
  auto& caps = comm->caps;
  for (size_t i = 0; i < caps.size(); i++) {
    if (caps[i].used && caps[i].id == id) {
      std::rotate(caps.begin(), caps.begin() + i, caps.begin() + i + 1);  // to the front
      *out = &caps[0];
      return ncclSuccess;
    }
  }
  if (!create || caps.empty()) return ncclSuccess;
  for (size_t i = caps.size(); i-- > 0;) {  // least recently used first
    if (capture_live(caps[i])) continue;
    std::rotate(caps.begin(), caps.begin() + i, caps.begin() + i + 1);
    caps[0].id = id;
    caps[0].used = true;
    caps[0].last = nullptr;
    caps[0].has = false;
    *out = &caps[0];
    return ncclSuccess;
  }
  VWARN("more than %d stream captures are active on this communicator at once", (int)caps.size());
  return ncclInvalidUsage;
}
// One capture query per call: stream_order fills `cs`, stream_mark and
// stream_last_event reuse it (the capture state of s cannot change between
// them — the caller holds the thread).
static ncclResult_t stream_order(ncclComm* comm, hipStream_t s, CaptureState* cs) {
  NCCLCHECK(capture_state(s, cs));
  if (cs->active) {
    ncclComm::CapOrder* c;
    NCCLCHECK(capture_entry(comm, cs->id, true, &c));  // reserved before the launch
    if (c && c->has && c->last != s) HIPCHECK(hipStreamWaitEvent(s, c->ev, 0));
    return ncclSuccess;
  }
  if (comm->hasLastLaunch && comm->lastStream != s)
    HIPCHECK(hipStreamWaitEvent(s, comm->lastLaunch, 0));
  return ncclSuccess;
}
// The event the launches of an eager call bind to their kernel's completion
// (hipExtLaunchKernel stopEvent): the comm's ordering event, recorded by the
// kernel's own completion signal instead of a separate marker packet — a
// marker costs ~5 us of GPU time per call on MI355X (profiles/r04q: LL 8 B
// 10.1 -> 5.7 us per call back to back, 1 MiB ring 17.5 -> 12.7).
// VCCL_LAUNCH_EVENT=0: record markers.  Captures keep markers (graph edges).
static hipEvent_t stop_event(ncclComm* comm, const CaptureState& cs) {
  static const bool bind = param_int("LAUNCH_EVENT", 1) != 0;
  return bind && !cs.active ? comm->lastLaunch : nullptr;
}
static ncclResult_t stream_mark(ncclComm* comm, hipStream_t s, const CaptureState& cs) {
  if (cs.active) {
    ncclComm::CapOrder* c;
    NCCLCHECK(capture_entry(comm, cs.id, true, &c));
    if (!c) return ncclInternalError;
    HIPCHECK(hipEventRecord(c->ev, s));
    c->last = s;
    c->has = true;
    return ncclSuccess;
  }
  // VCCL_DEBUG_NO_MARK=1: no marker packet (measurement only: correct for a
  // comm driven from ONE stream, where stream order suffices).  The launch is
  // still tracked: through the stop event when the kernel bound
  // it, else by its stream, so destroy / finalize / abort still wait for it.
  static const bool noMark = param_int("DEBUG_NO_MARK", 0) != 0;
  const bool bound = stop_event(comm, cs) != nullptr;
  if (!noMark && !bound) HIPCHECK(hipEventRecord(comm->lastLaunch, s));  // else bound to the kernel
  comm->lastUnmarked = noMark && !bound;
  comm->lastStream = s;
  comm->hasLastLaunch = true;
  return ncclSuccess;
}
// The event stream_mark just recorded on s (for joining other streams).
static hipEvent_t stream_last_event(ncclComm* comm, const CaptureState& cs) {
  return cs.active ? comm->caps[0].ev : comm->lastLaunch;
}

// ncclLaunchOneRank (onerank.cu:47-83): a copy, or the PreMulSum kernel.
static ncclResult_t launch_one_rank(const Task& t) {
  const size_t bytes = t.count * (size_t)type_size(t.datatype);
  if (is_copy_coll(t.coll) || t.devOp != OP_PREMULSUM) {  // AG: a plain copy
    if (t.recvbuff == t.sendbuff) return ncclSuccess;
    // Small buckets: the library's own byte-copy kernel (one launch) — a
    // hipMemcpyAsync D2D costs more host time than the whole 1 KiB copy
    // (BASELINE config 1).  Large ones: the runtime's copy engine path.
    static const size_t kKernelCopyMax = (size_t)param_int("ONERANK_KERNEL_COPY_BYTES", 1 << 20);
    if (bytes <= kKernelCopyMax) {
      RCArgs a = {};
      a.srcs[0] = (const char*)t.sendbuff;
      a.dsts[0] = (char*)t.recvbuff;
      a.nSrcs = a.nDsts = 1;
      hipError_t e = reduce_copy_launch(OP_COPY, (int)ncclUint8, 0, a, (int64_t)bytes, nullptr,
                                        t.stream);
      return e == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
    }
    HIPCHECK(hipMemcpyAsync(t.recvbuff, t.sendbuff, bytes, hipMemcpyDeviceToDevice, t.stream));
    return ncclSuccess;
  }
  RCArgs a = {};
  a.srcs[0] = (const char*)t.sendbuff;
  a.dsts[0] = (char*)t.recvbuff;
  a.nSrcs = a.nDsts = 1;
  a.preOpSrcs = 1;  // onerank.cu:43: PreOpSrcs=1, postOp=true
  a.postOp = 1;
  a.argPtr = t.argPtr;
  hipError_t e = reduce_copy_launch(t.devOp, (int)t.datatype, t.arg, a, (int64_t)t.count, nullptr,
                                    t.stream);
  return e == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

// VCCL's channel partition of ring collectives: the host side of
// scheduleCollTasksToPlan (enqueue.cc:518-769) with the ring channel tuning
// of topoGetAlgoInfo (:1902-1925) and calcCollChunking's RING chunk
// (:2027-2032, 2093), so every element lands on the same channel and the same
// chunk of the same loop as in VCCL — hence the same ring and fold order.
// `count` / `eltSize` are already AG-rewritten to bytes.  Restated for the
// tests in oracle/vccl_sched.py.
//
// proto: kProtoSimple or kProtoLL128.  stepBytes: that protocol's FIFO step
// (buffSize / NCCL_STEPS).  nThreads: maxThreads[RING][proto] — NCCL_NTHREADS
// for SIMPLE (the ring kernel's own block size here, comm->nThreads),
// NCCL_LL128_NTHREADS (640) for LL128 (tuning.cc:198-211).
constexpr uint64_t kMinTraffic = 16 << 10;  // MinTrafficPerChannel, enqueue.cc:528
static int64_t div_up(int64_t a, int64_t b) { return (a + b - 1) / b; }
static int64_t traffic_per_byte(int coll, int nRanks) {  // ncclFuncTrafficPerByte (enqueue.cc:67-74)
  return coll == kAllReduce ? 2 : coll == kBroadcast || coll == kReduce ? 1 : nRanks;
}

// nMaxChannels of a task (or of an aggregate of tasks, ncclPrepareTasks):
// the ring / tree channel tuning on nBytes = eltSize * ncclFuncMaxSendRecvCount
// (enqueue.cc:1955, 1921-1924); thread thresholds (comm.h:38-40,
// tuning.cc:489-493) SIMPLE 64, LL128 8, LL 8 — times nRanks for the ring's
// LL (reduce-scatter / all-gather), not for the all-reduce's LL, which VCCL
// runs on its tree.  nThreads: maxThreads of the protocol (tuning.cc:198-211:
// NCCL_NTHREADS for SIMPLE and LL, NCCL_LL128_NTHREADS for LL128).
static int ring_nmax_channels(int coll, int64_t count, int64_t eltSize, int nRanks, int commChannels,
                              int proto, int64_t nThreads) {
  const int64_t threshold = proto == kProtoSimple ? 64
                            : proto == kProtoLL128 || coll == kAllReduce ? 8 : 8 * (int64_t)nRanks;
  // ncclFuncMaxSendRecvCount (enqueue.h:36-38): RS / AG move n blocks
  const int64_t nBytes =
      eltSize * (coll == kReduceScatter || coll == kAllGather ? (int64_t)nRanks * count : count);
  int64_t nc = commChannels;
  while (nBytes < nc * nThreads * threshold && nc >= 2) nc--;
  return (int)nc;
}

// The running channel position of a plan (scheduleCollTasksToPlan's
// trafficPerChannel / channelId / currentTraffic, enqueue.cc:549-565).
struct PlanCursor {
  uint64_t trafficPerChannel;
  int channelId;
  uint64_t currentTraffic;
  int nMax;  // nMaxChannels[kind] = comm->nChannels
};

// VCCL's LL step (the default LL buffer, init.cc:617: 8 lines x 512 threads
// x NCCL_STEPS x 16 B, over NCCL_STEPS): only the chunk fields of an LL
// task's plan use it, and the one-hop LL kernels ignore those.
constexpr int64_t kLLStepBytes = 8 * 512 * 16;

// The cbd cell split of one task at the cursor (enqueue.cc:597-644; LL
// counts its traffic 4x, :599), then the cursor advanced past it (:667-681).
static CbdPlan cbd_place(PlanCursor& pc, int coll, int64_t count, int64_t eltSize, int nRanks,
                         int proto, int64_t stepBytes) {
  const bool ll128 = proto == kProtoLL128, ll = proto == kProtoLL;
  const uint64_t tpb = (uint64_t)traffic_per_byte(coll, nRanks) * (ll ? 4 : 1);
  const uint64_t cellSize = (uint64_t)div_up(div_up(kMinTraffic, tpb), 16) * 16;
  const uint64_t eltsPerCell = cellSize / (uint64_t)eltSize;
  const uint64_t cells = (uint64_t)div_up(count * eltSize, (int64_t)cellSize);
  const uint64_t trafficPerElement = (uint64_t)eltSize * tpb;
  const uint64_t trafficPerCell = cellSize * tpb;
  const uint64_t tpc = pc.trafficPerChannel;
  uint64_t cellsPerChannel = std::min(cells, (tpc + trafficPerCell - 1) / trafficPerCell);
  uint64_t cellsLo;
  if (pc.channelId + 1 == pc.nMax) cellsLo = cells;  // on the last channel everything goes to "lo"
  else cellsLo = std::min(cells, (tpc - pc.currentTraffic + trafficPerCell - 1) / trafficPerCell);
  int nMid = (int)((cells - cellsLo) / cellsPerChannel);
  uint64_t cellsHi = (cells - cellsLo) % cellsPerChannel;
  int nCh = (cellsLo != 0 ? 1 : 0) + nMid + (cellsHi != 0 ? 1 : 0);
  if (pc.nMax < pc.channelId + nCh) {  // overflowed the available channels
    nMid = pc.nMax - pc.channelId - 2;
    cellsPerChannel = (cells - cellsLo) / (uint64_t)(nMid + 1);
    cellsHi = cellsPerChannel + (cells - cellsLo) % (uint64_t)(nMid + 1);
  }
  if (cellsHi == 0 && nMid != 0) {
    cellsHi = cellsPerChannel;
    nMid -= 1;
  }
  if (cellsLo == 0) {  // least channel skipped: the next one becomes the least
    pc.channelId += 1;
    if (nMid == 0) {
      cellsLo = cellsHi;
      cellsHi = 0;
    } else {
      cellsLo = cellsPerChannel;
      nMid -= 1;
    }
  }
  CbdPlan p{};
  p.countMid = nMid != 0 ? (int64_t)(cellsPerChannel * eltsPerCell) : 0;
  p.countLo = (int64_t)(cellsLo * eltsPerCell);
  p.countHi = (int64_t)(cellsHi * eltsPerCell);
  (p.countHi != 0 ? p.countHi : p.countLo) -= (int64_t)(cells * eltsPerCell) - count;
  nCh = (p.countLo != 0 ? 1 : 0) + nMid + (cellsHi != 0 ? 1 : 0);
  p.channelLo = pc.channelId;
  p.channelHi = pc.channelId + nCh - 1;
  // RING chunk (calcCollChunking, enqueue.cc:2027-2032, 2093): SIMPLE =
  // chunkSteps (4) FIFO steps of buffSize / NCCL_STEPS (= one slot here);
  // LL128 = one step, 15/16 of it data; LL = half a step; rounded down to
  // the protocol grain (device.h:290-295: SIMPLE 512, LL128 1920, LL 16);
  // independent of size.
  // (broadcast / reduce: BROADCAST_CHUNKSTEPS / REDUCE_CHUNKSTEPS 1,
  // collectives.h:23-26)
  const int64_t grain = ll128 ? 1920 : ll ? 16 : 512;
  const int64_t chunkBytes =
      ll128 ? stepBytes / 16 * 15 : ll ? stepBytes / 2 : (coll == kBroadcast || coll == kReduce ? 1 : 4) * stepBytes;
  const int64_t chunkElts = chunkBytes / grain * grain / eltSize;
  p.chunkLo = p.chunkMid = p.chunkHi = chunkElts;
  // advance the cursor (enqueue.cc:667-681)
  if (p.countHi != 0) {
    pc.channelId += nCh - 1;
    pc.currentTraffic = cellsHi * eltsPerCell * trafficPerElement;
  } else if (nMid != 0) {
    pc.channelId += nCh;
    pc.currentTraffic = 0;
  } else {
    pc.currentTraffic += cellsLo * eltsPerCell * trafficPerElement;
  }
  if (pc.currentTraffic >= tpc && pc.channelId + 1 != pc.nMax) {
    pc.channelId += 1;
    pc.currentTraffic = 0;
  }
  return p;
}

// A plan holding one ring collective (a call outside a group).
static CbdPlan cbd_schedule(int coll, int64_t count, int64_t eltSize, int nRanks, int commChannels,
                            int proto, int64_t stepBytes, int64_t nThreads) {
  const int nc = ring_nmax_channels(coll, count, eltSize, nRanks, commChannels, proto, nThreads);
  const uint64_t traffic = std::max<uint64_t>(
      kMinTraffic, (uint64_t)(count * eltSize) * traffic_per_byte(coll, nRanks) * (proto == kProtoLL ? 4 : 1));
  PlanCursor pc{std::max<uint64_t>(kMinTraffic, traffic / (uint64_t)std::min(nc, commChannels)), 0, 0,
                commChannels};
  return cbd_place(pc, coll, count, eltSize, nRanks, proto, stepBytes);
}

// ---------------------------------------------------------------- paths
// The path of a bucket (VCCL's topoGetAlgoInfo, enqueue.cc:1805-1945, reduced
// to one node over a full xGMI mesh): buckets up to the LL threshold take the
// one-hop LL path, the LL128 window (when enabled) the LL128 ring, up to the
// direct threshold the direct path (all-reduce two-shot, reduce-scatter /
// all-gather one-hop), larger ones the SIMPLE ring.  NCCL_ALGO / NCCL_PROTO
// force one: Ring/SIMPLE -> ring; Tree/LL -> LL where it fits; Direct -> direct
// where the mesh has it; LL128 -> the LL128 ring where its FIFOs exist;
// anything that does not fit falls through to the ring.  A pure function of
// the comm's thresholds (AlgoPolicy), so the group planner can ask it for an
// aggregate of calls as ncclPrepareTasks asks getAlgoInfo (enqueue.cc:398).
struct AlgoPolicy {
  int nRanks = 1, algoForce = 0;
  int64_t llSlotBytes = 0;                 // 0: no LL buffers
  uint64_t llMax = 0, llRsAgMax = 0;
  bool ll128 = false;                      // LL128 FIFOs mapped
  uint64_t ll128Min = 0, ll128Max = 0;     // automatic LL128 window (max 0 = off)
  bool direct = false;                     // every peer's inbox mapped
  uint64_t directMax = 0, directRsAgMax = 0;
};
static AlgoPolicy policy_of(const ncclComm* c) {
  AlgoPolicy p;
  p.nRanks = c->nRanks;
  p.algoForce = c->algoForce;
  p.llSlotBytes = c->llBuf ? (int64_t)c->llLines * 8 : 0;
  p.llMax = c->llMaxBytes;
  p.llRsAgMax = c->llRsAgMaxBytes;
  p.ll128 = c->ll128Buf != nullptr;
  p.ll128Min = c->ll128MinBytes;
  p.ll128Max = c->ll128MaxBytes;
  p.direct = c->dPeers != nullptr;
  p.directMax = c->directMaxBytes;
  p.directRsAgMax = c->directRsAgMaxBytes;
  return p;
}
// count in elements of eltSize (all-gather: any element type, or bytes)
static int select_algo(const AlgoPolicy& p, int coll, int64_t eltSize, int64_t count) {
  if (p.nRanks < 2 || p.algoForce == 1) return kAlgoRing;
  // NCCL_PROTO=LL128 (or vcclCommSetAlgo): the LL128 ring for every size
  if (p.algoForce == 4) return p.ll128 ? kAlgoRingLL128 : kAlgoRing;
  if (coll == kBroadcast || coll == kReduce) {  // the rings of broadcast.h / reduce.h: SIMPLE or the LL128 window
    const uint64_t bytes = (uint64_t)(count * eltSize);
    return p.ll128 && p.ll128Max && bytes >= p.ll128Min && bytes <= p.ll128Max ? kAlgoRingLL128 : kAlgoRing;
  }
  const uint64_t block = (uint64_t)(count * eltSize);
  // Reduce-scatter / all-gather: one rank's block must fit an LL slot; the
  // thresholds are on the whole bucket (n blocks), as the reference's tuner
  // sizes RS / AG (enqueue.cc:1955, ncclFuncMaxSendRecvCount).
  const uint64_t bytes = coll == kAllReduce ? block : block * (uint64_t)p.nRanks;
  const bool llFits = coll == kAllReduce
                          ? p.llSlotBytes > 0 && bytes <= p.llMax
                          : p.llSlotBytes > 0 && p.nRanks <= kOrderMaxRanks &&
                                block <= (uint64_t)p.llSlotBytes && bytes <= p.llRsAgMax;
  const bool directFits = p.direct && bytes <= (coll == kAllReduce ? p.directMax : p.directRsAgMax);
  if (p.algoForce == 2) return llFits ? kAlgoLL : kAlgoRing;
  // Forced direct: any bucket the inbox can stream (the size threshold only
  // steers the automatic choice); needs every peer's inbox mapped (no net
  // peers)
  if (p.algoForce == 3) return p.direct && p.nRanks <= kDirectMaxRanks ? kAlgoDirect : kAlgoRing;
  if (llFits) return kAlgoLL;
  // the LL128 ring over its window (the bucket, as the tuner sizes it), ahead
  // of the direct path
  if (p.ll128 && p.ll128Max && bytes >= p.ll128Min && bytes <= p.ll128Max) return kAlgoRingLL128;
  if (directFits) return kAlgoDirect;
  return kAlgoRing;
}
// The protocol VCCL runs a path's calls with: the one-hop LL stands in for
// VCCL's LL (tree for the all-reduce, ring otherwise), the direct path for a
// SIMPLE ring call.
static int proto_of_algo(int algo) {
  return algo == kAlgoLL ? kProtoLL : algo == kAlgoRingLL128 ? kProtoLL128 : kProtoSimple;
}

// ---------------------------------------------------------------- group plan
// VCCL's plan for a group's collectives of one comm:
//  * taskAppend: trafficBytes = count * eltSize * trafficPerByte, inserted
//    into the size sorter (enqueue.cc:2405-2413; comm.h:294-343: 81 bins of
//    u32fpEncode(min(bytes, 1 GiB) >> 10, 2 bits) in descending size, LIFO
//    within a bin, bitops.h:252-262);
//  * ncclPrepareTasks (enqueue.cc:352-437): the sorted list binned by
//    (func, devOp, type) in LIFO order — each bin size-ascending, bins in
//    order of first appearance; runs within 4x of the run's first
//    trafficBytes aggregated; the path (select_algo, standing in for
//    getAlgoInfo's tuner) and nMaxChannels chosen on the aggregate's count
//    and given to every member; an LL member's trafficBytes x4 (:418);
//  * scheduleCollTasksToPlan (enqueue.cc:518-769): trafficPerChannel = the
//    plan's traffic / min(sum nMaxChannels, comm channels), each task placed
//    at the running channelId / currentTraffic under its protocol; a task
//    that would overflow the kernel-argument budget (testBudget :278-286:
//    16-byte work batches within 4 KiB - 32 B of kernel arguments, 96-byte
//    works within half the 1 MiB work FIFO; batches counted as
//    addWorkBatchToPlan :91-156 does, per device function and protocol)
//    starts the next plan.
// No policy: every call RING / SIMPLE.  Restated for the tests in
// oracle/vccl_sched.py (plan_schedule).
struct GroupTask {
  int coll;
  int64_t count, eltSize;  // AG in bytes
  int binKey;              // (func, devOp, type): ncclPrepareTasks' bins
  int funcKey;             // the device function (batches merge per function)
};
struct PlanGeometry {
  int64_t stepBytes, nThreads;            // SIMPLE: FIFO step, NCCL_NTHREADS
  int64_t ll128StepBytes, ll128Threads;   // LL128: step, NCCL_LL128_NTHREADS
};
struct GroupPlanOut {
  std::vector<int> order;        // tasks in execution (plan) order
  std::vector<int> planOf;       // per task: the plan (kernel) it lands in
  std::vector<int> algo;         // per task: the path of its aggregate
  std::vector<CbdPlan> cbd;      // per task, under the path's protocol
};
static uint32_t u32fp_encode(uint32_t x, int bitsPerPow2) {  // bitops.h:252-262
  const int log2x = 31 - __builtin_clz(x | 1);
  const uint32_t mantissa = x >> (log2x >= bitsPerPow2 ? log2x - bitsPerPow2 : 0) & ((1u << bitsPerPow2) - 1);
  const uint32_t exponent = log2x >= bitsPerPow2 ? log2x - (bitsPerPow2 - 1) : 0;
  return exponent << bitsPerPow2 | mantissa;
}
static void group_plan(const std::vector<GroupTask>& ts, int nRanks, int commChannels, const PlanGeometry& geo,
                       const AlgoPolicy* pol, GroupPlanOut* out) {
  const int n = (int)ts.size();
  std::vector<uint64_t> traffic(n);
  for (int i = 0; i < n; i++)
    traffic[i] = (uint64_t)(ts[i].count * ts[i].eltSize) * traffic_per_byte(ts[i].coll, nRanks);
  // the size sorter: bins in descending size, LIFO within a bin
  constexpr int kBinCount = 1 + (30 - 10) * 4;
  std::vector<std::vector<int>> bins(kBinCount);
  for (int i = 0; i < n; i++) {
    const uint32_t x = (uint32_t)(std::min<uint64_t>(traffic[i], 1ull << 30) >> 10);
    bins[kBinCount - 1 - (int)u32fp_encode(x, 2)].push_back(i);
  }
  std::vector<int> sorted;
  for (auto& b : bins) sorted.insert(sorted.end(), b.rbegin(), b.rend());
  // (func, op, type) bins, LIFO, in order of first appearance
  std::vector<int> keys;
  std::vector<std::vector<int>> byKey;
  for (int i : sorted) {
    const size_t k = std::find(keys.begin(), keys.end(), ts[i].binKey) - keys.begin();
    if (k == keys.size()) {
      keys.push_back(ts[i].binKey);
      byKey.emplace_back();
    }
    byKey[k].insert(byKey[k].begin(), i);
  }
  auto step_of = [&](int proto) {
    return proto == kProtoLL ? kLLStepBytes : proto == kProtoLL128 ? geo.ll128StepBytes : geo.stepBytes;
  };
  std::vector<int> nMax(n), proto(n), queue;
  out->algo.assign(n, kAlgoRing);
  for (auto& lst : byKey) {
    for (size_t a = 0; a < lst.size();) {
      size_t e = a + 1;
      int64_t aggCount = ts[lst[a]].count;
      while (e < lst.size() && traffic[lst[e]] < 4 * traffic[lst[a]]) aggCount += ts[lst[e++]].count;
      const GroupTask& h = ts[lst[a]];
      const int algo = pol ? select_algo(*pol, h.coll, h.eltSize, aggCount) : kAlgoRing;
      const int pr = proto_of_algo(algo);
      const int nc = ring_nmax_channels(h.coll, aggCount, h.eltSize, nRanks, commChannels, pr,
                                        pr == kProtoLL128 ? geo.ll128Threads : geo.nThreads);
      for (size_t j = a; j < e; j++) {
        nMax[lst[j]] = nc;
        proto[lst[j]] = pr;
        out->algo[lst[j]] = algo;
        if (pr == kProtoLL) traffic[lst[j]] *= 4;
      }
      a = e;
    }
    queue.insert(queue.end(), lst.begin(), lst.end());
  }
  out->order = queue;
  out->planOf.assign(n, -1);
  out->cbd.assign(n, CbdPlan{});
  constexpr int64_t kWorkBytes = 96, kBatchBytes = 16;   // sizeof ncclDevWorkColl / ncclDevWorkBatch
  constexpr int64_t kInArgs = (4 << 10) - 32;            // workArgsBytes - sizeof(ncclDevKernelArgs)
  constexpr int64_t kOutArgs = (1 << 20) / 2;            // workFifoBytes / 2
  auto budget_ok = [&](int64_t nBatches, int64_t workBytes) {
    const int64_t bb = nBatches * kBatchBytes;
    return bb + workBytes <= kInArgs || (bb <= kInArgs && workBytes <= kOutArgs);
  };
  size_t head = 0;
  for (int plan = 0; head < queue.size(); plan++) {
    int nPlanColls = 0;
    uint64_t tb = 0;
    int nch = 0;
    for (size_t q = head, wb = 0; q < queue.size(); q++) {
      if (!budget_ok(div_up(nPlanColls, 4), (int64_t)wb + kWorkBytes)) break;
      nPlanColls++;
      wb += kWorkBytes;
      tb += std::max<uint64_t>(kMinTraffic, traffic[queue[q]]);
      nch = std::min(nch + nMax[queue[q]], commChannels);
    }
    PlanCursor pc{std::max<uint64_t>(kMinTraffic, tb / (uint64_t)std::max(nch, 1)), 0, 0, commChannels};
    // per channel: the work batch being filled (addWorkBatchToPlan)
    std::vector<int> lastFunc(commChannels, -1);
    std::vector<int64_t> offsetBase(commChannels, 0), wipBytes(commChannels, 0);
    int64_t nWorkBatches = 0, workBytes = 0;
    while (nPlanColls != 0 && head < queue.size()) {
      const int i = queue[head];
      PlanCursor trial = pc;
      const CbdPlan p = cbd_place(trial, ts[i].coll, ts[i].count, ts[i].eltSize, nRanks, proto[i],
                                  step_of(proto[i]));
      const int nChTask = p.channelHi - p.channelLo + 1;
      if (!budget_ok(nWorkBatches + nChTask, workBytes + kWorkBytes)) break;  // the next plan
      pc = trial;
      const int func = ts[i].funcKey * 4 + proto[i];  // devFuncId: (func, op, type, algo, proto)
      for (int c = p.channelLo; c <= p.channelHi && c < commChannels; c++) {
        const bool fresh = lastFunc[c] < 0 || lastFunc[c] != func ||
                           wipBytes[c] + kWorkBytes > 1024;  // NCCL_MAX_DEV_WORK_BATCH_BYTES
        const int64_t off = fresh ? 0 : workBytes - offsetBase[c];
        if (fresh || 63 * kWorkBytes < off) {
          offsetBase[c] = workBytes;
          if (fresh) wipBytes[c] = 0;
          nWorkBatches++;
        }
        lastFunc[c] = func;
        wipBytes[c] += kWorkBytes;
      }
      workBytes += kWorkBytes;
      out->planOf[i] = plan;
      out->cbd[i] = p;
      head++;
      nPlanColls--;
    }
  }
}

static int dev_coll(int coll) {
  return coll == kAllReduce ? kCollAllReduce
         : coll == kReduceScatter ? kCollReduceScatter
         : coll == kBroadcast ? kCollBroadcast
         : coll == kReduce ? kCollReduce : kCollAllGather;
}

// A call's partition: its place in its group's plan (launch_planned, under
// the protocol of the path its aggregate took — the caller asks for that
// same protocol), else the plan of the call alone under `proto`.
static CbdPlan task_plan(const Task& t, int proto) {
  const ncclComm* comm = t.comm;
  if (t.planned) return t.plan;
  const bool ag = is_copy_coll(t.coll);
  const int64_t esz = ag ? 1 : type_size(t.datatype);
  const int64_t count = ag ? (int64_t)t.count * type_size(t.datatype) : (int64_t)t.count;
  if (proto == kProtoLL128)
    return cbd_schedule(t.coll, count, esz, comm->nRanks, comm->nChannels, kProtoLL128, comm->ll128StepBytes,
                        comm->ll128Threads);
  return cbd_schedule(t.coll, count, esz, comm->nRanks, comm->nChannels, proto,
                      proto == kProtoLL ? kLLStepBytes : comm->stepBytes, comm->nThreads);
}

// The ring work of one call (its kernel element type and device op too).
static ncclResult_t ring_work_of(const Task& t, bool ll128, RingWork* out, int* ktOut, int* devOpOut) {
  ncclComm* comm = t.comm;
  RingWork w{};
  w.comm = comm->devComm;
  w.channels = comm->devChannels;
  w.sendbuff = t.sendbuff;
  w.recvbuff = t.recvbuff;
  w.redArg = t.arg;
  w.preOp = t.devOp == OP_PREMULSUM;
  w.nChannels = comm->nChannels;
  w.slotBytes = comm->slotBytes;
  w.nRanks = comm->nRanks;
  int kt, devOp = t.devOp;
  if (is_copy_coll(t.coll)) {
    w.count = t.count * (uint64_t)type_size(t.datatype);  // bytes (enqueue.cc:2400-2404)
    kt = K_U8;
    devOp = OP_COPY;
  } else {
    w.count = t.count;
    kt = kernel_type_of(t.devOp, (int)t.datatype);
    if (kt < 0) return ncclInvalidArgument;
  }
  w.redArgPtr = t.argPtr;  // ncclScalarDevice: dereferenced by the kernel (nccl.h.in:255-262)
  w.redArgBytes = type_size(t.datatype);
  w.root = t.root;
  const CbdPlan p = ll128 ? task_plan(t, kProtoLL128) : task_plan(t, kProtoSimple);
  if (p.channelHi >= comm->nChannels || p.channelLo < 0 || p.channelLo > p.channelHi)
    return ncclInternalError;
  w.channelLo = p.channelLo;
  w.channelHi = p.channelHi;
  w.countLo = p.countLo;
  w.countMid = p.countMid;
  w.countHi = p.countHi;
  w.chunkLo = p.chunkLo;
  w.chunkMid = p.chunkMid;
  w.chunkHi = p.chunkHi;
  w.nChannels = p.channelHi + 1;  // idle channels above channelHi are not launched
  w.ll128SlotBytes = ll128 ? comm->ll128SlotBytes : 0;
  *out = w;
  *ktOut = kt;
  *devOpOut = devOp;
  return ncclSuccess;
}

// The per-wave SIMPLE ring kernels exist for the bandwidth regime only
// (ring_kernels.hip PART 4): sums over f32 / f16 / bf16 and the byte-copy
// all-gather / broadcast.
static bool ring_wave_kernel(int kt, int devOp, int coll) {
  if (coll == kCollAllGather || coll == kCollBroadcast) return kt == K_U8;
  return devOp == OP_SUM && (kt == K_F32 || kt == K_F16 || kt == K_BF16);
}

// 1 .. kRingMaxWorks ring calls of one comm with the same collective, kernel
// type and op (fusable) in one launch on ts[0].stream; SIMPLE or LL128.  A
// SIMPLE launch takes the per-wave hand-off when the comm asks for it
// (VCCL_RING_WAVE / vcclCommSetRingWave) and the kernel exists: same FIFOs,
// partition and fold, so the two mix freely on a channel.
static ncclResult_t launch_ring(const Task* ts, int nTasks, bool ll128, hipEvent_t stop) {
  const Task& t = ts[0];
  ncclComm* comm = t.comm;
  if (nTasks < 1 || nTasks > kRingMaxWorks) return ncclInternalError;
  if (ll128 && !comm->ll128Buf) return ncclInternalError;
  RingBatch b{};
  int kt = -1, devOp = -1;
  NCCLCHECK(ring_work_of(t, ll128, &b.w, &kt, &devOp));
  for (int i = 1; i < nTasks; i++) {
    RingWork wi;
    int kti, opi;
    NCCLCHECK(ring_work_of(ts[i], ll128, &wi, &kti, &opi));
    if (kti != kt || opi != devOp) return ncclInternalError;
    b.more[i - 1] = ring_part_of(wi);
    b.w.nChannels = std::max(b.w.nChannels, wi.nChannels);
  }
  b.nParts = nTasks;
  const int coll = dev_coll(t.coll);
  const int v = ll128 ? kRingVariantLL128
                : comm->ringWave && ring_wave_kernel(kt, devOp, coll) ? kRingVariantWave : kRingVariantSimple;
  hipError_t e = hipErrorInvalidValue;
  switch (kt) {
    case K_U8: e = ring_launch_any<K_U8>(v, coll, devOp, b, comm->nThreads, t.stream, stop); break;
    case K_U32: e = ring_launch_any<K_U32>(v, coll, devOp, b, comm->nThreads, t.stream, stop); break;
    case K_U64: e = ring_launch_any<K_U64>(v, coll, devOp, b, comm->nThreads, t.stream, stop); break;
    case K_F16: e = ring_launch_any<K_F16>(v, coll, devOp, b, comm->nThreads, t.stream, stop); break;
    case K_F32: e = ring_launch_any<K_F32>(v, coll, devOp, b, comm->nThreads, t.stream, stop); break;
    case K_F64: e = ring_launch_any<K_F64>(v, coll, devOp, b, comm->nThreads, t.stream, stop); break;
    case K_BF16: e = ring_launch_any<K_BF16>(v, coll, devOp, b, comm->nThreads, t.stream, stop); break;
    case K_F8E4M3: e = ring_launch_any<K_F8E4M3>(v, coll, devOp, b, comm->nThreads, t.stream, stop); break;
    case K_F8E5M2: e = ring_launch_any<K_F8E5M2>(v, coll, devOp, b, comm->nThreads, t.stream, stop); break;
  }
  if (e != hipSuccess) {
    VWARN("ring kernel launch failed: %s", hipGetErrorString(e));
    return ncclUnhandledCudaError;
  }
  if (v == kRingVariantWave) comm->waveLaunches++;
  return ncclSuccess;
}

// Dispatch a typed launcher over the kernel element type.
template <class F>
static hipError_t by_kernel_type(int kt, F&& f) {
  switch (kt) {
    case K_U8: return f.template operator()<K_U8>();
    case K_U32: return f.template operator()<K_U32>();
    case K_U64: return f.template operator()<K_U64>();
    case K_F16: return f.template operator()<K_F16>();
    case K_F32: return f.template operator()<K_F32>();
    case K_F64: return f.template operator()<K_F64>();
    case K_BF16: return f.template operator()<K_BF16>();
    case K_F8E4M3: return f.template operator()<K_F8E4M3>();
    case K_F8E5M2: return f.template operator()<K_F8E5M2>();
  }
  return hipErrorInvalidValue;
}


// The cbd partition of a reduce-scatter's block, for the one-hop LL / direct
// reduce-scatters' per-channel fold order: the ring's, under VCCL's protocol
// for the path (LL: the LL ring's cells, enqueue.cc:599; direct: SIMPLE).
static CbdLite rs_cbd(const Task& t, int proto) {
  const CbdPlan p = task_plan(t, proto);
  return CbdLite{p.channelLo, p.channelHi, p.countLo, p.countMid, (int64_t)t.count};
}

// One-hop LL collectives: `ts` holds 1 .. kLLMaxParts calls of one comm with
// the same collective, type and op (fusable) whose lines — all-reduce: the
// bucket's, reduce-scatter / all-gather: one rank's block's — fit one slot;
// they run as one launch on ts[0].stream (the caller orders the other
// streams around it).
static int64_t ll_lines_of(const Task& t) {
  return ((int64_t)t.count * type_size(t.datatype) + 7) / 8;
}
static ncclResult_t launch_ll(const Task* ts, int nTasks, hipEvent_t stop) {
  const Task& t = ts[0];
  ncclComm* comm = t.comm;
  LLWork w{};
  w.comm = comm->devComm;
  w.redArg = t.arg;
  w.redArgPtr = t.argPtr;
  w.redArgBytes = type_size(t.datatype);
  w.preOp = t.devOp == OP_PREMULSUM;
  w.nRanks = comm->nRanks;
  w.rank = comm->rank;
  w.linesPerSlot = comm->llLines;
  w.localBuf = comm->llBuf;
  for (int r = 0; r < comm->nRanks; r++) w.peerBuf[r] = comm->llPeer[r];
  if (nTasks < 1 || nTasks > kLLMaxParts) return ncclInternalError;
  int64_t lines = 0;
  for (int i = 0; i < nTasks; i++) {
    if (ts[i].coll != t.coll) return ncclInternalError;
    w.parts[i].send = (const char*)ts[i].sendbuff;
    w.parts[i].recv = (char*)ts[i].recvbuff;
    w.parts[i].nbytes = (int64_t)ts[i].count * type_size(ts[i].datatype);
    w.parts[i].line0 = lines;
    if (t.coll == kReduceScatter) w.parts[i].cbd = rs_cbd(ts[i], kProtoLL);
    lines += ll_lines_of(ts[i]);
  }
  w.nParts = nTasks;
  w.nLines = lines;
  if (lines > comm->llLines) return ncclInternalError;
  const int kt = t.coll == kAllGather ? K_U8 : kernel_type_of(t.devOp, (int)t.datatype);
  if (kt < 0) return ncclInvalidArgument;
  // A bounded grid (256-thread workgroups, each thread looping over lines):
  // one workgroup per 256 lines, within the comm's CTA bounds (minCTAs /
  // maxCTAs, default 1 / 128), and never above VCCL_LL_MAX_BLOCKS (256): every
  // rank's LL workgroups must be resident at once for the peers' spins to
  // complete, so that co-residency cap is applied LAST (tests that
  // put 8 ranks on ONE GPU lower it).
  int maxBlocks = (int)std::max<int64_t>(1, param_int("LL_MAX_BLOCKS", 256));
  if (comm->shareBlockCap > 0) maxBlocks = std::min(maxBlocks, comm->shareBlockCap);
  int grid = (int)std::max<int64_t>(1, (lines + 255) / 256);
  grid = std::max(std::min(grid, comm->maxCTAs), comm->minCTAs);
  grid = std::max(1, std::min(grid, maxBlocks));
  const int coll = dev_coll(t.coll), devOp = t.coll == kAllGather ? OP_COPY : t.devOp;
  const hipError_t e = by_kernel_type(kt, [&]<int K>() { return ll_launch<K>(coll, devOp, w, grid, t.stream, stop); });
  if (e != hipSuccess) {
    VWARN("LL kernel launch failed: %s", hipGetErrorString(e));
    return ncclUnhandledCudaError;
  }
  return ncclSuccess;
}

// The direct work of one call (direct.hpp): two-shot all-reduce, one-hop
// reduce-scatter / all-gather.  `blkForce` > 0 imposes the block length (a
// fused batch's common geometry, launch_direct).
static ncclResult_t direct_work_of(const Task& t, DirectWork* out, int* ktOut, int* devOpOut,
                                   int64_t blkForce = 0) {
  ncclComm* comm = t.comm;
  const int n = comm->nRanks;
  const bool ag = t.coll == kAllGather;
  const int64_t esz = ag ? 1 : type_size(t.datatype);  // all-gather: bytes
  const int64_t count = ag ? (int64_t)t.count * type_size(t.datatype) : (int64_t)t.count;
  const int64_t eltAlign = std::max<int64_t>(1, 16 / esz);
  auto align_up = [](int64_t x, int64_t a) { return (x + a - 1) / a * a; };
  DirectWork w{};
  w.comm = comm->devComm;
  w.peers = comm->dPeers;
  w.sendbuff = t.sendbuff;
  w.recvbuff = t.recvbuff;
  w.count = (uint64_t)count;
  w.redArg = t.arg;
  w.redArgPtr = t.argPtr;
  w.redArgBytes = type_size(t.datatype);
  w.preOp = t.devOp == OP_PREMULSUM;
  w.nRanks = n;
  w.rank = comm->rank;
  const int64_t regionElts = (comm->dRegionBytes - 16) / esz;
  int64_t shard0;
  if (t.coll == kAllReduce) {
    // Chunk: as many elements as fit one shard per inbox region, a multiple
    // of n x 16 bytes; the shard of the largest chunk is cut into blocks.
    const int64_t chunkMax = regionElts * n / (n * eltAlign) * (n * eltAlign);
    w.chunkElts = std::min<int64_t>(count, chunkMax);
    shard0 = direct_shard_elts(w.chunkElts, n, eltAlign);
    // the ring's partition of this bucket: phase 2 folds every element in the
    // order VCCL's ring all-reduce gives it on these channels (ar_chunk_of)
    const CbdPlan p = task_plan(t, kProtoSimple);
    w.cbd = CbdLite{p.channelLo, p.channelHi, p.countLo, p.countMid, count};
    w.arChunk = p.chunkLo;
  } else {
    // Reduce-scatter / all-gather: a chunk is a range of ONE rank's block
    // (count elements) that fits a region; it is cut into blocks directly.
    w.chunkElts = std::min<int64_t>(count, regionElts / eltAlign * eltAlign);
    shard0 = w.chunkElts;
    if (t.coll == kReduceScatter) w.cbd = rs_cbd(t, kProtoSimple);
  }
  w.nChunks = (int)((count + w.chunkElts - 1) / w.chunkElts);
  // Blocks of >= 16 KiB (one 512-thread x 2-pack hunk), at most the cap.
  const int64_t minBlk = (16 << 10) / esz;
  // CTA bounds first, then the co-residency caps (directMaxBlocks,
  // kDirectMaxBlocks) last, so NCCL_MIN_CTAS cannot push past them.
  int64_t nb = (shard0 + minBlk - 1) / minBlk;
  nb = std::max<int64_t>(std::min<int64_t>(nb, comm->maxCTAs), comm->minCTAs);
  nb = std::max<int64_t>(1, std::min<int64_t>({nb, (int64_t)comm->directMaxBlocks, (int64_t)kDirectMaxBlocks}));
  w.blkElts = align_up((shard0 + nb - 1) / nb, eltAlign);
  if (blkForce > 0) {
    if (blkForce < w.blkElts || blkForce % eltAlign) return ncclInternalError;
    w.blkElts = blkForce;
  }
  w.nBlocks = (int)((shard0 + w.blkElts - 1) / w.blkElts);
  w.regionBytes = comm->dRegionBytes;
  if (shard0 * esz > w.regionBytes || w.nBlocks > kDirectMaxBlocks || w.nBlocks < 1)
    return ncclInternalError;
  const int kt = ag ? K_U8 : kernel_type_of(t.devOp, (int)t.datatype);
  if (kt < 0) return ncclInvalidArgument;
  *out = w;
  *ktOut = kt;
  *devOpOut = ag ? OP_COPY : t.devOp;
  return ncclSuccess;
}

// 1 .. kDirectMaxWorks direct calls of one comm with the same collective,
// kernel type and op in one launch on ts[0].stream (the largest part's grid).
// Every part of a batch uses ONE block length (the largest part's): block b
// then covers the same inbox bytes [b * blkElts, (b + 1) * blkElts) in every
// part, so the per-block flags that order a part's region reuse also order
// the next part's (a kernel boundary no longer separates them) — with
// per-part lengths, workgroup b's next-part scatter could overwrite bytes a
// peer's workgroup b' was still folding.
static ncclResult_t launch_direct(const Task* ts, int nTasks, hipEvent_t stop) {
  const Task& t = ts[0];
  if (nTasks < 1 || nTasks > kDirectMaxWorks) return ncclInternalError;
  DirectBatch b{};
  int kt = -1, devOp = -1;
  int64_t blk = 0;
  for (int i = 0; i < nTasks; i++) {
    DirectWork wi;
    int kti, opi;
    NCCLCHECK(direct_work_of(ts[i], &wi, &kti, &opi));
    if (i > 0 && (kti != kt || opi != devOp)) return ncclInternalError;
    kt = kti;
    devOp = opi;
    blk = std::max(blk, wi.blkElts);
  }
  NCCLCHECK(direct_work_of(t, &b.w, &kt, &devOp, nTasks > 1 ? blk : 0));
  for (int i = 1; i < nTasks; i++) {
    DirectWork wi;
    int kti, opi;
    NCCLCHECK(direct_work_of(ts[i], &wi, &kti, &opi, blk));
    b.more[i - 1] = direct_part_of(wi);
    b.w.nBlocks = std::max(b.w.nBlocks, wi.nBlocks);
  }
  b.nParts = nTasks;
  const int coll = dev_coll(t.coll);
  const hipError_t e = by_kernel_type(kt, [&]<int K>() { return direct_launch<K>(coll, devOp, b, t.stream, stop); });
  if (e != hipSuccess) {
    VWARN("direct kernel launch failed: %s", hipGetErrorString(e));
    return ncclUnhandledCudaError;
  }
  return ncclSuccess;
}

// A call's path: select_algo on the comm's thresholds.
static int choose_algo(const Task& t) {
  return select_algo(policy_of(t.comm), t.coll, type_size(t.datatype), (int64_t)t.count);
}

static ncclResult_t launch_task(const Task& t) {
  int old = -1;
  HIPCHECK(hipGetDevice(&old));
  if (old != t.comm->device) HIPCHECK(hipSetDevice(t.comm->device));
  // A one-rank in-place call without a preOp enqueues nothing (onerank.cu:
  // 47-83): no stream bookkeeping either.
  if (t.comm->nRanks == 1 && t.sendbuff == t.recvbuff &&
      (is_copy_coll(t.coll) || t.devOp != OP_PREMULSUM)) {
    t.comm->opCount++;
    if (old != t.comm->device) (void)hipSetDevice(old);
    return ncclSuccess;
  }
  // One rank: the copy / PreMulSum kernel goes straight onto the caller's
  // stream with no cross-stream ordering, as ncclLaunchOneRank does
  // (enqueue.cc:2386-2388 — it bypasses the plan and the strong stream).
  if (t.comm->nRanks == 1) {
    const ncclResult_t r = launch_one_rank(t);
    t.comm->opCount++;
    if (old != t.comm->device) (void)hipSetDevice(old);
    return r;
  }
  CaptureState cs{false, 0};
  ncclResult_t r = stream_order(t.comm, t.stream, &cs);
  if (r == ncclSuccess) {
    const int algo = choose_algo(t);
    const hipEvent_t stop = stop_event(t.comm, cs);
    r = algo == kAlgoLL ? launch_ll(&t, 1, stop)
        : algo == kAlgoDirect ? launch_direct(&t, 1, stop) : launch_ring(&t, 1, algo == kAlgoRingLL128, stop);
  }
  if (r == ncclSuccess) r = stream_mark(t.comm, t.stream, cs);
  t.comm->opCount++;
  if (old != t.comm->device) (void)hipSetDevice(old);
  return r;
}

// Group aggregation (enqueue.cc:352-508 ncclPrepareTasks / :518-769
// scheduleCollTasksToPlan pack a group's collectives into one kernel plan,
// common.h:260-293 RunWorkBatch runs a plan's works in order): a run of
// consecutive calls of one comm that take the same algorithm — LL, direct or
// ring — with the same collective, kernel type and op becomes ONE launch
// carrying up to 16 works (LL all-reduces: lines within one slot).  A ZeRO
// loop's bucketed reduce-scatters launch once per group.  The decision
// depends only on the call sequence, never on streams, so every rank fuses
// identically.  The fused launch runs on the first task's stream; the other
// tasks' streams are joined before it and wait for it after.
static int fuse_key_algo(const Task& t) { return t.comm->nRanks > 1 ? choose_algo(t) : -1; }
// Same comm, collective, kernel type and op (the caller compares the paths).
static bool fusable(const Task& a, const Task& b) {
  if (a.comm != b.comm || a.coll != b.coll) return false;
  if (is_copy_coll(a.coll)) return true;  // byte copies: any type
  return a.datatype == b.datatype && a.devOp == b.devOp && a.arg == b.arg && a.argPtr == b.argPtr;
}
static int max_parts(int algo) {
  return algo == kAlgoLL ? kLLMaxParts : algo == kAlgoDirect ? kDirectMaxWorks : kRingMaxWorks;
}

// Runs of calls of one comm, each run one launch (1 .. max_parts calls), in
// order on the first task's stream; the other tasks' streams are joined
// before the first launch and wait for the last.
static ncclResult_t launch_runs(const std::vector<std::vector<Task>>& runs, const std::vector<int>& algos) {
  ncclComm* comm = runs[0][0].comm;
  const hipStream_t s0 = runs[0][0].stream;
  int old = -1;
  HIPCHECK(hipGetDevice(&old));
  if (old != comm->device) HIPCHECK(hipSetDevice(comm->device));
  std::vector<hipStream_t> others;
  size_t nTasks = 0;
  for (const auto& run : runs) {
    nTasks += run.size();
    for (const Task& t : run)
      if (t.stream != s0 && std::find(others.begin(), others.end(), t.stream) == others.end())
        others.push_back(t.stream);
  }
  CaptureState cs{false, 0};
  ncclResult_t r = stream_order(comm, s0, &cs);
  for (hipStream_t s : others) {
    if (r != ncclSuccess) break;
    if (hipEventRecord(comm->joinEvent, s) != hipSuccess ||
        hipStreamWaitEvent(s0, comm->joinEvent, 0) != hipSuccess)
      r = ncclUnhandledCudaError;
  }
  bool bound = false;  // a launch of this sequence carries the ordering event
  for (size_t k = 0; k < runs.size() && r == ncclSuccess; k++) {
    // every launch goes onto s0 (the launchers use their first task's
    // stream): runs of one comm must never overlap on its channels
    std::vector<Task> run = runs[k];
    for (Task& t : run) t.stream = s0;
    const int n = (int)run.size(), algo = algos[k];
    const hipEvent_t stop = stop_event(comm, cs);  // every launch: the last binding is the group's end
    r = algo == kAlgoLL ? launch_ll(run.data(), n, stop)
        : algo == kAlgoDirect ? launch_direct(run.data(), n, stop)
                              : launch_ring(run.data(), n, algo == kAlgoRingLL128, stop);
    bound |= r == ncclSuccess && stop != nullptr;
    if (n > 1) comm->fusedLaunches++;
  }
  if (r == ncclSuccess) {
    r = stream_mark(comm, s0, cs);
  } else if (bound) {
    // an earlier run already bound the ordering event to its
    // kernel on s0, so the next call from another stream must still wait on
    // it even though a later run of this sequence failed
    comm->lastStream = s0;
    comm->hasLastLaunch = true;
    comm->lastUnmarked = false;
  }
  const hipEvent_t done = stream_last_event(comm, cs);
  for (hipStream_t s : others)
    if (r == ncclSuccess && hipStreamWaitEvent(s, done, 0) != hipSuccess)
      r = ncclUnhandledCudaError;
  comm->opCount += nTasks;
  if (old != comm->device) (void)hipSetDevice(old);
  return r;
}

// A group's calls of one comm (`idx`, in call order, nRanks > 1) on VCCL's
// plan for them (group_plan): each (func, op, type) aggregate takes the path
// select_algo gives its summed count, as ncclPrepareTasks gives getAlgoInfo's
// choice to every member; every call is placed on the plan's channels under
// its path's protocol — the ring, LL128 ring and direct path fold every
// element in the order of that place, the LL reduce-scatter per channel of
// it, and LL calls shift the running channel cursor as in VCCL — and the
// calls launch in plan order, consecutive calls of one plan and path with the
// same collective, type and op fused (<= max_parts; LL calls while their lines
// fit one slot).
static ncclResult_t launch_planned(std::vector<Task>& tasks, const std::vector<int>& idx) {
  ncclComm* comm = tasks[idx[0]].comm;
  std::vector<GroupTask> g;
  for (int j : idx) {
    const Task& t = tasks[j];
    const bool ag = is_copy_coll(t.coll);
    const int tsz = type_size(t.datatype);
    const int op = ag ? OP_SUM : t.devOp;  // AG: int8 copies (enqueue.cc:2400-2404)
    const int dt = ag ? (int)ncclInt8 : (int)t.datatype;
    const int kt = ag ? K_U8 : kernel_type_of(t.devOp, (int)t.datatype);
    g.push_back(GroupTask{t.coll, ag ? (int64_t)t.count * tsz : (int64_t)t.count, ag ? 1 : tsz,
                          (t.coll * 16 + op) * 32 + dt, (t.coll * 16 + op) * 32 + kt});
  }
  GroupPlanOut plan;
  const AlgoPolicy pol = policy_of(comm);
  group_plan(g, comm->nRanks, comm->nChannels,
             PlanGeometry{comm->stepBytes, comm->nThreads, comm->ll128StepBytes, comm->ll128Threads}, &pol, &plan);
  for (size_t k = 0; k < idx.size(); k++) {
    if (plan.planOf[k] < 0) return ncclInternalError;
    tasks[idx[k]].planned = true;
    tasks[idx[k]].plan = plan.cbd[k];
  }
  std::vector<std::vector<Task>> runs;
  std::vector<int> runAlgo, runPlan;
  std::vector<int64_t> runLines;
  static const bool fusePlanned = param_int("GROUP_PLAN_FUSE", 1) != 0;
  for (int k : plan.order) {
    const Task& t = tasks[idx[k]];
    const int a = plan.algo[k];
    const int64_t lines = a == kAlgoLL ? ll_lines_of(t) : 0;
    if (fusePlanned && !runs.empty() && runPlan.back() == plan.planOf[k] && runAlgo.back() == a &&
        runs.back().size() < (size_t)max_parts(a) && fusable(runs.back()[0], t) &&
        (a != kAlgoLL || runLines.back() + lines <= comm->llLines)) {
      runs.back().push_back(t);
      runLines.back() += lines;
      continue;
    }
    runs.push_back({t});
    runAlgo.push_back(a);
    runPlan.push_back(plan.planOf[k]);
    runLines.push_back(lines);
  }
  return launch_runs(runs, runAlgo);
}

static ncclResult_t launch_group(std::vector<Task>& tasks) {
  ncclResult_t ret = ncclSuccess;
  const size_t n = tasks.size();
  std::vector<char> done(n, 0);
  const bool fuse = param_int("GROUP_FUSE", 1) != 0;
  // VCCL_GROUP_PLAN=0: every call keeps its own path and the partition of a
  // call planned alone (runs of consecutive fusable calls still fuse)
  const bool plan = fuse && param_int("GROUP_PLAN", 1) != 0;
  std::vector<int> algo(n, -1);
  if (fuse && !plan)
    for (size_t i = 0; i < n; i++) algo[i] = fuse_key_algo(tasks[i]);
  for (size_t i = 0; i < n; i++) {
    if (done[i]) continue;
    ncclResult_t r;
    if (plan && tasks[i].comm->nRanks > 1) {
      // every call of this comm in the group, one VCCL plan
      std::vector<int> idx;
      for (size_t j = i; j < n; j++)
        if (!done[j] && tasks[j].comm == tasks[i].comm) idx.push_back((int)j);
      for (int j : idx) done[j] = 1;
      r = launch_planned(tasks, idx);
    } else if (algo[i] >= 0) {
      std::vector<Task> batch{tasks[i]};
      int64_t lines = ll_lines_of(tasks[i]);
      for (size_t j = i + 1; j < n && batch.size() < (size_t)max_parts(algo[i]); j++) {
        if (done[j] || tasks[j].comm != tasks[i].comm) continue;
        if (algo[j] != algo[i] || !fusable(tasks[i], tasks[j])) break;
        if (algo[i] == kAlgoLL) {
          if (lines + ll_lines_of(tasks[j]) > tasks[i].comm->llLines) break;
          lines += ll_lines_of(tasks[j]);
        }
        batch.push_back(tasks[j]);
        done[j] = 1;
      }
      r = batch.size() == 1 ? launch_task(tasks[i]) : launch_runs({batch}, {algo[i]});
    } else {
      r = launch_task(tasks[i]);
    }
    if (ret == ncclSuccess) ret = r;
  }
  return ret;
}

static ncclResult_t enqueue_check_impl(int coll, const char* name, const void* sendbuff,
                                       void* recvbuff, size_t count, ncclDataType_t dt,
                                       ncclRedOp_t op, ncclComm* comm, hipStream_t stream, int root) {
  NCCLCHECK(comm_check(comm, name));
  if ((coll == kBroadcast || coll == kReduce) && (root < 0 || root >= comm->nRanks)) {  // argcheck.cc:66-69
    VWARN("%s : invalid root %d (root should be in the 0..%d range)", name, root, comm->nRanks);
    return ncclInvalidArgument;
  }
  NCCLCHECK(args_check(comm, name, dt, op, !is_copy_coll(coll)));
  VINFO("%s: opCount %lx sendbuff %p recvbuff %p count %zu datatype %d op %d comm %p [nranks=%d] stream %p",
        name, (unsigned long)comm->opCount, sendbuff, recvbuff, count, (int)dt, (int)op,
        (void*)comm, comm->nRanks, (void*)stream);
  if (count == 0) return ncclSuccess;  // enqueue.cc:2372
  // broadcast: a non-root's sendbuff is never read, reduce: a non-root's
  // recvbuff never written (argcheck.cc:76-81)
  if ((!recvbuff && !(coll == kReduce && comm->rank != root)) ||
      (!sendbuff && !(coll == kBroadcast && comm->rank != root))) {
    VWARN("%s : NULL buffer", name);
    return ncclInvalidArgument;
  }
  Task t{};
  t.coll = coll;
  t.sendbuff = sendbuff;
  t.recvbuff = recvbuff;
  t.count = count;
  t.datatype = dt;
  t.comm = comm;
  t.stream = stream;
  if (!is_copy_coll(coll)) NCCLCHECK(resolve_op(comm, op, dt, &t.devOp, &t.arg, &t.argPtr));
  else t.devOp = OP_COPY;
  t.root = root;
  if (*(volatile int*)comm->errorFlag) {
    const ncclResult_t e = error_word_result(comm);
    comm->asyncError = e;
    return e;
  }
  if (tl_groupDepth > 0) {
    tl_tasks.push_back(t);
    return ncclSuccess;
  }
  return launch_task(t);
}

// ncclGroupErrCheck (enqueue.cc:2516): inside a group the first failing call
// is remembered, and the outermost ncclGroupEnd then launches nothing of the
// group and returns that error (group.cc:528, :591).
static ncclResult_t enqueue_check(int coll, const char* name, const void* sendbuff, void* recvbuff,
                                  size_t count, ncclDataType_t dt, ncclRedOp_t op, ncclComm* comm,
                                  hipStream_t stream, int root = 0) {
  const ncclResult_t r =
      enqueue_check_impl(coll, name, sendbuff, recvbuff, count, dt, op, comm, stream, root);
  if (r != ncclSuccess && tl_groupDepth > 0 && tl_groupError == ncclSuccess) tl_groupError = r;
  return r;
}

}  // namespace vccl

using namespace vccl;

#define VCCL_EXPORT extern "C" __attribute__((visibility("default")))

// Out-of-scope calls of the reference API (include/nccl.h):
// exported so a binary linked against libnccl loads, never silently wrong.
static ncclResult_t out_of_scope(const char* name) {
  VWARN("%s is not part of this library's scope (AllReduce / ReduceScatter / AllGather / Broadcast / Reduce only)",
        name);
  return ncclInvalidUsage;
}

VCCL_EXPORT ncclResult_t ncclSend(const void*, size_t, ncclDataType_t, int, ncclComm_t,
                                  hipStream_t) {
  return out_of_scope("ncclSend");
}
VCCL_EXPORT ncclResult_t ncclRecv(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) {
  return out_of_scope("ncclRecv");
}
VCCL_EXPORT ncclResult_t ncclAllToAll(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) {
  return out_of_scope("ncclAllToAll");
}
VCCL_EXPORT ncclResult_t ncclAllToAllv(const void*, const size_t[], const size_t[], void*, const size_t[],
                                       const size_t[], ncclDataType_t, ncclComm_t, hipStream_t) {
  return out_of_scope("ncclAllToAllv");
}

#define VCCL_ALIAS(name) __attribute__((alias(#name), visibility("default")))

VCCL_EXPORT ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count,
                                       ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm,
                                       hipStream_t stream) {
  return enqueue_check(kAllReduce, "AllReduce", sendbuff, recvbuff, count, datatype, op, comm,
                       stream);
}

VCCL_EXPORT ncclResult_t ncclReduceScatter(const void* sendbuff, void* recvbuff, size_t recvcount,
                                           ncclDataType_t datatype, ncclRedOp_t op,
                                           ncclComm_t comm, hipStream_t stream) {
  return enqueue_check(kReduceScatter, "ReduceScatter", sendbuff, recvbuff, recvcount, datatype,
                       op, comm, stream);
}

VCCL_EXPORT ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount,
                                       ncclDataType_t datatype, ncclComm_t comm,
                                       hipStream_t stream) {
  return enqueue_check(kAllGather, "AllGather", sendbuff, recvbuff, sendcount, datatype, ncclSum,
                       comm, stream);
}

// broadcast.h / collectives.cc:125-158: the ring broadcast, count elements of
// datatype from root's sendbuff to every rank's recvbuff (bytes on the wire).
VCCL_EXPORT ncclResult_t ncclBroadcast(const void* sendbuff, void* recvbuff, size_t count,
                                       ncclDataType_t datatype, int root, ncclComm_t comm, hipStream_t stream) {
  return enqueue_check(kBroadcast, "Broadcast", sendbuff, recvbuff, count, datatype, ncclSum, comm, stream,
                       root);
}
// reduce.h / collectives.cc:132-143: the ring reduce, count elements of
// datatype reduced from every rank's sendbuff into root's recvbuff (a
// non-root's recvbuff is never written, argcheck.cc:79-81)
VCCL_EXPORT ncclResult_t ncclReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                                    ncclRedOp_t op, int root, ncclComm_t comm, hipStream_t stream) {
  return enqueue_check(kReduce, "Reduce", sendbuff, recvbuff, count, datatype, op, comm, stream, root);
}
// collectives.cc:112-123: the in-place broadcast
VCCL_EXPORT ncclResult_t ncclBcast(void* buff, size_t count, ncclDataType_t datatype, int root, ncclComm_t comm,
                                   hipStream_t stream) {
  return ncclBroadcast(buff, buff, count, datatype, root, comm, stream);
}

VCCL_EXPORT ncclResult_t ncclGroupStart(void) {
  tl_groupDepth++;
  return ncclSuccess;
}

VCCL_EXPORT ncclResult_t ncclGroupEnd(void) {
  if (tl_groupDepth == 0) {
    VWARN("ncclGroupEnd: not in a group call.");
    return ncclInvalidUsage;
  }
  if (--tl_groupDepth > 0) return ncclSuccess;
  const ncclResult_t err = tl_groupError;
  tl_groupError = ncclSuccess;
  std::vector<Task> tasks;
  tasks.swap(tl_tasks);
  if (err != ncclSuccess) {  // a call of the group failed: drop the whole group
    VWARN("ncclGroupEnd: a call in the group failed (%d); %zu queued collectives not launched",
          (int)err, tasks.size());
    return err;
  }
  return launch_group(tasks);
}

// nccl.h.in:472-473: ends the group like ncclGroupEnd but launches nothing;
// the run-time estimate needs the tuner's cost model (out of scope).
VCCL_EXPORT ncclResult_t ncclGroupSimulateEnd(ncclSimInfo_t* simInfo) {
  if (tl_groupDepth == 0) {
    VWARN("ncclGroupSimulateEnd: not in a group call.");
    return ncclInvalidUsage;
  }
  if (--tl_groupDepth > 0) return ncclSuccess;
  tl_groupError = ncclSuccess;
  tl_tasks.clear();
  if (simInfo) simInfo->estimatedTime = NCCL_UNDEF_FLOAT;
  return out_of_scope("ncclGroupSimulateEnd");
}

VCCL_EXPORT ncclResult_t ncclRedOpCreatePreMulSum(ncclRedOp_t* op, void* scalar,
                                                  ncclDataType_t datatype,
                                                  ncclScalarResidence_t residence,
                                                  ncclComm_t comm) {
  NCCLCHECK(comm_check(comm, "ncclRedOpCreatePreMulSum"));
  if (!op || !scalar) return ncclInvalidArgument;
  const int sz = type_size(datatype);
  if (sz < 1) return ncclInvalidArgument;
  int ix = -1;
  for (int i = 0; i < (int)comm->userOps.size(); i++)
    if (comm->userOps[i].freeNext != -1) { ix = i; break; }
  if (ix < 0) {
    comm->userOps.push_back(UserRedOp{});
    ix = (int)comm->userOps.size() - 1;
  }
  UserRedOp& u = comm->userOps[ix];
  u.freeNext = -1;
  u.datatype = datatype;
  u.devOp = OP_PREMULSUM;
  if (residence == ncclScalarHostImmediate) {
    u.argIsPtr = false;
    u.arg = 0;
    memcpy(&u.arg, scalar, (size_t)sz);
  } else {
    u.argIsPtr = true;
    u.arg = (uint64_t)(uintptr_t)scalar;
  }
  *op = (ncclRedOp_t)((int)ncclNumOps + ix);
  return ncclSuccess;
}

VCCL_EXPORT ncclResult_t ncclRedOpDestroy(ncclRedOp_t op, ncclComm_t comm) {
  if (0 <= (int)op && (int)op < (int)ncclNumOps) {
    VWARN("ncclRedOpDestroy : operator is a NCCL builtin.");
    return ncclInvalidArgument;
  }
  if ((int)op < 0) {
    VWARN("ncclRedOpDestroy :  operator is garbage.");
    return ncclInvalidArgument;
  }
  if (comm == nullptr) {
    VWARN("ncclRedOpDestroy : invalid communicator passed.");
    return ncclInvalidArgument;
  }
  NCCLCHECK(comm_check(comm, "ncclRedOpDestroy"));
  const int ix = (int)op - (int)ncclNumOps;
  if (ix >= (int)comm->userOps.size() || comm->userOps[ix].freeNext != -1) {
    VWARN("ncclRedOpDestroy : operator unknown to this communicator.");
    return ncclInvalidArgument;
  }
  comm->userOps[ix].freeNext = 0;  // free
  return ncclSuccess;
}

VCCL_EXPORT ncclResult_t vcclHostToDevRedOp(ncclRedOp_t op, ncclDataType_t datatype, int nRanks,
                                            int* devOp, uint64_t* opArg) {
  if (!devOp || !opArg || nRanks < 1) return ncclInvalidArgument;
  if ((int)datatype < 0 || (int)datatype >= (int)ncclNumTypes) return ncclInvalidArgument;
  return host_to_dev_redop(op, datatype, nRanks, devOp, opArg);
}

VCCL_EXPORT const char* vcclBuildInfo(void) {
#define VCCL_STR2(x) #x
#define VCCL_STR(x) VCCL_STR2(x)
  return "vccl-mi355x " __DATE__ " gfx950; one-shot LL / two-shot direct / SIMPLE ring / LL128 ring "
         "(" VCCL_STR(VCCL_LL128_LINE) "-byte lines) over xGMI (uncached receiver buffers); "
         "reduce-copy 16B packs; VCCL group plans";
}

extern "C" {
ncclResult_t pncclAllReduce(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) VCCL_ALIAS(ncclAllReduce);
ncclResult_t pncclReduceScatter(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t,
                                ncclComm_t, hipStream_t) VCCL_ALIAS(ncclReduceScatter);
ncclResult_t pncclAllGather(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t)
    VCCL_ALIAS(ncclAllGather);
ncclResult_t pncclGroupStart(void) VCCL_ALIAS(ncclGroupStart);
ncclResult_t pncclGroupEnd(void) VCCL_ALIAS(ncclGroupEnd);
ncclResult_t pncclGroupSimulateEnd(ncclSimInfo_t*) VCCL_ALIAS(ncclGroupSimulateEnd);
ncclResult_t pncclAllToAll(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t)
    VCCL_ALIAS(ncclAllToAll);
ncclResult_t pncclAllToAllv(const void*, const size_t[], const size_t[], void*, const size_t[], const size_t[],
                            ncclDataType_t, ncclComm_t, hipStream_t) VCCL_ALIAS(ncclAllToAllv);
ncclResult_t pncclRedOpCreatePreMulSum(ncclRedOp_t*, void*, ncclDataType_t, ncclScalarResidence_t,
                                       ncclComm_t) VCCL_ALIAS(ncclRedOpCreatePreMulSum);
ncclResult_t pncclRedOpDestroy(ncclRedOp_t, ncclComm_t) VCCL_ALIAS(ncclRedOpDestroy);
ncclResult_t pncclReduce(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t,
                         hipStream_t) VCCL_ALIAS(ncclReduce);
ncclResult_t pncclBcast(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t)
    VCCL_ALIAS(ncclBcast);
ncclResult_t pncclBroadcast(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t,
                            hipStream_t) VCCL_ALIAS(ncclBroadcast);
ncclResult_t pncclSend(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t)
    VCCL_ALIAS(ncclSend);
ncclResult_t pncclRecv(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t)
    VCCL_ALIAS(ncclRecv);
}

extern "C" ncclResult_t vcclCommCollAlgo(ncclComm_t comm, int coll, size_t count,
                                         ncclDataType_t datatype, int* algo) {
  NCCLCHECK(comm_check(comm, "vcclCommCollAlgo"));
  if (!algo || coll < kAllReduce || coll > kReduce || type_size(datatype) < 1) return ncclInvalidArgument;
  if (comm->nRanks == 1) {
    *algo = vcclAlgoOneRank;
    return ncclSuccess;
  }
  Task t{};
  t.comm = comm;
  t.coll = coll;  // the public codes are the Coll values (vccl_ext.h)
  t.count = count;
  t.datatype = datatype;
  const int a = choose_algo(t);
  *algo = a == kAlgoLL ? vcclAlgoLL
          : a == kAlgoDirect ? vcclAlgoDirect : a == kAlgoRingLL128 ? vcclAlgoLL128 : vcclAlgoRing;
  return ncclSuccess;
}

extern "C" __attribute__((visibility("default"))) ncclResult_t vcclRingPartition(
    int coll, size_t count, ncclDataType_t datatype, int nRanks, int nChannels, int proto,
    size_t stepBytes, int nThreads, int64_t* out) {
  if (!out || coll < kAllReduce || coll > kReduce || type_size(datatype) < 1 || nRanks < 1 ||
      nChannels < 1 || nChannels > kMaxChannels || count == 0 || stepBytes < 4096 || nThreads < 64 ||
      (proto != kProtoSimple && proto != kProtoLL128 && proto != kProtoLL))
    return ncclInvalidArgument;
  const int c = coll;
  const int64_t esz = is_copy_coll(c) ? 1 : type_size(datatype);
  const int64_t cnt = is_copy_coll(c) ? (int64_t)count * type_size(datatype) : (int64_t)count;
  const CbdPlan p = cbd_schedule(c, cnt, esz, nRanks, nChannels, proto, (int64_t)stepBytes, nThreads);
  const int64_t v[8] = {p.channelLo, p.channelHi, p.countLo, p.countMid,
                        p.countHi,   p.chunkLo,   p.chunkMid, p.chunkHi};
  memcpy(out, v, sizeof(v));
  return ncclSuccess;
}

extern "C" __attribute__((visibility("default"))) ncclResult_t vcclRingChunkOf(
    size_t count, ncclDataType_t datatype, int nRanks, int nChannels, size_t slotBytes, int nThreads,
    size_t i, int64_t* out) {
  if (!out || type_size(datatype) < 1 || nRanks < 1 || nChannels < 1 || nChannels > kMaxChannels ||
      count == 0 || i >= count || slotBytes < 4096 || nThreads < 64)
    return ncclInvalidArgument;
  const int64_t esz = type_size(datatype);
  const CbdPlan p = cbd_schedule(kAllReduce, (int64_t)count, esz, nRanks, nChannels, kProtoSimple,
                                 (int64_t)slotBytes, nThreads);
  const CbdLite cbd{p.channelLo, p.channelHi, p.countLo, p.countMid, (int64_t)count};
  int k;
  int64_t end;
  out[0] = ar_chunk_of(cbd, p.chunkLo, nRanks, std::max<int64_t>(1, 16 / esz), (int64_t)i, &k, &end);
  out[1] = k;
  out[2] = end;
  return ncclSuccess;
}

// vccl_ext.h: the group planner on explicit inputs (host only).
static ncclResult_t group_plan_export(int nCalls, const int* colls, const size_t* counts, const int* datatypes,
                                      const int* ops, int nRanks, int nChannels, const PlanGeometry& geo,
                                      const AlgoPolicy* pol, int* algos, int* order, int* planOf, int64_t* cbd) {
  if (nCalls < 1 || !colls || !counts || !datatypes || !ops || !order || !planOf || !cbd || nRanks < 1 ||
      nChannels < 1 || nChannels > kMaxChannels || geo.stepBytes < 4096 || geo.nThreads < 64 ||
      geo.ll128StepBytes < 1920 * 16 || geo.ll128Threads < 64)
    return ncclInvalidArgument;
  std::vector<GroupTask> g;
  for (int i = 0; i < nCalls; i++) {
    const ncclDataType_t dt = (ncclDataType_t)datatypes[i];
    const int tsz = type_size(dt);
    if (colls[i] < kAllReduce || colls[i] > kReduce || tsz < 1 || counts[i] == 0) return ncclInvalidArgument;
    const int c = colls[i];
    const bool ag = is_copy_coll(c);
    int devOp = OP_SUM;
    uint64_t arg = 0;
    if (!ag) NCCLCHECK(host_to_dev_redop((ncclRedOp_t)ops[i], dt, nRanks, &devOp, &arg));
    const int kt = ag ? K_U8 : kernel_type_of(devOp, (int)dt);
    if (kt < 0) return ncclInvalidArgument;
    g.push_back(GroupTask{c, ag ? (int64_t)counts[i] * tsz : (int64_t)counts[i], ag ? 1 : tsz,
                          (c * 16 + devOp) * 32 + (ag ? (int)ncclInt8 : (int)dt), (c * 16 + devOp) * 32 + kt});
  }
  GroupPlanOut p;
  group_plan(g, nRanks, nChannels, geo, pol, &p);
  for (int i = 0; i < nCalls; i++) {
    order[i] = p.order[i];
    planOf[i] = p.planOf[i];
    if (algos) {
      const int a = p.algo[i];
      algos[i] = a == kAlgoLL ? vcclAlgoLL : a == kAlgoDirect ? vcclAlgoDirect
                 : a == kAlgoRingLL128 ? vcclAlgoLL128 : vcclAlgoRing;
    }
    const CbdPlan& q = p.cbd[i];
    const int64_t v[8] = {q.channelLo, q.channelHi, q.countLo, q.countMid, q.countHi, q.chunkLo, q.chunkMid, q.chunkHi};
    memcpy(cbd + 8 * (size_t)i, v, sizeof(v));
  }
  return ncclSuccess;
}

extern "C" __attribute__((visibility("default"))) ncclResult_t vcclGroupPlan(
    int nCalls, const int* colls, const size_t* counts, const int* datatypes, const int* ops, int nRanks,
    int nChannels, size_t stepBytes, int nThreads, int* order, int* planOf, int64_t* cbd) {
  const PlanGeometry geo{(int64_t)stepBytes, nThreads, 120 * 640 * 8, 640};
  return group_plan_export(nCalls, colls, counts, datatypes, ops, nRanks, nChannels, geo, nullptr, nullptr, order,
                           planOf, cbd);
}

extern "C" __attribute__((visibility("default"))) ncclResult_t vcclGroupPlanEx(
    int nCalls, const int* colls, const size_t* counts, const int* datatypes, const int* ops, int nRanks,
    int nChannels, const int64_t* geometry, const int64_t* policy, int* algos, int* order, int* planOf,
    int64_t* cbd) {
  if (!geometry) return ncclInvalidArgument;
  const PlanGeometry geo{geometry[0], geometry[1], geometry[2], geometry[3]};
  AlgoPolicy pol;
  if (policy) {
    if (policy[0] < 0 || policy[0] > 4) return ncclInvalidArgument;
    pol.nRanks = nRanks;
    pol.algoForce = (int)policy[0];
    pol.llSlotBytes = policy[1];
    pol.llMax = (uint64_t)policy[2];
    pol.llRsAgMax = (uint64_t)policy[3];
    pol.ll128 = policy[4] != 0;
    pol.ll128Min = (uint64_t)policy[5];
    pol.ll128Max = (uint64_t)policy[6];
    pol.direct = policy[7] != 0;
    pol.directMax = (uint64_t)policy[8];
    pol.directRsAgMax = (uint64_t)policy[9];
  }
  return group_plan_export(nCalls, colls, counts, datatypes, ops, nRanks, nChannels, geo, policy ? &pol : nullptr,
                           algos, order, planOf, cbd);
}

// vccl_ext.h: the path every call of a group would take on this comm (its
// aggregate's, as launch_planned lays the group out); no launch.
extern "C" ncclResult_t vcclCommGroupAlgos(ncclComm_t comm, int nCalls, const int* colls, const size_t* counts,
                                           const int* datatypes, const int* ops, int* algos) {
  NCCLCHECK(comm_check(comm, "vcclCommGroupAlgos"));
  if (nCalls < 1 || !algos) return ncclInvalidArgument;
  if (comm->nRanks == 1) {
    for (int i = 0; i < nCalls; i++) algos[i] = vcclAlgoOneRank;
    return ncclSuccess;
  }
  std::vector<int> order(nCalls), planOf(nCalls);
  std::vector<int64_t> cbd(8 * (size_t)nCalls);
  const AlgoPolicy pol = policy_of(comm);
  // without LL128 FIFOs no call takes the LL128 ring: its geometry is moot
  const PlanGeometry geo{comm->stepBytes, comm->nThreads,
                         comm->ll128StepBytes > 0 ? comm->ll128StepBytes : 120 * 640 * 8,
                         comm->ll128StepBytes > 0 ? comm->ll128Threads : 640};
  return group_plan_export(nCalls, colls, counts, datatypes, ops, comm->nRanks, comm->nChannels, geo, &pol, algos,
                           order.data(), planOf.data(), cbd.data());
}

extern "C" ncclResult_t vcclCommSetAlgo(ncclComm_t comm, int algo) {
  NCCLCHECK(comm_check(comm, "vcclCommSetAlgo"));
  switch (algo) {
    case -1: comm->algoForce = 0; return ncclSuccess;
    case vcclAlgoRing: comm->algoForce = 1; return ncclSuccess;
    case vcclAlgoLL: comm->algoForce = 2; return ncclSuccess;
    case vcclAlgoDirect: comm->algoForce = 3; return ncclSuccess;
    case vcclAlgoLL128: comm->algoForce = 4; return ncclSuccess;  // SIMPLE ring without LL128 buffers
  }
  return ncclInvalidArgument;
}

extern "C" ncclResult_t vcclCommRingTrace(ncclComm_t comm, void* hostBuf, size_t bytes, int* nChannels,
                                          int* cap) {
  NCCLCHECK(comm_check(comm, "vcclCommRingTrace"));
  if (nChannels) *nChannels = comm->nChannels;
  if (cap) *cap = comm->ringTraceCap;
  if (!comm->ringTrace) return ncclInvalidUsage;
  const size_t need = (size_t)comm->nChannels * comm->ringTraceCap * sizeof(RingTraceRec);
  if (!hostBuf || bytes < need) return ncclInvalidArgument;
  int old = -1;
  HIPCHECK(hipGetDevice(&old));
  if (old != comm->device) HIPCHECK(hipSetDevice(comm->device));
  const hipError_t e = hipMemcpy(hostBuf, comm->ringTrace, need, hipMemcpyDeviceToHost);
  if (e == hipSuccess) (void)hipMemset(comm->ringTrace, 0, need);
  if (old != comm->device) (void)hipSetDevice(old);
  return e == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

extern "C" ncclResult_t vcclCommLaunchStats(ncclComm_t comm, unsigned long long* collectives,
                                            unsigned long long* fusedLaunches) {
  NCCLCHECK(comm_check(comm, "vcclCommLaunchStats"));
  if (collectives) *collectives = comm->opCount;
  if (fusedLaunches) *fusedLaunches = comm->fusedLaunches;
  return ncclSuccess;
}
