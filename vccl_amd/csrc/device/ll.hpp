// Low-latency (LL) all-reduce for small buckets, MI355X-native.
//
// Reference: the intra-node "tree" all-reduce over the LL protocol
// (all_reduce.h:148-229 runTreeSplit, prims_ll.h:89-128, 224-298): the tree is
// a chain (graph/connect.cc:64-65), data moves in 16-byte lines carrying two
// {4 B data, 4 B flag} halves (device.h:46-59), flag = step+1, the receiver
// polls the line itself (no separate flag / fence), each hop computes
// peer (+) own, the root applies postOp and the result is broadcast back down.
//
// MI355X design: the 8 GPUs are fully connected by xGMI, so instead of
// 2(n-1) dependent hops the bucket moves ONE hop: every rank writes its input,
// as LL lines tagged with the call's epoch, into its slot of every peer's LL
// buffer (sc0 sc1 write-through 16-byte stores; each 8-byte half is one
// granule), then every rank folds all n inputs locally in the reference's
// chain order — x_0 (+) (x_1 (+) (... (+) x_{n-1})), preOp on every input,
// postOp once — so every rank produces the chain-tree result bit-identically.
// Buffers are double-buffered by epoch parity: a peer can only run one call
// ahead of us (it needs our contribution to finish), so parity reuse is safe
// and no buffer is ever cleared.
//
// Group aggregation (the reference's planner packing several collectives of
// one ncclGroupStart/End into one kernel, enqueue.cc:352-508 / :518-769): one
// launch carries up to kLLMaxParts all-reduces of the same type and op; part
// i occupies lines [line0_i, line0_i + ceil(bytes_i / 8)) of the slot, so the
// whole batch costs one hop and one epoch.
#pragma once
#include "coll_types.hpp"
#include "reduce_copy.hpp"
#include "ring_types.hpp"

namespace vccl {

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// 8 data bytes of element stream `p` (bytes [8*line, 8*line+8)), zero padded.
__device__ __forceinline__ uint64_t ll_load8(const char* p, int64_t line, int64_t nbytes) {
  const int64_t b = line * 8;
  if (b + 8 <= nbytes && (((uintptr_t)p + b) & 7) == 0) return *(const uint64_t*)(p + b);
  uint64_t v = 0;
  for (int k = 0; k < 8 && b + k < nbytes; k++) v |= (uint64_t)(uint8_t)p[b + k] << (8 * k);
  return v;
}
__device__ __forceinline__ void ll_store8(char* p, int64_t line, int64_t nbytes, uint64_t v) {
  const int64_t b = line * 8;
  if (b + 8 <= nbytes && (((uintptr_t)p + b) & 7) == 0) {
    *(uint64_t*)(p + b) = v;
    return;
  }
  for (int k = 0; k < 8 && b + k < nbytes; k++) p[b + k] = (char)(v >> (8 * k));
}

template <class Fn>
__device__ __forceinline__ uint64_t ll_apply(const Fn& fn, uint64_t acc, uint64_t x, int mode) {
  using T = typename Fn::EltType;
  union U { uint64_t u; T e[8 / sizeof(T)]; } a, b;
  a.u = acc;
  b.u = x;
#pragma unroll
  for (int i = 0; i < (int)(8 / sizeof(T)); i++) {
    if (mode == 0) a.e[i] = fn.reduce(a.e[i], b.e[i]);
    else if (mode == 1) a.e[i] = fn.preOp(b.e[i]);
    else a.e[i] = fn.postOp(a.e[i]);
  }
  return a.u;
}

// Poll one LL line until both halves carry `epoch`; returns the 8 data bytes.
__device__ __forceinline__ bool ll_read_line(const char* line, uint32_t epoch, const DevComm* comm,
                                             uint64_t* out) {
  const SysAddr s = sys_addr_window(line);  // lanes may poll different ranks' slots
  uint64_t spins = 0, start = 0;
  for (;;) {
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(s.r, s.voff, 0, kSysAux);
    if (v.y == epoch && v.w == epoch) {
      *out = (uint64_t)v.x | ((uint64_t)v.z << 32);
      return true;
    }
    if ((++spins & 63) == 0) {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (start == 0) start = now;
      if (*comm->abortFlag) return false;
      if (__hip_atomic_load(comm->errorFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return false;
      if (now - start > comm->spinTimeoutTicks) {
        __hip_atomic_store(comm->errorFlag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
      }
    }
  }
}

// Successor of epoch e: e + 1, except that the wrap skips 0 (the cleared
// state of every line and flag) AND 1, going 0xffffffff -> 2, so consecutive
// epochs always alternate parity — the LL path's double buffering depends on
// it (a peer one call ahead writes the other parity's slot).
__host__ __device__ __forceinline__ uint32_t epoch_after(uint32_t e) {
  return e + 1 == 0 ? 2u : e + 1;
}
// Epoch of this call: the successor of *epochWord.  The last workgroup to
// finish (ticket in *doneWord) stores it back for the next call, so the
// counter is device-resident and graph replays stay in step.
__device__ __forceinline__ uint32_t epoch_next(const uint32_t* epochWord) {
  return epoch_after(__hip_atomic_load(epochWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void epoch_retire(uint32_t* epochWord, uint32_t* doneWord, uint32_t e) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t done = __hip_atomic_fetch_add(doneWord, 1u, __ATOMIC_ACQ_REL,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    if (done == gridDim.x - 1) {
      __hip_atomic_store(doneWord, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(epochWord, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
__device__ __forceinline__ uint32_t ll_epoch_of(const DevComm* comm) { return epoch_next(&comm->llEpoch); }
__device__ __forceinline__ void ll_epoch_retire(DevComm* comm, uint32_t e) {
  epoch_retire(&comm->llEpoch, &comm->llDone, e);
}

// Part table in LDS (filled through constant indices: a runtime index into
// the by-value kernel argument would copy it to scratch); `advance` moves a
// thread's part cursor forward to the part holding line l (lines visited by a
// thread only grow).
struct LLParts {
  LLPart p[kLLMaxParts];
};
__device__ __forceinline__ void ll_load_parts(const LLWork& w, LLParts* sh) {
#pragma unroll
  for (int i = 0; i < kLLMaxParts; i++)
    if ((int)threadIdx.x == i && i < w.nParts) sh->p[i] = w.parts[i];
  __syncthreads();
}
__device__ __forceinline__ int ll_advance(const LLParts& sh, int nParts, int cur, int64_t l) {
  while (cur + 1 < nParts && l >= sh.p[cur + 1].line0) cur++;
  return cur;
}

template <class Fn>
__device__ void ll_allreduce(const LLWork& w) {
  const Fn fn(load_op_arg(w.redArgPtr, w.redArgBytes, w.redArg));
  __shared__ LLParts sh;
  ll_load_parts(w, &sh);
  const uint32_t epoch = ll_epoch_of(w.comm);
  const int64_t nLines = w.nLines;
  const int nParts = w.nParts;
  const int parity = (int)(epoch & 1);
  const int64_t gtid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t gthreads = (int64_t)gridDim.x * blockDim.x;
  const uint32_t e = epoch;
  // Phase 1: publish my input to every peer (one hop over xGMI).
  int pc = 0;
  for (int64_t l = gtid; l < nLines; l += gthreads) {
    pc = ll_advance(sh, nParts, pc, l);
    const LLPart& part = sh.p[pc];
    const uint64_t v = ll_load8(part.send, l - part.line0, part.nbytes);
    u32x4 line;
    line.x = (uint32_t)v;
    line.y = e;
    line.z = (uint32_t)(v >> 32);
    line.w = e;
    for (int k = 1; k < w.nRanks; k++) {
      const int peer = w.rank + k < w.nRanks ? w.rank + k : w.rank + k - w.nRanks;
      const SysAddr d = sys_addr(w.peerBuf[peer] + ll_slot_off(parity, w.rank, w.nRanks, w.linesPerSlot) + l * 16);
      __builtin_amdgcn_raw_buffer_store_b128(line, d.r, d.voff, 0, kSysAux);
    }
  }
  // Phase 2: fold all inputs along the chain (DevComm::llChain, root first),
  // from the leaf up: acc = x_{c[n-1]}, acc = acc (+) x_{c[k]} for k = n-2..0
  // — with the identity chain x_0 (+) (x_1 (+) (... x_{n-1})).
  // Loads for up to kLLBatch sources of a line are issued together (their
  // latencies overlap); a source whose line has not arrived yet is re-polled.
  constexpr int kLLBatch = 8;
  bool ok = true;
  pc = 0;
  const int8_t* chain = w.comm->llChain;  // n <= kOrderMaxRanks; identity beyond
  const bool useChain = w.nRanks <= kOrderMaxRanks;
  for (int64_t l = gtid; l < nLines && ok; l += gthreads) {
    pc = ll_advance(sh, nParts, pc, l);
    const LLPart& part = sh.p[pc];
    const int64_t pl = l - part.line0;
    uint64_t acc = 0;
    for (int hi = w.nRanks - 1; hi >= 0 && ok; hi -= kLLBatch) {
      const int lo = hi - kLLBatch + 1 > 0 ? hi - kLLBatch + 1 : 0;
      u32x4 v[kLLBatch];
#pragma unroll
      for (int b = 0; b < kLLBatch; b++) {
        const int pos = hi - b;
        const int p = pos < lo ? w.rank : useChain ? __builtin_amdgcn_readfirstlane(chain[pos]) : pos;
        if (pos >= lo && p != w.rank) {
          const SysAddr a = sys_addr(w.localBuf + ll_slot_off(parity, p, w.nRanks, w.linesPerSlot) + l * 16);
          v[b] = __builtin_amdgcn_raw_buffer_load_b128(a.r, a.voff, 0, kSysAux);
        }
      }
#pragma unroll
      for (int b = 0; b < kLLBatch; b++) {
        const int pos = hi - b;
        if (pos < lo) break;
        const int p = useChain ? __builtin_amdgcn_readfirstlane(chain[pos]) : pos;
        uint64_t x;
        if (p == w.rank) {
          x = ll_load8(part.send, pl, part.nbytes);
        } else if (v[b].y == e && v[b].w == e) {
          x = (uint64_t)v[b].x | ((uint64_t)v[b].z << 32);
        } else {
          ok = ll_read_line(w.localBuf + ll_slot_off(parity, p, w.nRanks, w.linesPerSlot) + l * 16, e,
                            w.comm, &x);
          if (!ok) break;
        }
        if (Fn::kPreOp && w.preOp) x = ll_apply(fn, 0, x, 1);
        acc = (pos == w.nRanks - 1) ? x : ll_apply(fn, acc, x, 0);  // LL order: child (+) own
      }
    }
    if (!ok) break;
    if (Fn::kPostOp) acc = ll_apply(fn, acc, 0, 2);
    ll_store8(part.recv, pl, part.nbytes, acc);
  }
  ll_epoch_retire(w.comm, e);
}

// ------------------------------------------------------------ reduce-scatter
// One-hop LL reduce-scatter: line l of my contribution to rank p's block goes
// to p's slot (parity, me); p folds its block line by line from the n-1 slots
// and its own input, in the order of the line's ring (lines never straddle a
// channel part: parts are 16-byte multiples of the block, lines 8 bytes).
// Up to kLLMaxParts calls per launch (a group's run): part i's block lines
// sit at [line0_i, line0_i + ceil(nbytes_i / 8)) of every slot.
template <class Fn>
__device__ void ll_reducescatter(const LLWork& w) {
  using T = typename Fn::EltType;
  const Fn fn(load_op_arg(w.redArgPtr, w.redArgBytes, w.redArg));
  __shared__ LLParts sh;
  ll_load_parts(w, &sh);
  const uint32_t e = ll_epoch_of(w.comm);
  const int parity = (int)(e & 1);
  const int n = w.nRanks, me = w.rank, nParts = w.nParts;
  const int64_t nLines = w.nLines;
  const int64_t gtid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t gthreads = (int64_t)gridDim.x * blockDim.x;
  int pc = 0;
  for (int64_t l = gtid; l < nLines; l += gthreads) {
    pc = ll_advance(sh, nParts, pc, l);
    const LLPart& part = sh.p[pc];
    const int64_t nb = part.nbytes, pl = l - part.line0;
    for (int k = 1; k < n; k++) {
      const int p = me + k < n ? me + k : me + k - n;
      const uint64_t v = ll_load8(part.send + (int64_t)p * nb, pl, nb);
      u32x4 line;
      line.x = (uint32_t)v;
      line.y = e;
      line.z = (uint32_t)(v >> 32);
      line.w = e;
      const SysAddr d = sys_addr(w.peerBuf[p] + ll_slot_off(parity, me, n, w.linesPerSlot) + l * 16);
      __builtin_amdgcn_raw_buffer_store_b128(line, d.r, d.voff, 0, kSysAux);
    }
  }
  bool ok = true;
  pc = 0;
  for (int64_t l = gtid; l < nLines && ok; l += gthreads) {
    pc = ll_advance(sh, nParts, pc, l);
    const LLPart& part = sh.p[pc];
    const int64_t nb = part.nbytes, pl = l - part.line0;
    int64_t end;
    const int ch = cbd_channel_of(part.cbd, pl * 8 / (int64_t)sizeof(T), &end);
    const int8_t* order = w.comm->rsOrder[ch % w.comm->nRings];
    u32x4 v[kOrderMaxRanks];
#pragma unroll
    for (int j = 0; j < kOrderMaxRanks; j++) {  // every peer line of l in flight at once
      const int q = j < n ? order[j] : me;
      if (q != me) {
        // q differs between lanes whose lines sit in different channel parts
        const SysAddr a = sys_addr_window(w.localBuf + ll_slot_off(parity, q, n, w.linesPerSlot) + l * 16);
        v[j] = __builtin_amdgcn_raw_buffer_load_b128(a.r, a.voff, 0, kSysAux);
      }
    }
    uint64_t acc = 0;
#pragma unroll
    for (int j = 0; j < kOrderMaxRanks; j++) {
      if (j >= n) break;
      const int q = order[j];
      uint64_t x;
      if (q == me) {
        x = ll_load8(part.send + (int64_t)me * nb, pl, nb);
      } else if (v[j].y == e && v[j].w == e) {
        x = (uint64_t)v[j].x | ((uint64_t)v[j].z << 32);
      } else {
        ok = ll_read_line(w.localBuf + ll_slot_off(parity, q, n, w.linesPerSlot) + l * 16, e, w.comm,
                          &x);
        if (!ok) break;
      }
      if (Fn::kPreOp && w.preOp) x = ll_apply(fn, 0, x, 1);
      acc = j == 0 ? x : ll_apply(fn, acc, x, 0);
    }
    if (!ok) break;
    if (Fn::kPostOp) acc = ll_apply(fn, acc, 0, 2);
    ll_store8(part.recv, pl, nb, acc);
  }
  ll_epoch_retire(w.comm, e);
}

// ---------------------------------------------------------------- all-gather
// One-hop LL all-gather (bytes): my block's lines go to every peer's slot
// (parity, me); every rank copies each rank's block out of its slots (its own
// from its input) to output + rank * bytes.  Up to kLLMaxParts calls per
// launch, as the reduce-scatter.
__device__ inline void ll_allgather(const LLWork& w) {
  __shared__ LLParts sh;
  ll_load_parts(w, &sh);
  const uint32_t e = ll_epoch_of(w.comm);
  const int parity = (int)(e & 1);
  const int n = w.nRanks, me = w.rank, nParts = w.nParts;
  const int64_t nLines = w.nLines;
  const int64_t gtid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t gthreads = (int64_t)gridDim.x * blockDim.x;
  int pc = 0;
  for (int64_t l = gtid; l < nLines; l += gthreads) {
    pc = ll_advance(sh, nParts, pc, l);
    const LLPart& part = sh.p[pc];
    const int64_t nb = part.nbytes, pl = l - part.line0;
    const char* in = part.send;
    char* out = part.recv;
    const uint64_t v = ll_load8(in, pl, nb);
    u32x4 line;
    line.x = (uint32_t)v;
    line.y = e;
    line.z = (uint32_t)(v >> 32);
    line.w = e;
    for (int k = 1; k < n; k++) {
      const int p = me + k < n ? me + k : me + k - n;
      const SysAddr d = sys_addr(w.peerBuf[p] + ll_slot_off(parity, me, n, w.linesPerSlot) + l * 16);
      __builtin_amdgcn_raw_buffer_store_b128(line, d.r, d.voff, 0, kSysAux);
    }
    if (out + (int64_t)me * nb != in) ll_store8(out + (int64_t)me * nb, pl, nb, v);
  }
  bool ok = true;
  pc = 0;
  for (int64_t l = gtid; l < nLines && ok; l += gthreads) {
    pc = ll_advance(sh, nParts, pc, l);
    const LLPart& part = sh.p[pc];
    const int64_t nb = part.nbytes, pl = l - part.line0;
    for (int k = 1; k < n; k++) {
      const int q = me + k < n ? me + k : me + k - n;
      uint64_t x;
      ok = ll_read_line(w.localBuf + ll_slot_off(parity, q, n, w.linesPerSlot) + l * 16, e, w.comm, &x);
      if (!ok) break;
      ll_store8(part.recv + (int64_t)q * nb, pl, nb, x);
    }
  }
  ll_epoch_retire(w.comm, e);
}

}  // namespace vccl
