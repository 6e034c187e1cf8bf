// Ring-step copy probe (measurement tool, not product code; built into
// vccl_amd/lib/libvccl_stepprobe.so, driven by tools/step_probe.py).
//
// Each workgroup plays one ring channel and repeats ONE primitive shape over
// its own 512 KiB slot `reps` times, with the ring primitive's per-slot
// drain (s_waitcnt vmcnt(0)) and barrier but no flags and no peer: the
// per-channel copy rate of the reduce-copy engine (reduce_copy.hpp) in each
// shape of ring.hpp's schedules, without the protocol's waits.  Operands: S =
// own input (normal memory, nt loads), F / F2 = FIFO slots (uncached memory,
// sc0 sc1), O = own output (normal memory, policy per variant).  S and O
// stream through large buffers (slot r*nWG + b of `span` bytes), as the own
// input / output stream through a bucket; F / F2 stay put, as FIFO slots.
#include <hip/hip_runtime.h>

#include "../vccl_amd/csrc/device/reduce_copy.hpp"

using namespace vccl;

namespace {

// shape: 0 S->F  1 S+F->F2  2 S+F->O  3 S->F+O  4 F->O  5 F->F2+O  6 S+F->F2+O
template <int SHAPE, int U, int OPOL, int SPOL>
__global__ __launch_bounds__(512) void k_step(const char* S, const char* F, char* F2, char* O,
                                               int64_t slotBytes, int reps, int64_t span) {
  const int64_t base = (int64_t)blockIdx.x * slotBytes;
  constexpr int NS = (SHAPE == 1 || SHAPE == 2 || SHAPE == 6) ? 2 : 1;
  constexpr int ND = (SHAPE == 3 || SHAPE == 5 || SHAPE == 6) ? 2 : 1;
  constexpr bool srcIsS = SHAPE != 4 && SHAPE != 5;
  constexpr int S0 = srcIsS ? SPOL : kSys;
  // destinations in ring.hpp's order: FIFO slot first (sc0 sc1), then the output
  constexpr bool dstF = SHAPE != 2 && SHAPE != 4;
  constexpr int D0 = dstF ? kSys : OPOL;
  constexpr int POLS = mkpol(S0, kSys, kSys, kSys, D0, kNT, kNT, kNT);
  RCArgs a;
  a.srcs[0] = (srcIsS ? S : F) + base;
  a.srcs[1] = F + base;
  a.srcs[2] = a.srcs[3] = a.srcs[0];
  a.dsts[0] = (dstF ? F2 : O) + base;
  a.dsts[1] = O + base;
  a.dsts[2] = a.dsts[3] = a.dsts[0];
  a.nSrcs = NS;
  a.nDsts = ND;
  a.preOpSrcs = 0;
  a.postOp = 0;
  a.argPtr = nullptr;
  a.argBytes = 0;
  const FnSum<float> fn(0);
  const int64_t nSlots = span / slotBytes;
  for (int r = 0; r < reps; r++) {
    const int64_t so = (((int64_t)r * gridDim.x + blockIdx.x) % nSlots) * slotBytes;
    a.srcs[0] = (srcIsS ? S + so : F + base);
    a.dsts[1] = O + so;
    if (!dstF) a.dsts[0] = O + so;
    reduce_copy<FnSum<float>, NS, ND, U, POLS, 0, true>(fn, a, slotBytes / 4, 0, 1, threadIdx.x, blockDim.x);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

template <int SHAPE, int U, int SPOL>
hipError_t launch_p(int opol, const void* S, const void* F, void* F2, void* O, int64_t slot, int nWG,
                    int threads, int reps, int64_t span, hipStream_t st) {
  if (opol == kNT)
    hipLaunchKernelGGL((k_step<SHAPE, U, kNT, SPOL>), dim3(nWG), dim3(threads), 0, st, (const char*)S,
                       (const char*)F, (char*)F2, (char*)O, slot, reps, span);
  else
    hipLaunchKernelGGL((k_step<SHAPE, U, kSys, SPOL>), dim3(nWG), dim3(threads), 0, st, (const char*)S,
                       (const char*)F, (char*)F2, (char*)O, slot, reps, span);
  return hipGetLastError();
}
template <int SHAPE, int U>
hipError_t launch_u(int opol, int spol, const void* S, const void* F, void* F2, void* O, int64_t slot,
                    int nWG, int threads, int reps, int64_t span, hipStream_t st) {
  if (spol == kPlain) return launch_p<SHAPE, U, kPlain>(opol, S, F, F2, O, slot, nWG, threads, reps, span, st);
  return launch_p<SHAPE, U, kNT>(opol, S, F, F2, O, slot, nWG, threads, reps, span, st);
}

template <int SHAPE>
hipError_t launch_s(int unroll, int opol, int spol, const void* S, const void* F, void* F2, void* O,
                    int64_t slot, int nWG, int threads, int reps, int64_t span, hipStream_t st) {
  switch (unroll) {
    case 4: return launch_u<SHAPE, 4>(opol, spol, S, F, F2, O, slot, nWG, threads, reps, span, st);
    case 8: return launch_u<SHAPE, 8>(opol, spol, S, F, F2, O, slot, nWG, threads, reps, span, st);
  }
  return hipErrorInvalidValue;
}

}  // namespace

extern "C" int step_probe_alloc_uncached(void** p, size_t bytes) {
  return (int)hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached);
}
extern "C" int step_probe_free(void* p) { return (int)hipFree(p); }

// F / F2 hold nWG * slot bytes, S / O `span` bytes (a multiple of slot, at
// least nWG * slot); slot a multiple of 16 KiB.
extern "C" int step_probe_run(int shape, int unroll, int opol, int spol, const void* S, const void* F,
                              void* F2, void* O, long slot, int nWG, int threads, int reps, long span,
                              hipStream_t st) {
  if (slot <= 0 || slot % (16 << 10) || nWG <= 0 || threads % 64 || threads > 512 || reps <= 0 ||
      span % slot || span < (long)nWG * slot)
    return (int)hipErrorInvalidValue;
  switch (shape) {
    case 0: return (int)launch_s<0>(unroll, opol, spol, S, F, F2, O, slot, nWG, threads, reps, span, st);
    case 1: return (int)launch_s<1>(unroll, opol, spol, S, F, F2, O, slot, nWG, threads, reps, span, st);
    case 2: return (int)launch_s<2>(unroll, opol, spol, S, F, F2, O, slot, nWG, threads, reps, span, st);
    case 3: return (int)launch_s<3>(unroll, opol, spol, S, F, F2, O, slot, nWG, threads, reps, span, st);
    case 4: return (int)launch_s<4>(unroll, opol, spol, S, F, F2, O, slot, nWG, threads, reps, span, st);
    case 5: return (int)launch_s<5>(unroll, opol, spol, S, F, F2, O, slot, nWG, threads, reps, span, st);
    case 6: return (int)launch_s<6>(unroll, opol, spol, S, F, F2, O, slot, nWG, threads, reps, span, st);
  }
  return (int)hipErrorInvalidValue;
}
