// Line-tearing probe for an LL128-style wire format (test-only; built into
// vccl_amd/lib/libvccl_probe.so, loaded by tests/test_gpu_ll128.py).
//
// VCCL's LL128 protocol (src/device/prims_ll128.h:176-324) stores a 128-byte
// line — 15 data words + 1 flag word — with 8 threads x 16 B and lets the
// reader trust the 15 data words as soon as the flag word carries the
// expected step.  That needs the line's 16-byte pieces to become visible
// together (NVLink delivers a warp's 128 B store that way).  This probe asks
// the same of gfx950: writer workgroup 2p stores lines {data(it), flag(it)}
// with sc0 sc1 buffer stores (8 lanes x 16 B per 128-byte line, or 4 lanes per
// 64-byte line), reader workgroup 2p+1 — on another XCD under round-robin
// dispatch — polls each line with sc0 sc1 loads (the same instruction loads
// the flag lane and the data lanes) and counts lines whose flag shows
// iteration `it` while a data word still shows an older one ("flag before
// data": a tear LL128 cannot tolerate).  The reader acknowledges each
// iteration before the writer starts the next, as LL128's credits would.
// Intra-GPU only: a clean result is necessary for xGMI, not sufficient.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int kAux = 1 | 16;  // sc0 | sc1

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base) {
  const uint64_t x = (uint64_t)(uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), 0,
                                           0x7fffffff, 0x00020000);
}

struct Ctl {
  uint64_t ack;      // last iteration the reader finished (per pair, own 128 B)
  uint64_t pad[15];
};

__device__ __forceinline__ bool spin_until(const uint64_t* p, uint64_t want, uint64_t deadline,
                                           int* fail) {
  while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() > deadline ||
        __hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
      __hip_atomic_store(fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
  }
  return true;
}

// counts: [0] lines checked, [1] flag before data, [2] data ahead of flag,
// [3] timeouts.  lineBytes 128 (LL128) or 64.
__global__ __launch_bounds__(256) void k_line_probe(char* lines, Ctl* ctl, int linesPerPair,
                                                    int iters, int lineBytes,
                                                    unsigned long long* counts, int* fail,
                                                    uint64_t timeoutTicks) {
  const int pair = blockIdx.x >> 1;
  const bool writer = (blockIdx.x & 1) == 0;
  const int tid = threadIdx.x;
  const int parts = lineBytes / 16;        // 16-byte pieces per line
  const int linesPerRound = 256 / parts;   // lines one workgroup instruction round covers
  char* base = lines + (int64_t)pair * linesPerPair * lineBytes;
  const __amdgpu_buffer_rsrc_t r = rsrc_of(base);
  uint64_t* ack = &ctl[pair].ack;
  __shared__ int shFail;
  if (tid == 0) shFail = 0;
  __syncthreads();
  const uint64_t deadline = __builtin_amdgcn_s_memrealtime() + timeoutTicks;
  unsigned long long checked = 0, flagFirst = 0, dataAhead = 0;
  const int part = tid % parts, lineInRound = tid / parts;
  const bool flagLane = part == parts - 1;
  for (uint64_t it = 1; it <= (uint64_t)iters; it++) {
    if (writer) {
      if (tid == 0 && !spin_until(ack, it - 1, deadline, fail)) shFail = 1;
      __syncthreads();
      if (shFail) break;
      for (int l0 = 0; l0 < linesPerPair; l0 += linesPerRound) {
        const int l = l0 + lineInRound;
        if (l >= linesPerPair) continue;
        const uint64_t w0 = (it << 32) | (uint64_t)(l * 16 + 2 * part);
        const uint64_t w1 = flagLane ? it : ((it << 32) | (uint64_t)(l * 16 + 2 * part + 1));
        u32x4 v = {(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
        __builtin_amdgcn_raw_buffer_store_b128(v, r, l * lineBytes + part * 16, 0, kAux);
      }
    } else {
      for (int l0 = 0; l0 < linesPerPair; l0 += linesPerRound) {
        const int l = l0 + lineInRound;
        const bool mine = l < linesPerPair;
        const int off = (mine ? l : 0) * lineBytes + part * 16;
        u32x4 v = {0, 0, 0, 0};
        bool ready = false;
        for (;;) {
          if (!ready) v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAux);
          // the flag of my line: lane (group base + parts - 1)'s upper word
          const int src = (__lane_id() / parts) * parts + parts - 1;
          const uint32_t flag = (uint32_t)__shfl((int)v.z, src);
          ready = !mine || (uint64_t)flag >= it;
          if (__all(ready)) break;
          if (__builtin_amdgcn_s_memrealtime() > deadline ||
              __hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
            __hip_atomic_store(fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            shFail = 1;
            break;
          }
        }
        if (shFail) break;
        if (mine) {
          const int src = (__lane_id() / parts) * parts + parts - 1;
          const uint64_t flag = (uint32_t)__shfl((int)v.z, src);
          const uint64_t s0 = v.y;                 // sequence of word 2*part
          const uint64_t s1 = flagLane ? flag : v.w;
          if (part == 0) checked++;
          if (s0 < flag || s1 < flag) flagFirst++;
          if (s0 > flag || s1 > flag) dataAhead++;
        }
      }
      __syncthreads();
      if (shFail) break;
      if (tid == 0) __hip_atomic_store(ack, it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if (!writer) {
    atomicAdd(&counts[0], checked);
    atomicAdd(&counts[1], flagFirst);
    atomicAdd(&counts[2], dataAhead);
  }
  if (tid == 0 && shFail) atomicAdd(&counts[3], 1ull);
}

}  // namespace

// Runs the probe; counts[4] as above.  Returns 0 on success (the counts
// report tears), nonzero on a HIP error or invalid arguments.
extern "C" __attribute__((visibility("default"))) int vcclProbeLineTearing(
    int pairs, int linesPerPair, int iters, int lineBytes, double timeoutS,
    unsigned long long* countsOut) {
  if (pairs < 1 || pairs > 128 || linesPerPair < 1 || linesPerPair > 4096 || iters < 1 ||
      (lineBytes != 64 && lineBytes != 128) || !countsOut)
    return 1;
  char* lines = nullptr;
  Ctl* ctl = nullptr;
  unsigned long long* counts = nullptr;
  int* fail = nullptr;
  const size_t bytes = (size_t)pairs * linesPerPair * lineBytes;
  int rc = 0;
  if (hipExtMallocWithFlags((void**)&lines, bytes, hipDeviceMallocUncached) != hipSuccess ||
      hipExtMallocWithFlags((void**)&ctl, sizeof(Ctl) * pairs, hipDeviceMallocUncached) != hipSuccess ||
      hipMalloc((void**)&counts, 4 * sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc((void**)&fail, sizeof(int)) != hipSuccess) {
    rc = 2;
  } else {
    (void)hipMemset(lines, 0, bytes);
    (void)hipMemset(ctl, 0, sizeof(Ctl) * pairs);
    (void)hipMemset(counts, 0, 4 * sizeof(unsigned long long));
    (void)hipMemset(fail, 0, sizeof(int));
    const uint64_t ticks = (uint64_t)(timeoutS * 1e8);  // s_memrealtime: 100 MHz
    hipLaunchKernelGGL(k_line_probe, dim3(2 * pairs), dim3(256), 0, 0, lines, ctl, linesPerPair,
                       iters, lineBytes, counts, fail, ticks);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = 3;
    else if (hipMemcpy(countsOut, counts, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost) !=
             hipSuccess)
      rc = 4;
  }
  if (lines) (void)hipFree(lines);
  if (ctl) (void)hipFree(ctl);
  if (counts) (void)hipFree(counts);
  if (fail) (void)hipFree(fail);
  return rc;
}
