// The gfx950 code sequences of HIP's system-scope fences, for DESIGN.md §4.2
// (the fence-free slot hand-off argument).  Compile only, never run:
//   tools/fence_isa.sh > profiles/r06a/fence_isa.txt
#include <hip/hip_runtime.h>

// release: payload stores, then the flag (what VCCL_FENCES=1 does per slot)
extern "C" __global__ void release_system(int* data, int* flag, int v) {
  data[threadIdx.x] = v;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// acquire: the flag, then payload loads
extern "C" __global__ void acquire_system(int* flag, int* data, int* out) {
  const int f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  out[threadIdx.x] = f + data[threadIdx.x];
}
// the default hand-off's shape: system-scope (sc0 sc1) payload stores, a
// full store drain, then the relaxed system-scope flag store — no fence
extern "C" __global__ void handoff_fence_free(int* data, int* flag, int v) {
  __hip_atomic_store(data + threadIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
