// Host cost per call of the pieces under an eager collective call, and of
// the call itself through the C API (measurement tool, not product code).
//
//   launch_cost [iters]
//
// Each row: host wall time of `iters` back-to-back calls / iters (the host
// side only: the GPU work is queued, then drained before the next row), and
// for the launches the GPU time per call from events around the loop.
// Rows: hipGetDevice, hipStreamGetCaptureInfo, hipEventRecord, an empty
// kernel via hipLaunchKernelGGL and via hipExtLaunchKernelGGL with a stop
// event (the library's ordering event), then ncclAllReduce on a world-1 comm
// (1 KiB out of place) and, on two comms of ONE process sharing device 0
// (ncclCommInitAll, VCCL_ALLOW_SHARED_DEVICE), a grouped 8 B f16 all-reduce
// (the LL path) per call and per group.  Prints one JSON object.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "nccl.h"

#define CK(cmd)                                                                  \
  do {                                                                           \
    auto r_ = (cmd);                                                             \
    if ((int)r_ != 0) {                                                          \
      fprintf(stderr, "%s failed (%d) at line %d\n", #cmd, (int)r_, __LINE__); \
      exit(2);                                                                   \
    }                                                                            \
  } while (0)

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1;
}

struct Row {
  double hostUs, gpuUs;
};

static Row time_loop(int iters, hipStream_t s, const std::function<void()>& fn) {
  for (int i = 0; i < 200; i++) fn();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; i++) fn();
  const double host = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  CK(hipEventRecord(e1, s));
  CK(hipDeviceSynchronize());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return {host / iters, ms * 1e3 / iters};
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 5000;
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  int* flag;
  CK(hipMalloc(&flag, 64));
  std::vector<std::pair<std::string, Row>> rows;
  int dev = 0;
  rows.push_back({"hipGetDevice", time_loop(iters, s, [&] { CK(hipGetDevice(&dev)); })});
  rows.push_back({"hipStreamGetCaptureInfo", time_loop(iters, s, [&] {
                    hipStreamCaptureStatus st;
                    unsigned long long id;
                    CK(hipStreamGetCaptureInfo(s, &st, &id));
                  })});
  rows.push_back({"hipEventRecord", time_loop(iters, s, [&] { CK(hipEventRecord(ev, s)); })});
  rows.push_back({"launch_empty", time_loop(iters, s, [&] {
                    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, flag);
                  })});
  rows.push_back({"ext_launch_empty_stop_event", time_loop(iters, s, [&] {
                    hipExtLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr, ev, 0, flag);
                  })});
  rows.push_back({"launch_empty_256wg", time_loop(iters, s, [&] {
                    hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, flag);
                  })});

  // world-1 comm: config 1's call
  {
    ncclComm_t c1;
    int d0 = 0;
    CK(ncclCommInitAll(&c1, 1, &d0));
    float *x, *y;
    CK(hipMalloc(&x, 1024));
    CK(hipMalloc(&y, 1024));
    rows.push_back({"ncclAllReduce_world1_1KiB_oop", time_loop(iters, s, [&] {
                      CK(ncclAllReduce(x, y, 256, ncclFloat32, ncclSum, c1, s));
                    })});
    rows.push_back({"ncclAllReduce_world1_1KiB_inplace", time_loop(iters, s, [&] {
                      CK(ncclAllReduce(x, x, 256, ncclFloat32, ncclSum, c1, s));
                    })});
    CK(ncclCommDestroy(c1));
    CK(hipFree(x));
    CK(hipFree(y));
  }
  // two ranks in one process on device 0: the LL all-reduce's host path
  {
    setenv("VCCL_ALLOW_SHARED_DEVICE", "1", 1);
    ncclComm_t cs[2];
    int devs[2] = {0, 0};
    CK(ncclCommInitAll(cs, 2, devs));
    hipStream_t s2[2];
    void* b[2];
    for (int r = 0; r < 2; r++) {
      CK(hipStreamCreateWithFlags(&s2[r], hipStreamNonBlocking));
      CK(hipMalloc(&b[r], 4096));
      CK(hipMemset(b[r], 0, 4096));
    }
    CK(hipDeviceSynchronize());
    const int gi = iters / 4;
    for (size_t bytes : {(size_t)8, (size_t)4096}) {
      Row r = time_loop(gi, s2[0], [&] {
        CK(ncclGroupStart());
        for (int k = 0; k < 2; k++)
          CK(ncclAllReduce(b[k], b[k], bytes / 2, ncclFloat16, ncclSum, cs[k], s2[k]));
        CK(ncclGroupEnd());
      });
      rows.push_back({"group2_allreduce_f16_" + std::to_string(bytes) + "B_per_group", r});
      rows.push_back({"group2_allreduce_f16_" + std::to_string(bytes) + "B_per_call",
                      Row{r.hostUs / 2, r.gpuUs}});
    }
    for (int r = 0; r < 2; r++) {
      CK(ncclCommDestroy(cs[r]));
      CK(hipStreamDestroy(s2[r]));
      CK(hipFree(b[r]));
    }
  }
  printf("{\"iters\": %d", iters);
  for (auto& [k, r] : rows) printf(", \"%s\": {\"host_us\": %.3f, \"gpu_us\": %.3f}", k.c_str(), r.hostUs, r.gpuUs);
  printf("}\n");
  CK(hipFree(flag));
  return 0;
}
