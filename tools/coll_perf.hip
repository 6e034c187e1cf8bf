// nccl-tests-style driver (all_reduce_perf / reduce_scatter_perf /
// all_gather_perf / broadcast_perf / reduce_perf) written against the C API only: include/nccl.h +
// libvccl.so, exactly as a C/C++ caller of the reference links libnccl.
// SURVEY.md §8b names nccl-tests as the path's caller; this is the same
// shape of program (size sweep, algbw / busbw columns, #wrong), not a copy.
//
//   coll_perf -C allreduce|reducescatter|allgather|broadcast|reduce -r <ranks>
//             -b <min bytes> -e <max bytes> -f <factor> -n <iters> -w <warmup>
//             -d float|half|bfloat16|int32|double -o sum|max|min -R <root>
//
// One process per rank: the parent creates the unique id (sockets only, no
// GPU call), forks the ranks and waits; each rank uses GPU (rank % ndev).
// Inputs are small integers (exact in every type and fold order), so every
// element of every output is checked against its closed form.
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "nccl.h"

#define CK(cmd)                                                                          \
  do {                                                                                   \
    auto r_ = (cmd);                                                                     \
    if ((int)r_ != 0) {                                                                  \
      fprintf(stderr, "rank %d: %s failed (%d) at line %d\n", g_rank, #cmd, (int)r_, __LINE__); \
      exit(2);                                                                           \
    }                                                                                    \
  } while (0)

static int g_rank = -1;

// Input element i of rank r: ((i * 7 + r * 3) % 9) - 4, a small integer.
__device__ __host__ inline int val(size_t i, int r) { return (int)((i * 7 + (size_t)r * 3) % 9) - 4; }

template <class T>
__device__ __host__ inline T from_int(int v) { return (T)v; }
template <>
__device__ __host__ inline __half from_int<__half>(int v) { return __float2half((float)v); }
template <>
__device__ __host__ inline __hip_bfloat16 from_int<__hip_bfloat16>(int v) {
  return __float2bfloat16((float)v);
}
template <class T>
__host__ inline double to_double(T v) { return (double)v; }
template <>
__host__ inline double to_double<__half>(__half v) { return (double)__half2float(v); }
template <>
__host__ inline double to_double<__hip_bfloat16>(__hip_bfloat16 v) {
  return (double)__bfloat162float(v);
}

template <class T>
__global__ void fill(T* p, size_t n, size_t base, int r) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = from_int<T>(val(base + i, r));
}

struct Args {
  std::string coll = "allreduce", dtype = "float", op = "sum";
  int ranks = 2, iters = 20, warmup = 5, root = 0;
  size_t minBytes = 8, maxBytes = 64 << 20;
  double factor = 2;
};

static ncclRedOp_t op_of(const std::string& s) {
  return s == "max" ? ncclMax : s == "min" ? ncclMin : ncclSum;
}

// Expected output element j (AR / reduce: element j; RS: element rank*count + j
// of the sum; AG: element j of the concatenation; broadcast: the root's).
static double expect(const Args& a, int nranks, int rank, size_t count, size_t j) {
  if (a.coll == "allgather") return val(j % count, (int)(j / count));
  if (a.coll == "broadcast") return val(j, a.root);
  const size_t i = a.coll == "reducescatter" ? rank * count + j : j;
  double acc = a.op == "sum" ? 0 : val(i, 0);
  for (int r = 0; r < nranks; r++) {
    const double v = val(i, r);
    acc = a.op == "sum" ? acc + v : a.op == "max" ? std::max(acc, v) : std::min(acc, v);
  }
  return acc;
}

template <class T>
static int run_rank(const Args& a, int rank, ncclUniqueId id, ncclDataType_t dt) {
  g_rank = rank;
  int ndev = 0;
  CK(hipGetDeviceCount(&ndev));
  CK(hipSetDevice(rank % ndev));
  ncclComm_t comm;
  CK(ncclCommInitRank(&comm, a.ranks, id, rank));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int n = a.ranks;
  // nccl-tests' bus factors: AR 2(n-1)/n, RS / AG (n-1)/n, broadcast / reduce 1
  const double busFactor = a.coll == "allreduce"                           ? 2.0 * (n - 1) / n
                           : a.coll == "broadcast" || a.coll == "reduce" ? 1.0
                                                                         : (double)(n - 1) / n;
  if (rank == 0) {
    printf("# coll_perf %s  ranks %d  dtype %s  op %s  iters %d  warmup %d (libvccl via include/nccl.h)\n",
           a.coll.c_str(), n, a.dtype.c_str(), a.op.c_str(), a.iters, a.warmup);
    printf("#%12s %12s %8s %6s %10s %9s %9s %7s %8s\n", "size", "count", "type", "redop", "time(us)",
           "algbw", "busbw", "#wrong", "host(us)");
  }
  double* tdev;
  CK(hipMalloc(&tdev, sizeof(double)));
  long long wrongTotal = 0;
  for (size_t bytes = a.minBytes; bytes <= a.maxBytes;
       bytes = std::max(bytes + 1, (size_t)(bytes * a.factor))) {
    // size = the larger buffer per rank (nccl-tests convention)
    size_t count = std::max<size_t>(1, bytes / sizeof(T));
    size_t inElts = count, outElts = count, collCount = count;
    if (a.coll == "reducescatter") {
      collCount = std::max<size_t>(1, count / n);
      inElts = collCount * n;
      outElts = collCount;
    } else if (a.coll == "allgather") {
      collCount = std::max<size_t>(1, count / n);
      inElts = collCount;
      outElts = collCount * n;
    }
    T *in, *out;
    CK(hipMalloc(&in, inElts * sizeof(T)));
    CK(hipMalloc(&out, outElts * sizeof(T)));
    if (a.coll != "allgather") {
      hipLaunchKernelGGL(fill<T>, dim3(256), dim3(256), 0, s, in, inElts, (size_t)0, rank);
    } else {
      // AG input = this rank's block of the concatenation: val(j % count, owner)
      std::vector<T> h(inElts);
      for (size_t j = 0; j < inElts; j++) h[j] = from_int<T>(val(j, rank));
      CK(hipMemcpy(in, h.data(), inElts * sizeof(T), hipMemcpyHostToDevice));
    }
    auto call = [&]() {
      if (a.coll == "allreduce")
        CK(ncclAllReduce(in, out, collCount, dt, op_of(a.op), comm, s));
      else if (a.coll == "reducescatter")
        CK(ncclReduceScatter(in, out, collCount, dt, op_of(a.op), comm, s));
      else if (a.coll == "broadcast")
        CK(ncclBroadcast(in, out, collCount, dt, a.root, comm, s));
      else if (a.coll == "reduce")
        CK(ncclReduce(in, out, collCount, dt, op_of(a.op), a.root, comm, s));
      else
        CK(ncclAllGather(in, out, collCount, dt, comm, s));
    };
    for (int w = 0; w < a.warmup; w++) call();
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    // host(us): wall time of the enqueue loop alone per call (the host side
    // of a call; equals time(us) when the host is the bottleneck)
    const auto h0 = std::chrono::steady_clock::now();
    for (int it = 0; it < a.iters; it++) call();
    const double hostUs =
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count() / a.iters;
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    double us = ms * 1e3 / a.iters;
    // slowest rank's time, through the library itself (f64 max all-reduce)
    CK(hipMemcpy(tdev, &us, sizeof(double), hipMemcpyHostToDevice));
    CK(ncclAllReduce(tdev, tdev, 1, ncclFloat64, ncclMax, comm, s));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(&us, tdev, sizeof(double), hipMemcpyDeviceToHost));
    std::vector<T> h(outElts);
    CK(hipMemcpy(h.data(), out, outElts * sizeof(T), hipMemcpyDeviceToHost));
    long long wrong = 0;
    const bool checked = a.coll != "reduce" || rank == a.root;  // a non-root's reduce output is untouched
    for (size_t j = 0; checked && j < outElts; j++)
      wrong += to_double(h[j]) != expect(a, n, rank, collCount, j);
    ncclResult_t ae;
    CK(ncclCommGetAsyncError(comm, &ae));
    if (ae != ncclSuccess) wrong += 1000000;
    wrongTotal += wrong;
    const double sz = (double)std::max(inElts, outElts) * sizeof(T);
    const double algbw = sz / (us * 1e-6) / 1e9;
    if (rank == 0)
      printf(" %12zu %12zu %8s %6s %10.2f %9.2f %9.2f %7lld %8.2f\n", (size_t)sz, collCount,
             a.dtype.c_str(), a.coll == "allgather" || a.coll == "broadcast" ? "none" : a.op.c_str(), us, algbw,
             algbw * busFactor, wrong, hostUs);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    CK(hipFree(in));
    CK(hipFree(out));
  }
  CK(hipFree(tdev));
  CK(ncclCommDestroy(comm));
  if (rank == 0) printf("# Out of bounds values : %lld %s\n", wrongTotal, wrongTotal ? "FAILED" : "OK");
  return wrongTotal ? 1 : 0;
}

int main(int argc, char** argv) {
  Args a;
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string k = argv[i], v = argv[i + 1];
    if (k == "-C") a.coll = v;
    else if (k == "-r") a.ranks = atoi(v.c_str());
    else if (k == "-b") a.minBytes = strtoull(v.c_str(), nullptr, 0);
    else if (k == "-e") a.maxBytes = strtoull(v.c_str(), nullptr, 0);
    else if (k == "-f") a.factor = atof(v.c_str());
    else if (k == "-n") a.iters = atoi(v.c_str());
    else if (k == "-w") a.warmup = atoi(v.c_str());
    else if (k == "-d") a.dtype = v;
    else if (k == "-o") a.op = v;
    else if (k == "-R") a.root = atoi(v.c_str());
    else {
      fprintf(stderr, "unknown option %s\n", k.c_str());
      return 2;
    }
  }
  // The unique id holds the bootstrap root (a socket thread of THIS
  // process); no HIP call happens before the fork.
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return 2;
  fflush(stdout);
  std::vector<pid_t> kids;
  for (int r = 0; r < a.ranks; r++) {
    pid_t p = fork();
    if (p == 0) {
      int rc = 2;
      if (a.dtype == "float") rc = run_rank<float>(a, r, id, ncclFloat32);
      else if (a.dtype == "half") rc = run_rank<__half>(a, r, id, ncclFloat16);
      else if (a.dtype == "bfloat16") rc = run_rank<__hip_bfloat16>(a, r, id, ncclBfloat16);
      else if (a.dtype == "int32") rc = run_rank<int>(a, r, id, ncclInt32);
      else if (a.dtype == "double") rc = run_rank<double>(a, r, id, ncclFloat64);
      fflush(stdout);
      _exit(rc);
    }
    kids.push_back(p);
  }
  int worst = 0;
  for (pid_t p : kids) {
    int st = 0;
    waitpid(p, &st, 0);
    const int rc = WIFEXITED(st) ? WEXITSTATUS(st) : 3;
    worst = std::max(worst, rc);
  }
  return worst;
}
