// Host-only exercise of the library's C ABI under AddressSanitizer and
// UndefinedBehaviorSanitizer (`make sanitize`; the reference's ASAN=1 /
// UBSAN=1 build knobs, makefiles/common.mk:98-109).  No GPU call is made:
// the planner exports (vcclGroupPlanEx, vcclRingPartition, vcclRingChunkOf,
// vcclAlgoSelection), the op encoding, error strings and the argument checks
// that reject bad handles before any device work.  Random inputs from a fixed
// seed; prints a summary and exits non-zero on an unexpected result (the
// sanitizers abort on any memory or UB error).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "nccl.h"
#include "vccl_device.h"
#include "vccl_ext.h"

static int g_fail = 0;
#define EXPECT(c)                                                  \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "FAILED %s at line %d\n", #c, __LINE__);     \
      g_fail++;                                                    \
    }                                                              \
  } while (0)

int main() {
  std::mt19937_64 rng(20261018);
  auto pick = [&](std::initializer_list<int64_t> v) { return *(v.begin() + rng() % v.size()); };
  const int dts[] = {ncclInt8, ncclUint8, ncclInt32, ncclUint32, ncclInt64, ncclUint64,
                     ncclFloat16, ncclFloat32, ncclFloat64, ncclBfloat16};
  long groups = 0, calls = 0;
  for (int trial = 0; trial < 3000; trial++) {
    const int n = (int)pick({1, 2, 3, 4, 6, 7, 8});
    const int nch = (int)pick({1, 2, 14, 16, 56, 63, 64, 128});
    const int k = 1 + (int)(rng() % 40);
    std::vector<int> colls(k), dt(k), ops(k), algos(k, -1), order(k, -1), planOf(k, -1);
    std::vector<size_t> counts(k);
    for (int i = 0; i < k; i++) {
      colls[i] = (int)(rng() % 5);  // AR, RS, AG, broadcast, reduce
      dt[i] = dts[rng() % 10];
      ops[i] = (int)(rng() % 4);
      counts[i] = (size_t)pick({1, 7, 100, 4096, 65537, 1 << 20, (1 << 22) + 3}) + rng() % 17;
    }
    std::vector<int64_t> cbd(8 * (size_t)k, -1);
    const int64_t geo[4] = {(int64_t)pick({64 << 10, 256 << 10, 512 << 10}), pick({256, 512}),
                            120 * 640 * 8, 640};
    const int64_t ll = pick({0, 64 << 10, 1 << 20});
    const int64_t pol[10] = {pick({0, 0, 1, 2, 3, 4}), pick({0, 1 << 20}), ll, n * ll, pick({0, 1}),
                             64 << 10, pick({0, 1 << 20}), pick({0, 1}), pick({0, 4 << 20, 8 << 20}),
                             pick({0, 64 << 20})};
    const ncclResult_t r = vcclGroupPlanEx(k, colls.data(), counts.data(), dt.data(), ops.data(), n, nch, geo,
                                           (trial & 1) ? pol : nullptr, algos.data(), order.data(),
                                           planOf.data(), cbd.data());
    EXPECT(r == ncclSuccess);
    if (r != ncclSuccess) continue;
    groups++;
    calls += k;
    std::vector<int> seen(k, 0);
    for (int i = 0; i < k; i++) {
      EXPECT(order[i] >= 0 && order[i] < k);
      if (order[i] >= 0 && order[i] < k) seen[order[i]]++;
      EXPECT(planOf[i] >= 0);
      EXPECT(algos[i] == vcclAlgoRing || algos[i] == vcclAlgoLL || algos[i] == vcclAlgoDirect ||
             algos[i] == vcclAlgoLL128);
      const int64_t* c = &cbd[8 * (size_t)i];
      EXPECT(c[0] >= 0 && c[0] <= c[1] && c[1] < nch);
      // the parts cover the call: lo + mid * (channels - 2) + hi (AG in bytes)
      const int64_t nCh = c[1] - c[0] + 1;
      const int64_t cover = nCh == 1 ? c[2] : c[2] + c[3] * (nCh - 2) + c[4];
      const int64_t want = colls[i] == 2 || colls[i] == 3 ? (int64_t)counts[i] * (dt[i] == ncclFloat64 || dt[i] == ncclInt64 ||
                                                                  dt[i] == ncclUint64 ? 8
                                                                  : dt[i] == ncclFloat16 || dt[i] == ncclBfloat16 ? 2
                                                                  : dt[i] <= ncclUint8 ? 1 : 4)
                                         : (int64_t)counts[i];
      EXPECT(cover == want);
    }
    for (int i = 0; i < k; i++) EXPECT(seen[i] == 1);
  }
  // invalid planner inputs are rejected, not read past
  {
    int c = 0, d = ncclFloat32, o = 0, a, ord, p;
    size_t cnt = 0;
    int64_t cb[8];
    const int64_t geo[4] = {512 << 10, 512, 120 * 640 * 8, 640};
    EXPECT(vcclGroupPlanEx(1, &c, &cnt, &d, &o, 2, 8, geo, nullptr, &a, &ord, &p, cb) == ncclInvalidArgument);
    cnt = 10;
    EXPECT(vcclGroupPlanEx(0, &c, &cnt, &d, &o, 2, 8, geo, nullptr, &a, &ord, &p, cb) == ncclInvalidArgument);
    EXPECT(vcclGroupPlanEx(1, &c, &cnt, &d, &o, 2, 0, geo, nullptr, &a, &ord, &p, cb) == ncclInvalidArgument);
    EXPECT(vcclGroupPlanEx(1, &c, &cnt, &d, &o, 2, 8, nullptr, nullptr, &a, &ord, &p, cb) == ncclInvalidArgument);
    d = 99;
    EXPECT(vcclGroupPlanEx(1, &c, &cnt, &d, &o, 2, 8, geo, nullptr, &a, &ord, &p, cb) == ncclInvalidArgument);
  }
  // single-call partitions and the direct all-reduce's chunk lookup
  long parts = 0;
  for (int trial = 0; trial < 20000; trial++) {
    const int n = (int)pick({1, 2, 4, 8}), nch = (int)pick({1, 3, 16, 64});
    const int proto = (int)pick({0, 1, 2});
    const size_t count = 1 + rng() % (3 << 20);
    const int d = dts[rng() % 10];
    int64_t out[8];
    const size_t step = proto == 1 ? 614400 : proto == 0 ? 65536 : 512 << 10;
    EXPECT(vcclRingPartition((int)(rng() % 5), count, (ncclDataType_t)d, n, nch, proto, step,
                             proto == 1 ? 640 : 512, out) == ncclSuccess);
    int64_t ck[3];
    EXPECT(vcclRingChunkOf(count, (ncclDataType_t)d, n, nch, 512 << 10, 512, rng() % count, ck) == ncclSuccess);
    EXPECT(ck[0] >= 0 && ck[0] < nch && ck[1] >= 0 && ck[1] < n);
    parts++;
  }
  // NCCL_ALGO / NCCL_PROTO strings: random garbage never crashes
  const char* words[] = {"Ring", "Tree", "Direct", "LL", "LL128", "Simple", "^", ",", ";", ":", "allreduce",
                         "", " ", "ring", "^ll", "x"};
  long strs = 0;
  for (int trial = 0; trial < 20000; trial++) {
    std::string a, p;
    for (int j = (int)(rng() % 5); j > 0; j--) a += words[rng() % 16];
    for (int j = (int)(rng() % 5); j > 0; j--) p += words[rng() % 16];
    int f = -1, al = -1;
    const ncclResult_t r = vcclAlgoSelection(rng() % 4 ? a.c_str() : nullptr, rng() % 4 ? p.c_str() : nullptr,
                                             &f, &al);
    EXPECT(r == ncclSuccess || r == ncclInvalidUsage);
    strs++;
  }
  // op encoding, error strings, handle checks (no device work)
  for (int op = 0; op < 6; op++)
    for (int d = 0; d < 13; d++) {
      int devOp = -1;
      uint64_t arg = 0;
      (void)vcclHostToDevRedOp((ncclRedOp_t)op, (ncclDataType_t)d, 4, &devOp, &arg);
    }
  for (int e = -1; e < 12; e++) EXPECT(ncclGetErrorString((ncclResult_t)e) != nullptr);
  int v = 0;
  EXPECT(ncclCommCount(nullptr, &v) == ncclInvalidArgument);
  {
    int c = 0, d = ncclFloat32, o = 0, a = -1;
    size_t cnt = 4;
    EXPECT(vcclCommGroupAlgos(nullptr, 1, &c, &cnt, &d, &o, &a) == ncclInvalidArgument);
  }
  EXPECT(ncclAllReduce(nullptr, nullptr, 4, ncclFloat32, ncclSum, nullptr, nullptr) == ncclInvalidArgument);
  EXPECT(ncclGroupStart() == ncclSuccess);
  EXPECT(ncclAllGather(nullptr, nullptr, 4, ncclFloat32, nullptr, nullptr) == ncclInvalidArgument);
  const ncclResult_t ge = ncclGroupEnd();
  EXPECT(ge == ncclInvalidArgument);  // the group fails as a whole (enqueue.cc:2516)
  EXPECT(vcclBuildInfo() != nullptr);
  printf("host_api_check: %ld groups (%ld calls), %ld partitions, %ld selection strings, %d failures\n", groups,
         calls, parts, strs, g_fail);
  return g_fail == 0 ? 0 : 1;
}
