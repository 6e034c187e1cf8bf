/* ORACLE — test infrastructure only (bench.py's cpu_baseline legs; never on
 * the product path).
 *
 * Host-core baselines run by the oracle's own reduce-copy (ref_reduce_copy,
 * reduce_ref.c) on persistent worker threads, each pinned to one CPU of the
 * caller's list and owning one page-aligned slice of every buffer:
 *   - config 2's shape (2-src f32 sum, d = a + b): ref_cpu_bench_{alloc,run,free};
 *   - one rank's share of a ring all-reduce of S bytes over n ranks, as host
 *     work (ref_cpu_bench_rank_*): an n-source f32 sum over m = S / (4 n)
 *     elements into the rank's shard (the reduce-scatter's reductions), then a
 *     copy of the S gathered bytes (the all-gather); `ncopy` = 0 drops the copy.
 * Both shapes:
 *   alloc  mmap the buffers (page size chosen so no page is shared by two
 *          workers' slices) and let each pinned worker FIRST-TOUCH its own
 *          slices, so on a multi-socket host every slice lives on the NUMA
 *          node of the core that works on it (the caller may pin the pages
 *          afterwards with hipHostRegister, which keeps them where they are);
 *   run    the same workers loop passes over their slices for `seconds`, one
 *          barrier per pass, then check their slices bit-exactly (the sum in
 *          the reduce-copy's left-to-right fold order, the copy byte for byte);
 *   free   munmap.
 * Thread creation stays outside the timed region (a pthread_create per call
 * and thread would cost ~ms per pass at hundreds of threads).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

#include "reduce_ref.h"

#define MAXT 1024
#define MAXSRC 16

typedef struct {
  char** bufs; /* [0, nsrc) sources, nsrc dst, nsrc+1 copy src, nsrc+2 copy dst */
  int nsrc, type, esz; /* element type (ncclDataType_t: f32, f16 or bf16) and its size */
  size_t lo, hi;   /* reduce slice */
  size_t clo, chi; /* copy slice */
  int cpu, leader;
  int mode; /* 0 first touch + fill, 1 timed loop, 2 check */
  double seconds;
  pthread_barrier_t* bar;
  volatile int* stop;
  long iters;
  double elapsed;
  int ok;
} worker_t;

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* Deterministic uniform[-1, 1) value of element i of buffer `which`
 * (splitmix64, exactly representable in f32: 24-bit fractions). */
static float val_at(size_t i, int which) {
  uint64_t z = (uint64_t)i * MAXSRC + (uint64_t)which + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)((int32_t)(z >> 40) - (1 << 23)) / (float)(1 << 23);
}

static void pin_to(int cpu) {
  if (cpu < 0) return;
  cpu_set_t s;
  CPU_ZERO(&s);
  CPU_SET(cpu, &s);
  pthread_setaffinity_np(pthread_self(), sizeof(s), &s);
}

/* Element i of buffer `which` in the bench's type: val_at rounded to it. */
static void put(char* buf, size_t i, int type, int which) {
  const float v = val_at(i, which);
  if (type == 7) {
    memcpy(buf + i * 4, &v, 4);
  } else {
    const uint16_t h = type == 6 ? ref_f32_to_f16(v) : ref_f32_to_bf16(v);
    memcpy(buf + i * 2, &h, 2);
  }
}
static uint64_t bits_at(const char* buf, size_t i, int esz) {
  uint64_t x = 0;
  memcpy(&x, buf + i * esz, esz);
  return x;
}

static void* worker(void* arg) {
  worker_t* w = (worker_t*)arg;
  pin_to(w->cpu);
  char** B = w->bufs;
  const int ns = w->nsrc, esz = w->esz;
  char* d = B[ns];
  char *cs = B[ns + 1], *cd = B[ns + 2];
  if (w->mode == 0) {
    for (int s = 0; s < ns; s++)
      for (size_t i = w->lo; i < w->hi; i++) put(B[s], i, w->type, s);
    if (w->hi > w->lo) memset(d + w->lo * esz, 0, (w->hi - w->lo) * esz);
    for (size_t i = w->clo; i < w->chi; i++) put(cs, i, w->type, MAXSRC - 1);
    if (w->chi > w->clo) memset(cd + w->clo * esz, 0, (w->chi - w->clo) * esz);
    return NULL;
  }
  if (w->mode == 2) {
    /* the sum in the reduce-copy's left-to-right fold order, element by
     * element through the oracle's own primitive (ref_reduce1) */
    int ok = 1;
    for (size_t i = w->lo; i < w->hi && ok; i++) {
      uint64_t acc = bits_at(B[0], i, esz);
      for (int s = 1; s < ns; s++) acc = ref_reduce1(0, w->type, 0, acc, bits_at(B[s], i, esz));
      ok = acc == bits_at(d, i, esz);
    }
    if (ok && w->chi > w->clo) ok = memcmp(cs + w->clo * esz, cd + w->clo * esz, (w->chi - w->clo) * esz) == 0;
    w->ok = ok;
    return NULL;
  }
  const void* srcs[MAXSRC];
  for (int s = 0; s < ns; s++) srcs[s] = B[s] + w->lo * esz;
  void* dsts[1] = {d + w->lo * esz};
  const void* csrc[1] = {cs + w->clo * esz};
  void* cdst[1] = {cd + w->clo * esz};
  const double t0 = now_s();
  long it = 0;
  for (;;) {
    if (w->hi > w->lo)
      ref_reduce_copy(0, w->type, 0, NULL, 0, 0, ns, srcs, 1, dsts, w->hi - w->lo, 1);
    if (w->chi > w->clo)  /* the gather: a one-source reduce-copy is a copy */
      ref_reduce_copy(0, w->type, 0, NULL, 0, 0, 1, csrc, 1, cdst, w->chi - w->clo, 1);
    it++;
    /* thread 0 decides when to stop; everyone sees the same decision */
    if (w->leader && now_s() - t0 >= w->seconds) *w->stop = 1;
    pthread_barrier_wait(w->bar);
    const int stop = *w->stop;
    pthread_barrier_wait(w->bar);
    if (stop) break;
  }
  w->iters = it;
  w->elapsed = now_s() - t0;
  return NULL;
}

/* Elements per worker slice: whole 2 MiB huge pages when every slice spans
 * at least one (huge pages advised), else whole 4 KiB pages (huge pages
 * refused, so a 2 MiB page is never shared by two workers' first touches). */
static size_t slice_elems(size_t n, int nthreads, int esz, int* huge) {
  const size_t grain4k = 4096 / esz, grain2m = (2u << 20) / esz;
  const size_t raw = (n + nthreads - 1) / nthreads;
  const int h = raw >= grain2m;
  if (huge) *huge = h;
  const size_t g = h ? grain2m : grain4k;
  return (raw + g - 1) / g * g;
}

static void slice(size_t n, int nthreads, int esz, int t, size_t* lo, size_t* hi) {
  const size_t per = slice_elems(n, nthreads, esz, NULL);
  *lo = per * t < n ? per * t : n;
  *hi = per * (t + 1) < n ? per * (t + 1) : n;
  if (t == 0) *lo = 0;
}

static int run_workers(char** bufs, int nsrc, int type, size_t m, size_t ncopy, int nthreads, const int* cpus,
                       int mode, double seconds, long* iters, double* elapsed) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > MAXT) nthreads = MAXT;
  static worker_t ws[MAXT];
  pthread_t tids[MAXT];
  pthread_barrier_t bar;
  volatile int stop = 0;
  pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
  for (int t = 0; t < nthreads; t++) {
    worker_t* w = &ws[t];
    memset(w, 0, sizeof(*w));
    w->bufs = bufs;
    w->nsrc = nsrc;
    w->type = type;
    w->esz = ref_type_size(type);
    slice(m, nthreads, w->esz, t, &w->lo, &w->hi);
    slice(ncopy, nthreads, w->esz, t, &w->clo, &w->chi);
    w->cpu = cpus ? cpus[t] : -1;
    w->leader = t == 0;
    w->mode = mode;
    w->seconds = seconds;
    w->bar = &bar;
    w->stop = &stop;
  }
  /* worker 0 is the calling thread: give it back its own affinity after */
  cpu_set_t own;
  const int haveOwn = pthread_getaffinity_np(pthread_self(), sizeof(own), &own) == 0;
  for (int t = 1; t < nthreads; t++) pthread_create(&tids[t], NULL, worker, &ws[t]);
  worker(&ws[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(tids[t], NULL);
  if (haveOwn) pthread_setaffinity_np(pthread_self(), sizeof(own), &own);
  if (elapsed) *elapsed = ws[0].elapsed;  /* thread 0's timed loop (all threads in step) */
  pthread_barrier_destroy(&bar);
  if (iters) *iters = ws[0].iters;
  int ok = 1;
  if (mode == 2)
    for (int t = 0; t < nthreads; t++) ok &= ws[t].ok;
  return ok;
}

static size_t map_bytes(size_t n, int esz) { return (n * esz + 4095) / 4096 * 4096; }

static void* map_buf(size_t n, int esz, int nthreads) {
  if (n == 0) return NULL;
  void* p = mmap(NULL, map_bytes(n, esz), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return NULL;
  int huge;
  slice_elems(n, nthreads, esz, &huge);
  madvise(p, map_bytes(n, esz), huge ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
  return p;
}

static int type_ok(int type) { return type == 6 || type == 7 || type == 9; }

void ref_cpu_bench_rank_free(void** bufs, size_t m, int nsrc, size_t ncopy, int type) {
  for (int i = 0; i < nsrc + 3; i++) {
    if (!bufs[i]) continue;
    munmap(bufs[i], map_bytes(i <= nsrc ? m : ncopy, ref_type_size(type)));
    bufs[i] = NULL;
  }
}

int ref_cpu_bench_rank_alloc(size_t m, int nsrc, size_t ncopy, int type, int nthreads, const int* cpus,
                             void** bufs) {
  if (nsrc < 1 || nsrc > MAXSRC || m == 0 || !type_ok(type)) return -1;
  for (int i = 0; i < nsrc + 3; i++) bufs[i] = NULL;
  for (int i = 0; i < nsrc + 3; i++) {
    const size_t n = i <= nsrc ? m : ncopy;
    if (n && !(bufs[i] = map_buf(n, ref_type_size(type), nthreads))) {
      ref_cpu_bench_rank_free(bufs, m, nsrc, ncopy, type);
      return -1;
    }
  }
  run_workers((char**)bufs, nsrc, type, m, ncopy, nthreads, cpus, 0, 0, NULL, NULL);
  return 0;
}

/* Returns 1 when every slice checks bit-exactly after the timed loop. */
int ref_cpu_bench_rank_run(void** bufs, size_t m, int nsrc, size_t ncopy, int type, int nthreads,
                           const int* cpus, double seconds, long* iters, double* elapsed) {
  run_workers((char**)bufs, nsrc, type, m, ncopy, nthreads, cpus, 1, seconds, iters, elapsed);
  return run_workers((char**)bufs, nsrc, type, m, ncopy, nthreads, cpus, 2, 0, NULL, NULL);
}

/* Config 2's shape: the f32 rank shape with two sources and no copy. */
int ref_cpu_bench_alloc(size_t n, int nthreads, const int* cpus, void** a, void** b, void** d) {
  void* bufs[5];
  if (ref_cpu_bench_rank_alloc(n, 2, 0, 7, nthreads, cpus, bufs) != 0) return -1;
  *a = bufs[0];
  *b = bufs[1];
  *d = bufs[2];
  return 0;
}

int ref_cpu_bench_run(void* a, void* b, void* d, size_t n, int nthreads, const int* cpus,
                      double seconds, long* iters, double* elapsed) {
  void* bufs[5] = {a, b, d, NULL, NULL};
  return ref_cpu_bench_rank_run(bufs, n, 2, 0, 7, nthreads, cpus, seconds, iters, elapsed);
}

void ref_cpu_bench_free(void* a, void* b, void* d, size_t n) {
  void* bufs[5] = {a, b, d, NULL, NULL};
  ref_cpu_bench_rank_free(bufs, n, 2, 0, 7);
}
