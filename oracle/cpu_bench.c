/* ORACLE — test infrastructure only (bench.py's cpu_baseline leg; never on
 * the product path).
 *
 * Host-core baseline of BASELINE config 2's shape (2-src f32 sum, dst =
 * a + b) run by the oracle's own reduce-copy (ref_reduce_copy, reduce_ref.c)
 * on persistent worker threads, each pinned to one CPU of the caller's list
 * and owning one page-aligned slice of every buffer:
 *   ref_cpu_bench_alloc  mmap the three buffers (page size chosen so no page
 *                        is shared by two workers' slices) and let
 *                        each pinned worker FIRST-TOUCH its own slices, so on
 *                        a multi-socket host every slice lives on the NUMA
 *                        node of the core that reduces it (the caller may pin
 *                        the pages afterwards with hipHostRegister, which
 *                        keeps them where they are);
 *   ref_cpu_bench_run    the same workers loop reduce-copies over their
 *                        slices for `seconds`, one barrier per pass, then
 *                        check their slices bit-exactly;
 *   ref_cpu_bench_free   munmap.
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

typedef struct {
  float *a, *b, *d;
  size_t lo, hi;
  int cpu;
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
  uint64_t z = (uint64_t)i * 2 + (uint64_t)which + 0x9E3779B97F4A7C15ull;
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

static void* worker(void* arg) {
  worker_t* w = (worker_t*)arg;
  pin_to(w->cpu);
  if (w->mode == 0) {
    for (size_t i = w->lo; i < w->hi; i++) {
      w->a[i] = val_at(i, 0);
      w->b[i] = val_at(i, 1);
      w->d[i] = 0.0f;
    }
    return NULL;
  }
  if (w->mode == 2) {
    int ok = 1;
    for (size_t i = w->lo; i < w->hi && ok; i++) ok = w->d[i] == w->a[i] + w->b[i];
    w->ok = ok;
    return NULL;
  }
  const void* srcs[2] = {w->a + w->lo, w->b + w->lo};
  void* dsts[1] = {w->d + w->lo};
  const double t0 = now_s();
  long it = 0;
  for (;;) {
    if (w->hi > w->lo)
      ref_reduce_copy(0, 7 /* ncclFloat32 */, 0, NULL, 0, 0, 2, srcs, 1, dsts, w->hi - w->lo, 1);
    it++;
    /* thread 0 decides when to stop; everyone sees the same decision */
    if (w->lo == 0 && now_s() - t0 >= w->seconds) *w->stop = 1;
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
static size_t slice_elems(size_t n, int nthreads, int* huge) {
  const size_t grain4k = 1024, grain2m = 512 * 1024;
  const size_t raw = (n + nthreads - 1) / nthreads;
  const int h = raw >= grain2m;
  if (huge) *huge = h;
  const size_t g = h ? grain2m : grain4k;
  return (raw + g - 1) / g * g;
}

static int run_workers(float* a, float* b, float* d, size_t n, int nthreads, const int* cpus,
                       int mode, double seconds, long* iters, double* elapsed) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > MAXT) nthreads = MAXT;
  static worker_t ws[MAXT];
  pthread_t tids[MAXT];
  pthread_barrier_t bar;
  volatile int stop = 0;
  pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
  const size_t per = slice_elems(n, nthreads, NULL);
  for (int t = 0; t < nthreads; t++) {
    worker_t* w = &ws[t];
    memset(w, 0, sizeof(*w));
    w->a = a; w->b = b; w->d = d;
    w->lo = per * t < n ? per * t : n;
    w->hi = per * (t + 1) < n ? per * (t + 1) : n;
    if (t == 0) w->lo = 0;
    w->cpu = cpus ? cpus[t] : -1;
    w->mode = mode;
    w->seconds = seconds;
    w->bar = &bar;
    w->stop = &stop;
  }
  for (int t = 1; t < nthreads; t++) pthread_create(&tids[t], NULL, worker, &ws[t]);
  worker(&ws[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(tids[t], NULL);
  if (elapsed) *elapsed = ws[0].elapsed;  /* thread 0's timed loop (all threads in step) */
  pthread_barrier_destroy(&bar);
  if (iters) *iters = ws[0].iters;
  int ok = 1;
  if (mode == 2)
    for (int t = 0; t < nthreads; t++) ok &= ws[t].ok;
  return ok;
}

int ref_cpu_bench_alloc(size_t n, int nthreads, const int* cpus, void** a, void** b, void** d) {
  const size_t bytes = (n * 4 + 4095) / 4096 * 4096;
  void* p[3];
  for (int i = 0; i < 3; i++) {
    p[i] = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p[i] == MAP_FAILED) return -1;
    int huge;
    slice_elems(n, nthreads, &huge);
    madvise(p[i], bytes, huge ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
  }
  run_workers((float*)p[0], (float*)p[1], (float*)p[2], n, nthreads, cpus, 0, 0, NULL, NULL);
  *a = p[0];
  *b = p[1];
  *d = p[2];
  return 0;
}

/* Returns 1 when every slice checks bit-exactly after the timed loop. */
int ref_cpu_bench_run(void* a, void* b, void* d, size_t n, int nthreads, const int* cpus,
                      double seconds, long* iters, double* elapsed) {
  run_workers((float*)a, (float*)b, (float*)d, n, nthreads, cpus, 1, seconds, iters, elapsed);
  return run_workers((float*)a, (float*)b, (float*)d, n, nthreads, cpus, 2, 0, NULL, NULL);
}

void ref_cpu_bench_free(void* a, void* b, void* d, size_t n) {
  const size_t bytes = (n * 4 + 4095) / 4096 * 4096;
  munmap(a, bytes);
  munmap(b, bytes);
  munmap(d, bytes);
}
