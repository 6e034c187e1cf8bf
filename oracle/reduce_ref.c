/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see reduce_ref.h for scope and parity
 * status).  Plain C99, no compiler half/bfloat types: every narrow-float
 * rounding is done on integer bits so the restatement does not share code
 * (or bugs) with the HIP product path.
 */
#include "reduce_ref.h"

#include <math.h>
#include <pthread.h>
#include <string.h>

int ref_type_size(int type) {
  switch (type) {
    case R_I8: case R_U8: case R_F8E4M3: case R_F8E5M2: return 1;
    case R_F16: case R_BF16: return 2;
    case R_I32: case R_U32: case R_F32: return 4;
    case R_I64: case R_U64: case R_F64: return 8;
    default: return 0;
  }
}

static int is_signed_int(int t) { return t == R_I8 || t == R_I32 || t == R_I64; }
static int is_int(int t) { return t <= R_U64; }

/* ---------------------------------------------------------------- floats */
static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint64_t d2u(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static double u2d(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }

float ref_f16_to_f32(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1f;
  uint32_t man = h & 0x3ffu;
  if (exp == 0x1f) return u2f(sign | 0x7f800000u | (man << 13));  /* inf / NaN */
  if (exp == 0) {
    if (man == 0) return u2f(sign);
    /* subnormal: value = man * 2^-24, exact in f32 */
    float v = (float)man * 5.9604644775390625e-08f;
    return sign ? -v : v;
  }
  return u2f(sign | ((exp + 112) << 23) | (man << 13));
}

/* Round-to-nearest-even of |x| (given as f32 bits) to binary16. */
uint16_t ref_f32_to_f16(float f) {
  uint32_t u = f2u(f);
  uint16_t sign = (uint16_t)((u >> 16) & 0x8000u);
  uint32_t a = u & 0x7fffffffu;
  if (a >= 0x7f800000u) {                       /* inf or NaN */
    if (a == 0x7f800000u) return sign | 0x7c00u;
    return sign | 0x7e00u | (uint16_t)((a >> 13) & 0x3ffu); /* quiet NaN */
  }
  int32_t e = (int32_t)(a >> 23) - 127;         /* unbiased exponent */
  if (e > 15) return sign | 0x7c00u;            /* overflow (also >= 65520) */
  uint32_t m = (a & 0x7fffffu) | 0x800000u;     /* 24-bit significand */
  if (e >= -14) {                               /* normal result */
    uint32_t keep = m >> 13, rem = m & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (keep & 1))) keep++;
    uint32_t r = ((uint32_t)(e + 15) << 10) + (keep - 0x400u);  /* carry ok */
    return sign | (uint16_t)r;                  /* may round up to inf */
  }
  if (a < 0x33000000u) return sign;             /* < 2^-25: rounds to 0 */
  /* subnormal: value = m * 2^(e-23); unit = 2^-24 -> shift = -(e+1) */
  int shift = -e - 1;                           /* 14 .. 24 */
  uint32_t keep = m >> shift, rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
  if (rem > half || (rem == half && (keep & 1))) keep++;
  return sign | (uint16_t)keep;                 /* may carry into normal */
}

float ref_bf16_to_f32(uint16_t h) { return u2f((uint32_t)h << 16); }

uint16_t ref_f32_to_bf16(float f) {
  uint32_t u = f2u(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x0040u); /* qNaN */
  uint32_t lsb = (u >> 16) & 1u;
  return (uint16_t)((u + 0x7fffu + lsb) >> 16);
}

/* fp8: E5M2 is binary16 truncated to 8 bits; E4M3 is decoded field by field. */
float ref_fp8_to_f32(int type, uint8_t b) {
  if (type == R_F8E5M2) return ref_f16_to_f32((uint16_t)(b << 8));
  uint32_t e = (b >> 3) & 15u, m = b & 7u;
  float v;
  if (e == 15 && m == 7) return u2f(0x7fc00000u);
  if (e == 0) v = ldexpf((float)m, -9);
  else v = ldexpf((float)(8 + m), (int)e - 10);
  return (b & 0x80u) ? -v : v;
}

/* RN-even of a finite f32 to `mbits` mantissa bits, exponent bias `bias`,
 * computed on the 24-bit integer significand. */
uint8_t ref_f32_to_fp8(int type, float f) {
  const int mbits = type == R_F8E4M3 ? 3 : 2, bias = type == R_F8E4M3 ? 7 : 15;
  const uint32_t maxCode = type == R_F8E4M3 ? 0x7eu : 0x7bu;
  uint32_t u = f2u(f), sign = (u >> 24) & 0x80u, a = u & 0x7fffffffu;
  if (a > 0x7f800000u) return 0x7fu;
  if (a == 0) return (uint8_t)sign;
  int e = (int)(a >> 23) - 127, emin = 1 - bias;
  uint64_t m = (a & 0x7fffffu) | 0x800000u;
  if ((a >> 23) == 0) { m = a & 0x7fffffu; e = -126; }  /* f32 subnormal */
  int ue = (e > emin ? e : emin) - mbits;                 /* result unit 2^ue */
  int shift = ue - (e - 23);
  uint64_t q = 0;
  if (shift < 60) {
    uint64_t rem = m & ((1ull << shift) - 1), half = 1ull << (shift - 1);
    q = m >> shift;
    if (rem > half || (rem == half && (q & 1))) q++;
  }
  uint64_t code;
  if (e >= emin) code = ((uint64_t)(e + bias) << mbits) + q - (1ull << mbits);
  else code = q;                                        /* subnormal; may reach min normal */
  if (e > 30 || code > maxCode) code = maxCode;
  return (uint8_t)(sign | code);
}

/* IEEE minNum / maxNum (fminf/fmaxf, __hmin/__hmax: NaN-avoiding). */
static double minnum(double x, double y, int isMin) {
  if (isnan(x)) return y;
  if (isnan(y)) return x;
  if (isMin) return (y < x) ? y : x;
  return (y > x) ? y : x;
}

/* ---------------------------------------------------------------- op arg */
int ref_host_to_dev_redop(int op, int type, int nranks, int* devOp, uint64_t* opArg) {
  int nbits = 8 * ref_type_size(type);
  if (nbits <= 0) return 4;                     /* ncclInvalidArgument */
  uint64_t allBits = ~0ull >> (64 - nbits);
  uint64_t signBit = allBits ^ (allBits >> 1);
  *opArg = 0;
  switch (op) {
    case R_OP_SUM: *devOp = R_SUM; return 0;
    case R_OP_PROD: *devOp = R_PROD; return 0;
    case R_OP_MIN: case R_OP_MAX:               /* enqueue.cc:2240-2256 */
      *devOp = R_MINMAX;
      if (is_signed_int(type)) *opArg ^= signBit;
      if (op == R_OP_MAX) *opArg ^= allBits;
      return 0;
    case R_OP_AVG:                              /* enqueue.cc:2257-2290 */
      if (is_int(type)) {
        *devOp = R_SUMPOSTDIV;
        *opArg = ((uint64_t)nranks << 1) | (uint64_t)is_signed_int(type);
      } else {
        *devOp = R_PREMULSUM;
        double inv = 1.0 / nranks;
        if (type == R_F16) *opArg = ref_f32_to_f16((float)inv);
        else if (type == R_BF16) *opArg = ref_f32_to_bf16((float)inv);
        else if (type == R_F8E4M3 || type == R_F8E5M2) *opArg = ref_f32_to_fp8(type, (float)inv);
        else if (type == R_F32) *opArg = f2u((float)inv);
        else *opArg = d2u(inv);
      }
      return 0;
    default: return 4;
  }
}

/* ---------------------------------------------------------------- elements */
static uint64_t mask_of(int type) {
  int n = ref_type_size(type);
  return n == 8 ? ~0ull : ((1ull << (8 * n)) - 1);
}

/* Narrow-float op through f32 then one RN-even rounding.  Exactly the
 * __hadd/__hmul result: f32 carries 24 >= 2*11+2 significand bits, so the
 * double rounding is innocuous for + and * (Figueroa). */
static uint64_t narrow_op(int devOp, int type, uint64_t opArg, uint64_t a, uint64_t b) {
  float x = type == R_F16 ? ref_f16_to_f32((uint16_t)a) : ref_bf16_to_f32((uint16_t)a);
  float y = type == R_F16 ? ref_f16_to_f32((uint16_t)b) : ref_bf16_to_f32((uint16_t)b);
  float r;
  switch (devOp) {
    case R_PROD: r = x * y; break;
    case R_MINMAX: r = (float)minnum(x, y, (opArg & 1) == 0); break;
    default: r = x + y; break;                  /* Sum, PreMulSum */
  }
  return type == R_F16 ? ref_f32_to_f16(r) : ref_f32_to_bf16(r);
}

uint64_t ref_reduce1(int devOp, int type, uint64_t opArg, uint64_t a, uint64_t b) {
  uint64_t m = mask_of(type);
  a &= m; b &= m;
  if (is_int(type)) {                           /* run as unsigned (generate.py:129-137) */
    switch (devOp) {
      case R_PROD: return (a * b) & m;
      case R_MINMAX: {                          /* reduce_kernel.h:193-198 */
        uint64_t x = opArg & m;
        return ((a ^ x) < (b ^ x)) ? a : b;
      }
      default: return (a + b) & m;              /* Sum, PreMulSum, SumPostDiv */
    }
  }
  if (type == R_F16 || type == R_BF16) return narrow_op(devOp, type, opArg, a, b);
  if (type == R_F8E4M3 || type == R_F8E5M2) {
    /* reduce_kernel.h:309-321: fp8(__hop(half(a), half(b))) — the op in f32
     * is exact for fp8 operands, then RN to binary16, then RN-satfinite to
     * fp8 (two roundings, as the reference). */
    float x = ref_fp8_to_f32(type, (uint8_t)a), y = ref_fp8_to_f32(type, (uint8_t)b), r;
    switch (devOp) {
      case R_PROD: r = x * y; break;
      case R_MINMAX: r = (float)minnum(x, y, (opArg & 1) == 0); break;
      default: r = x + y; break;
    }
    return ref_f32_to_fp8(type, ref_f16_to_f32(ref_f32_to_f16(r)));
  }
  if (type == R_F32) {
    float x = u2f((uint32_t)a), y = u2f((uint32_t)b), r;
    switch (devOp) {
      case R_PROD: r = x * y; break;
      case R_MINMAX: r = (float)minnum(x, y, (opArg & 1) == 0); break;
      default: r = x + y; break;
    }
    return f2u(r);
  }
  /* f64 */
  double x = u2d(a), y = u2d(b), r;
  switch (devOp) {
    case R_PROD: r = x * y; break;
    case R_MINMAX: r = minnum(x, y, (opArg & 1) == 0); break;
    default: r = x + y; break;
  }
  return d2u(r);
}

/* PreMulSum preOp: x * scalar in T (reduce_kernel.h:522-583). */
uint64_t ref_preop1(int devOp, int type, uint64_t opArg, uint64_t a) {
  if (devOp != R_PREMULSUM) return a & mask_of(type);
  return ref_reduce1(R_PROD, type, 0, a, opArg);
}

/* SumPostDiv postOp (reduce_kernel.h:641-688): truncating divide through
 * the reciprocal + one fix-up, on the unsigned kernel type. */
uint64_t ref_postop1(int devOp, int type, uint64_t opArg, uint64_t a) {
  uint64_t m = mask_of(type);
  a &= m;
  if (devOp != R_SUMPOSTDIV) return a;
  int isSigned = (int)(opArg & 1);
  uint32_t divisor = (uint32_t)((opArg >> 1) & 0x7fffffffu);
  int wide = ref_type_size(type) == 8;
  int xneg = isSigned && (a & ~(m >> 1));
  uint64_t xabs = xneg ? ((0 - a) & m) : a;
  uint64_t q;
  if (wide) {
    uint64_t recip = ~0ull / divisor;
    q = (uint64_t)(((unsigned __int128)xabs * recip) >> 64);
    if (xabs - q * divisor >= divisor) q += 1;
  } else {
    uint32_t recip = 0xffffffffu / divisor;
    uint32_t x32 = (uint32_t)xabs;
    uint32_t q32 = (uint32_t)(((uint64_t)x32 * recip) >> 32);
    if (x32 - q32 * divisor >= divisor) q32 += 1;
    q = q32;
  }
  return (xneg ? (0 - q) : q) & m;
}

/* ---------------------------------------------------------------- arrays */
static uint64_t ld(const void* p, size_t i, int sz) {
  uint64_t v = 0;
  memcpy(&v, (const char*)p + i * sz, sz);     /* little-endian host */
  return v;
}
static void st(void* p, size_t i, int sz, uint64_t v) { memcpy((char*)p + i * sz, &v, sz); }

typedef struct {
  int devOp, type, preOpSrcs, postOp, nSrcs, nDsts;
  uint64_t redArg;
  const uint64_t* preOpArgs;
  const void* const* srcs;
  void* const* dsts;
  size_t lo, hi;
} rc_job;

/* Fast path for the benchmark shape (f32 sum, no pre/post op): a plain loop
 * the host compiler can vectorise; same per-element semantics. */
static int rc_fast_f32_sum(const rc_job* j) {
  if (j->type != R_F32 || j->devOp != R_SUM || j->preOpSrcs || j->postOp) return 0;
  for (size_t i = j->lo; i < j->hi;) {
    float buf[1024];
    size_t n = j->hi - i < 1024 ? j->hi - i : 1024;
    const float* s0 = (const float*)j->srcs[0] + i;
    for (size_t k = 0; k < n; k++) buf[k] = s0[k];
    for (int s = 1; s < j->nSrcs; s++) {
      const float* sp = (const float*)j->srcs[s] + i;
      for (size_t k = 0; k < n; k++) buf[k] = buf[k] + sp[k];
    }
    for (int d = 0; d < j->nDsts; d++) memcpy((float*)j->dsts[d] + i, buf, n * 4);
    i += n;
  }
  return 1;
}

static void* rc_run(void* arg) {
  const rc_job* j = (const rc_job*)arg;
  if (rc_fast_f32_sum(j)) return NULL;
  int sz = ref_type_size(j->type);
  for (size_t i = j->lo; i < j->hi; i++) {
    uint64_t acc = ld(j->srcs[0], i, sz);
    if (0 < j->preOpSrcs) acc = ref_preop1(j->devOp, j->type, j->preOpArgs[0], acc);
    for (int s = 1; s < j->nSrcs; s++) {
      uint64_t v = ld(j->srcs[s], i, sz);
      if (s < j->preOpSrcs) v = ref_preop1(j->devOp, j->type, j->preOpArgs[s], v);
      acc = ref_reduce1(j->devOp, j->type, j->redArg, acc, v);
    }
    if (j->postOp) acc = ref_postop1(j->devOp, j->type, j->redArg, acc);
    for (int d = 0; d < j->nDsts; d++) st(j->dsts[d], i, sz, acc);
  }
  return NULL;
}

void ref_reduce_copy(int devOp, int type, uint64_t redArg, const uint64_t* preOpArgs,
                     int preOpSrcs, int postOp, int nSrcs, const void* const* srcs,
                     int nDsts, void* const* dsts, size_t nElts, int nthreads) {
  if (nSrcs <= 0 || nDsts <= 0 || nElts == 0) return;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  rc_job jobs[256];
  pthread_t tids[256];
  size_t per = (nElts + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; t++) {
    rc_job* j = &jobs[t];
    j->devOp = devOp; j->type = type; j->preOpSrcs = preOpSrcs; j->postOp = postOp;
    j->nSrcs = nSrcs; j->nDsts = nDsts; j->redArg = redArg; j->preOpArgs = preOpArgs;
    j->srcs = srcs; j->dsts = dsts;
    j->lo = per * t < nElts ? per * t : nElts;
    j->hi = per * (t + 1) < nElts ? per * (t + 1) : nElts;
  }
  if (nthreads == 1) { rc_run(&jobs[0]); return; }
  for (int t = 1; t < nthreads; t++) pthread_create(&tids[t], NULL, rc_run, &jobs[t]);
  rc_run(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(tids[t], NULL);
}

void ref_ring_fold(int devOp, int type, uint64_t redArg, int preOp, int nranks,
                   const void* const* inputs, const int32_t* owner, void* out,
                   size_t nElts) {
  int sz = ref_type_size(type);
  for (size_t i = 0; i < nElts; i++) {
    int o = owner[i];
    int k = (o + 1) % nranks;                   /* step 0: directSend of preOp(x) */
    uint64_t acc = ld(inputs[k], i, sz);
    if (preOp) acc = ref_preop1(devOp, type, redArg, acc);
    for (int j = 2; j <= nranks; j++) {         /* own (+) recv, ending at o */
      k = (o + j) % nranks;
      uint64_t own = ld(inputs[k], i, sz);
      if (preOp) own = ref_preop1(devOp, type, redArg, own);
      acc = ref_reduce1(devOp, type, redArg, own, acc);
    }
    acc = ref_postop1(devOp, type, redArg, acc);
    st(out, i, sz, acc);
  }
}

void ref_chain_fold(int devOp, int type, uint64_t redArg, int preOp, int nranks,
                    const void* const* inputs, void* out, size_t nElts) {
  int sz = ref_type_size(type);
  for (size_t i = 0; i < nElts; i++) {
    uint64_t acc = ld(inputs[nranks - 1], i, sz);
    if (preOp) acc = ref_preop1(devOp, type, redArg, acc);
    for (int p = nranks - 2; p >= 0; p--) {     /* LL: peer (+) own */
      uint64_t own = ld(inputs[p], i, sz);
      if (preOp) own = ref_preop1(devOp, type, redArg, own);
      acc = ref_reduce1(devOp, type, redArg, acc, own);
    }
    acc = ref_postop1(devOp, type, redArg, acc);
    st(out, i, sz, acc);
  }
}
