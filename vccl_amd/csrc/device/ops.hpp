// Reduction-op functors for the bucket-reduction path, written for gfx950.
//
// Semantics follow VCCL src/device/reduce_kernel.h (file:line per functor);
// the implementation is CDNA4-native: 16-byte packs are processed as plain
// element loops that hipcc lowers to packed VALU (v_pk_add_f32, v_pk_add_f16,
// v_pk_mul_f32, ...); bf16 goes through f32 and v_cvt_pk_bf16_f32 (RN-even,
// NaN-preserving), which is bit-identical to __hadd/__hmul on bf16 because f32
// carries 24 >= 2*8+2 significand bits (no double-rounding error).
//
// Kernel element types (KT) follow generate.py:129-137: signed integers run the
// unsigned kernel (two's-complement wrap; MinMax restores signed order through
// the xormask, reduce_kernel.h:193-198 / enqueue.cc:2240-2256).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vccl {

// ---------------------------------------------------------------- bf16 bits
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __builtin_bit_cast(float, (uint32_t)h << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);  // v_cvt_pk_bf16_f32: RN-even
}

struct bf16_t { uint16_t bits; };  // storage-only tag type

// ---------------------------------------------------------------- fp8 bits
// OCP FP8 (gfx950's native formats): E4M3 ("fn": bias 7, no infinity, NaN =
// S.1111.111, max 448) and E5M2 (bias 15, IEEE-like, max 57344).  The
// reference reduces fp8 through __half (reduce_kernel.h:309-321): widen to
// half (exact), __hadd/__hmul/__hmin/__hmax in half (one RN-even rounding),
// narrow with __NV_SATFINITE (RN-even; beyond max finite -> max finite,
// infinity -> max finite, NaN -> NaN).  Here the same two roundings run on
// _Float16 (v_add_f16 / v_mul_f16 are correctly rounded) plus integer
// narrowing on the half bits.
struct f8e4m3_t { uint8_t bits; };
struct f8e5m2_t { uint8_t bits; };

__device__ __forceinline__ _Float16 h_of_bits(uint16_t b) { return __builtin_bit_cast(_Float16, b); }
__device__ __forceinline__ uint16_t bits_of_h(_Float16 h) { return __builtin_bit_cast(uint16_t, h); }

// E5M2 is binary16 with the low 8 mantissa bits dropped: widening is a shift.
__device__ __forceinline__ _Float16 f8_to_h(f8e5m2_t x) { return h_of_bits((uint16_t)(x.bits << 8)); }
// E4M3 magnitude bits placed in binary16 with exponent bias 15 are the value
// times 2^-8 (subnormals included), so one exact multiply by 256 rebiases.
__device__ __forceinline__ _Float16 f8_to_h(f8e4m3_t x) {
  const uint32_t a = x.bits & 0x7fu;
  if (a == 0x7fu) return h_of_bits(0x7fffu);
  const _Float16 v = h_of_bits((uint16_t)(a << 7)) * (_Float16)256.0f;
  return (x.bits & 0x80u) ? -v : v;
}
// binary16 -> E5M2, RN-even on the dropped 8 bits, saturating.
__device__ __forceinline__ uint8_t h_to_e5m2(_Float16 h) {
  const uint32_t b = bits_of_h(h), a = b & 0x7fffu, s = (b >> 8) & 0x80u;
  if (a > 0x7c00u) return 0x7fu;
  uint32_t r = (a + 0x7fu + ((a >> 8) & 1u)) >> 8;
  if (r > 0x7bu) r = 0x7bu;
  return (uint8_t)(s | r);
}
// binary16 -> E4M3, RN-even, saturating.  Normal E4M3 results (half exponent
// >= 9) drop 7 mantissa bits and rebias by 8 exponents; below 2^-6 the result
// counts units of 2^-9: rint(|h| * 512) (exact scaling in f32).
__device__ __forceinline__ uint8_t h_to_e4m3(_Float16 h) {
  const uint32_t b = bits_of_h(h), a = b & 0x7fffu, s = (b >> 8) & 0x80u;
  if (a > 0x7c00u) return 0x7fu;
  uint32_t code;
  if (a >= (9u << 10)) code = ((a + 0x3fu + ((a >> 7) & 1u)) >> 7) - (8u << 3);
  else code = (uint32_t)__builtin_rintf((float)h_of_bits((uint16_t)a) * 512.0f);
  if (code > 0x7eu) code = 0x7eu;
  return (uint8_t)(s | code);
}
__device__ __forceinline__ f8e4m3_t f8_from_h(_Float16 h, f8e4m3_t) { return {h_to_e4m3(h)}; }
__device__ __forceinline__ f8e5m2_t f8_from_h(_Float16 h, f8e5m2_t) { return {h_to_e5m2(h)}; }

// ---------------------------------------------------------------- helpers
template <typename T> struct IsFloat { static constexpr bool value = false; };
template <> struct IsFloat<_Float16> { static constexpr bool value = true; };
template <> struct IsFloat<float> { static constexpr bool value = true; };
template <> struct IsFloat<double> { static constexpr bool value = true; };
template <> struct IsFloat<bf16_t> { static constexpr bool value = true; };
template <> struct IsFloat<f8e4m3_t> { static constexpr bool value = true; };
template <> struct IsFloat<f8e5m2_t> { static constexpr bool value = true; };
template <typename T> struct IsF8 { static constexpr bool value = false; };
template <> struct IsF8<f8e4m3_t> { static constexpr bool value = true; };
template <> struct IsF8<f8e5m2_t> { static constexpr bool value = true; };

template <typename T>
__device__ __forceinline__ T from_arg(uint64_t arg) {
  union { uint64_t u; T v; } x;
  x.u = arg;
  return x.v;
}

// IEEE minNum/maxNum as fminf/fmaxf (reduce_kernel.h:264-265) and
// __hmin/__hmax (:282-284, :297-299): NaN-avoiding.
__device__ __forceinline__ float minmax_f32(float a, float b, bool isMin) {
  return isMin ? __builtin_fminf(a, b) : __builtin_fmaxf(a, b);
}

// ---------------------------------------------------------------- Sum
// reduce_kernel.h:181-186 (generic), :267-272 (f16 __hadd), :291-293 (bf16)
template <typename T> struct FnSum {
  using EltType = T;
  static constexpr bool kPreOp = false, kPostOp = false;
  __device__ FnSum(uint64_t = 0) {}
  __device__ __forceinline__ T reduce(T a, T b) const { return a + b; }
  __device__ __forceinline__ T preOp(T a) const { return a; }
  __device__ __forceinline__ T postOp(T a) const { return a; }
};
template <> struct FnSum<bf16_t> {
  using EltType = bf16_t;
  static constexpr bool kPreOp = false, kPostOp = false;
  __device__ FnSum(uint64_t = 0) {}
  __device__ __forceinline__ bf16_t reduce(bf16_t a, bf16_t b) const {
    return {f32_to_bf16(bf16_to_f32(a.bits) + bf16_to_f32(b.bits))};
  }
  __device__ __forceinline__ bf16_t preOp(bf16_t a) const { return a; }
  __device__ __forceinline__ bf16_t postOp(bf16_t a) const { return a; }
};

// ---------------------------------------------------------------- Prod
// reduce_kernel.h:187-192, :273-275 (f16 __hmul), :294-296 (bf16)
template <typename T> struct FnProd {
  using EltType = T;
  static constexpr bool kPreOp = false, kPostOp = false;
  __device__ FnProd(uint64_t = 0) {}
  __device__ __forceinline__ T reduce(T a, T b) const { return a * b; }
  __device__ __forceinline__ T preOp(T a) const { return a; }
  __device__ __forceinline__ T postOp(T a) const { return a; }
};
template <> struct FnProd<uint8_t> {  // per-byte product mod 256 (:237-250)
  using EltType = uint8_t;
  static constexpr bool kPreOp = false, kPostOp = false;
  __device__ FnProd(uint64_t = 0) {}
  __device__ __forceinline__ uint8_t reduce(uint8_t a, uint8_t b) const {
    return (uint8_t)((uint32_t)a * (uint32_t)b);
  }
  __device__ __forceinline__ uint8_t preOp(uint8_t a) const { return a; }
  __device__ __forceinline__ uint8_t postOp(uint8_t a) const { return a; }
};
template <> struct FnProd<bf16_t> {
  using EltType = bf16_t;
  static constexpr bool kPreOp = false, kPostOp = false;
  __device__ FnProd(uint64_t = 0) {}
  __device__ __forceinline__ bf16_t reduce(bf16_t a, bf16_t b) const {
    return {f32_to_bf16(bf16_to_f32(a.bits) * bf16_to_f32(b.bits))};
  }
  __device__ __forceinline__ bf16_t preOp(bf16_t a) const { return a; }
  __device__ __forceinline__ bf16_t postOp(bf16_t a) const { return a; }
};

// ---------------------------------------------------------------- MinMax
// reduce_kernel.h:47-56 (ctor: xormask, isMinNotMax = (opArg&1)==0), :193-198
template <typename T> struct FnMinMax {  // unsigned integer kernels
  using EltType = T;
  static constexpr bool kPreOp = false, kPostOp = false;
  T xormask;
  __device__ FnMinMax(uint64_t arg = 0) : xormask((T)arg) {}
  __device__ __forceinline__ T reduce(T a, T b) const {
    return (T)(a ^ xormask) < (T)(b ^ xormask) ? a : b;
  }
  __device__ __forceinline__ T preOp(T a) const { return a; }
  __device__ __forceinline__ T postOp(T a) const { return a; }
};
template <> struct FnMinMax<float> {
  using EltType = float;
  static constexpr bool kPreOp = false, kPostOp = false;
  bool isMin;
  __device__ FnMinMax(uint64_t arg = 0) : isMin((arg & 1) == 0) {}
  __device__ __forceinline__ float reduce(float a, float b) const { return minmax_f32(a, b, isMin); }
  __device__ __forceinline__ float preOp(float a) const { return a; }
  __device__ __forceinline__ float postOp(float a) const { return a; }
};
template <> struct FnMinMax<double> {
  using EltType = double;
  static constexpr bool kPreOp = false, kPostOp = false;
  bool isMin;
  __device__ FnMinMax(uint64_t arg = 0) : isMin((arg & 1) == 0) {}
  __device__ __forceinline__ double reduce(double a, double b) const {
    return isMin ? __builtin_fmin(a, b) : __builtin_fmax(a, b);
  }
  __device__ __forceinline__ double preOp(double a) const { return a; }
  __device__ __forceinline__ double postOp(double a) const { return a; }
};
template <> struct FnMinMax<_Float16> {
  using EltType = _Float16;
  static constexpr bool kPreOp = false, kPostOp = false;
  bool isMin;
  __device__ FnMinMax(uint64_t arg = 0) : isMin((arg & 1) == 0) {}
  __device__ __forceinline__ _Float16 reduce(_Float16 a, _Float16 b) const {
    return (_Float16)minmax_f32((float)a, (float)b, isMin);  // exact both ways
  }
  __device__ __forceinline__ _Float16 preOp(_Float16 a) const { return a; }
  __device__ __forceinline__ _Float16 postOp(_Float16 a) const { return a; }
};
template <> struct FnMinMax<bf16_t> {
  using EltType = bf16_t;
  static constexpr bool kPreOp = false, kPostOp = false;
  bool isMin;
  __device__ FnMinMax(uint64_t arg = 0) : isMin((arg & 1) == 0) {}
  __device__ __forceinline__ bf16_t reduce(bf16_t a, bf16_t b) const {
    return {f32_to_bf16(minmax_f32(bf16_to_f32(a.bits), bf16_to_f32(b.bits), isMin))};
  }
  __device__ __forceinline__ bf16_t preOp(bf16_t a) const { return a; }
  __device__ __forceinline__ bf16_t postOp(bf16_t a) const { return a; }
};

// ---------------------------------------------------------------- PreMulSum
// reduce_kernel.h:424-583: reduce = Sum, preOp = x * scalar (in T).
template <typename T> struct FnPreMulSum {
  using EltType = T;
  static constexpr bool kPreOp = true, kPostOp = false;
  T scalar;
  __device__ FnPreMulSum(uint64_t arg = 0) : scalar(from_arg<T>(arg)) {}
  __device__ __forceinline__ T reduce(T a, T b) const { return a + b; }
  __device__ __forceinline__ T preOp(T a) const { return a * scalar; }
  __device__ __forceinline__ T postOp(T a) const { return a; }
};
template <> struct FnPreMulSum<uint8_t> {
  using EltType = uint8_t;
  static constexpr bool kPreOp = true, kPostOp = false;
  uint8_t scalar;
  __device__ FnPreMulSum(uint64_t arg = 0) : scalar((uint8_t)arg) {}
  __device__ __forceinline__ uint8_t reduce(uint8_t a, uint8_t b) const { return (uint8_t)(a + b); }
  __device__ __forceinline__ uint8_t preOp(uint8_t a) const { return (uint8_t)((uint32_t)a * scalar); }
  __device__ __forceinline__ uint8_t postOp(uint8_t a) const { return a; }
};
template <> struct FnPreMulSum<bf16_t> {
  using EltType = bf16_t;
  static constexpr bool kPreOp = true, kPostOp = false;
  float scalar;
  __device__ FnPreMulSum(uint64_t arg = 0) : scalar(bf16_to_f32((uint16_t)arg)) {}
  __device__ __forceinline__ bf16_t reduce(bf16_t a, bf16_t b) const {
    return {f32_to_bf16(bf16_to_f32(a.bits) + bf16_to_f32(b.bits))};
  }
  __device__ __forceinline__ bf16_t preOp(bf16_t a) const {
    return {f32_to_bf16(bf16_to_f32(a.bits) * scalar)};
  }
  __device__ __forceinline__ bf16_t postOp(bf16_t a) const { return a; }
};

// ---------------------------------------------------------------- fp8 ops
// reduce_kernel.h:309-321 (Sum / Prod / MinMax through __half) and :489-511,
// :586-624 (PreMulSum: the scalar arrives as fp8 bits, widened to half once;
// preOp = fp8(__hmul(half(x), scalar))).
#define VCCL_F8_FUNCTORS(F8)                                                              \
  template <> struct FnSum<F8> {                                                          \
    using EltType = F8;                                                                   \
    static constexpr bool kPreOp = false, kPostOp = false;                                \
    __device__ FnSum(uint64_t = 0) {}                                                     \
    __device__ __forceinline__ F8 reduce(F8 a, F8 b) const {                              \
      return f8_from_h(f8_to_h(a) + f8_to_h(b), F8{});                                    \
    }                                                                                     \
    __device__ __forceinline__ F8 preOp(F8 a) const { return a; }                         \
    __device__ __forceinline__ F8 postOp(F8 a) const { return a; }                        \
  };                                                                                      \
  template <> struct FnProd<F8> {                                                         \
    using EltType = F8;                                                                   \
    static constexpr bool kPreOp = false, kPostOp = false;                                \
    __device__ FnProd(uint64_t = 0) {}                                                    \
    __device__ __forceinline__ F8 reduce(F8 a, F8 b) const {                              \
      return f8_from_h(f8_to_h(a) * f8_to_h(b), F8{});                                    \
    }                                                                                     \
    __device__ __forceinline__ F8 preOp(F8 a) const { return a; }                         \
    __device__ __forceinline__ F8 postOp(F8 a) const { return a; }                        \
  };                                                                                      \
  template <> struct FnMinMax<F8> {                                                       \
    using EltType = F8;                                                                   \
    static constexpr bool kPreOp = false, kPostOp = false;                                \
    bool isMin;                                                                           \
    __device__ FnMinMax(uint64_t arg = 0) : isMin((arg & 1) == 0) {}                      \
    __device__ __forceinline__ F8 reduce(F8 a, F8 b) const {                              \
      return f8_from_h((_Float16)minmax_f32((float)f8_to_h(a), (float)f8_to_h(b), isMin), \
                       F8{});                                                             \
    }                                                                                     \
    __device__ __forceinline__ F8 preOp(F8 a) const { return a; }                         \
    __device__ __forceinline__ F8 postOp(F8 a) const { return a; }                        \
  };                                                                                      \
  template <> struct FnPreMulSum<F8> {                                                    \
    using EltType = F8;                                                                   \
    static constexpr bool kPreOp = true, kPostOp = false;                                 \
    _Float16 scalar;                                                                      \
    __device__ FnPreMulSum(uint64_t arg = 0) : scalar(f8_to_h(F8{(uint8_t)arg})) {}       \
    __device__ __forceinline__ F8 reduce(F8 a, F8 b) const {                              \
      return f8_from_h(f8_to_h(a) + f8_to_h(b), F8{});                                    \
    }                                                                                     \
    __device__ __forceinline__ F8 preOp(F8 a) const {                                     \
      return f8_from_h(f8_to_h(a) * scalar, F8{});                                        \
    }                                                                                     \
    __device__ __forceinline__ F8 postOp(F8 a) const { return a; }                        \
  };
VCCL_F8_FUNCTORS(f8e4m3_t)
VCCL_F8_FUNCTORS(f8e5m2_t)
#undef VCCL_F8_FUNCTORS

// ---------------------------------------------------------------- SumPostDiv
// reduce_kernel.h:641-688: integer avg = sum, then truncating divide at the
// final step through a 32/64-bit reciprocal and one fix-up.
template <typename T> struct FnSumPostDiv {
  using EltType = T;
  using U = typename std::conditional<sizeof(T) == 8, uint64_t, uint32_t>::type;
  static constexpr bool kPreOp = false, kPostOp = true;
  uint32_t divisor;
  bool isSigned;
  U recip;
  __device__ FnSumPostDiv(uint64_t arg = 0)
      : divisor((uint32_t)((arg >> 1) & 0x7fffffffu)), isSigned(arg & 1),
        recip(divisor ? U(-1) / divisor : 0) {}
  __device__ __forceinline__ T reduce(T a, T b) const { return (T)(a + b); }
  __device__ __forceinline__ T preOp(T a) const { return a; }
  __device__ __forceinline__ T postOp(T x) const {
    bool xneg = isSigned && (x & ~(T(-1) >> 1));
    U xabs = xneg ? (U)(T)(T(0) - x) : (U)x;
    U q;
    if constexpr (sizeof(T) == 8) q = __umul64hi(xabs, recip);
    else q = __umulhi(xabs, recip);
    if (xabs - q * divisor >= divisor) q += 1;
    return xneg ? (T)(T(0) - (T)q) : (T)q;
  }
};

// ---------------------------------------------------------------- Copy
// FuncCopy (reduce_kernel.h:41, :176-180): used by all-gather / one-rank copy.
template <typename T> struct FnCopy {
  using EltType = T;
  static constexpr bool kPreOp = false, kPostOp = false;
  __device__ FnCopy(uint64_t = 0) {}
  __device__ __forceinline__ T reduce(T a, T) const { return a; }
  __device__ __forceinline__ T preOp(T a) const { return a; }
  __device__ __forceinline__ T postOp(T a) const { return a; }
};

// ---------------------------------------------------------------- packs
// 16-byte pack = one global_load_dwordx4 per lane.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
union Pack16 {
  u32x4 v;
  T e[16 / sizeof(T)];
};

template <class Fn>
__device__ __forceinline__ u32x4 pack_reduce(const Fn& fn, u32x4 a, u32x4 b) {
  using T = typename Fn::EltType;
  Pack16<T> x, y;
  x.v = a;
  y.v = b;
#pragma unroll
  for (int i = 0; i < (int)(16 / sizeof(T)); i++) x.e[i] = fn.reduce(x.e[i], y.e[i]);
  return x.v;
}
// u8 sum on whole 32-bit words (SWAR): add the low 7 bits of every byte, then
// restore each byte's top bit by XOR — per-byte wrap-around, no cross-byte
// carry (reduce_kernel.h:200-211 computes the same per-byte sum).
__device__ __forceinline__ uint32_t swar_add_u8(uint32_t a, uint32_t b) {
  return ((a & 0x7f7f7f7fu) + (b & 0x7f7f7f7fu)) ^ ((a ^ b) & 0x80808080u);
}
__device__ __forceinline__ u32x4 pack_reduce(const FnSum<uint8_t>&, u32x4 a, u32x4 b) {
  return u32x4{swar_add_u8(a.x, b.x), swar_add_u8(a.y, b.y), swar_add_u8(a.z, b.z),
               swar_add_u8(a.w, b.w)};
}
__device__ __forceinline__ u32x4 pack_reduce(const FnPreMulSum<uint8_t>&, u32x4 a, u32x4 b) {
  return pack_reduce(FnSum<uint8_t>(), a, b);
}
__device__ __forceinline__ u32x4 pack_reduce(const FnSumPostDiv<uint8_t>&, u32x4 a, u32x4 b) {
  return pack_reduce(FnSum<uint8_t>(), a, b);
}
// u8 product / min / max on 16-bit lanes: even and odd bytes are widened into
// the two halves of a word and run through v_pk_{mul_lo,min}_u16, two bytes
// per instruction (per-element semantics unchanged: product mod 256, and the
// xormask-transformed unsigned min of FnMinMax).
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t swar_mul_u8(uint32_t a, uint32_t b) {
  uint32_t lo = as_u32(as_u16x2(a & 0x00ff00ffu) * as_u16x2(b & 0x00ff00ffu)) & 0x00ff00ffu;
  uint32_t hi = as_u32(as_u16x2((a >> 8) & 0x00ff00ffu) * as_u16x2((b >> 8) & 0x00ff00ffu));
  return lo | ((hi & 0x00ff00ffu) << 8);
}
__device__ __forceinline__ uint32_t swar_min_u8(uint32_t a, uint32_t b) {
  uint32_t lo = as_u32(__builtin_elementwise_min(as_u16x2(a & 0x00ff00ffu), as_u16x2(b & 0x00ff00ffu)));
  uint32_t hi = as_u32(__builtin_elementwise_min(as_u16x2(a & 0xff00ff00u), as_u16x2(b & 0xff00ff00u)));
  return lo | hi;
}
__device__ __forceinline__ u32x4 pack_reduce(const FnProd<uint8_t>&, u32x4 a, u32x4 b) {
  return u32x4{swar_mul_u8(a.x, b.x), swar_mul_u8(a.y, b.y), swar_mul_u8(a.z, b.z),
               swar_mul_u8(a.w, b.w)};
}
__device__ __forceinline__ u32x4 pack_reduce(const FnMinMax<uint8_t>& fn, u32x4 a, u32x4 b) {
  uint32_t m = 0x01010101u * fn.xormask;
  u32x4 r;
  r.x = swar_min_u8(a.x ^ m, b.x ^ m) ^ m;
  r.y = swar_min_u8(a.y ^ m, b.y ^ m) ^ m;
  r.z = swar_min_u8(a.z ^ m, b.z ^ m) ^ m;
  r.w = swar_min_u8(a.w ^ m, b.w ^ m) ^ m;
  return r;
}

// fp8 sum on packed half pairs.  Each 32-bit word's even and odd bytes are
// widened into two 16-bit lanes and added with v_pk_add_f16 (RN-even, the
// __hadd2 of reduce_kernel.h:310/317).
//  E5M2: byte << 8 IS the binary16 value.
//  E4M3: magnitude << 7 (+ sign << 8) is the binary16 value times 2^-8, for
//        subnormals too; the scaled sum is exact where the unscaled half sum
//        would be (results < 2^-6 are multiples of 2^-9 with <= 3 significant
//        bits; above, both live in half's normal range), and the scaled half's
//        exponent field equals E4M3's, so narrowing is RN-even on the low 7 bits
//        for every result.  NaN codes (S.1111.111) are forced to 0x7f.
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
template <bool E4M3>
__device__ __forceinline__ uint32_t f8x2_widen(uint32_t lanes) {  // two bytes in 16-bit lanes
  if constexpr (E4M3) return ((lanes & 0x007f007fu) << 7) | ((lanes & 0x00800080u) << 8);
  return lanes << 8;
}
template <bool E4M3>
__device__ __forceinline__ uint32_t f8x2_narrow(uint32_t h) {  // two halves -> two codes in lanes
  const u16x2 mag = as_u16x2(h & 0x7fff7fffu);
  const uint32_t sign = (h >> 8) & 0x00800080u;
  if constexpr (E4M3) {
    u16x2 r = (mag + (u16x2)0x3f + ((mag >> 7) & (u16x2)1)) >> 7;
    r = __builtin_elementwise_min(r, (u16x2)0x7e);
    return as_u32(r) | sign;
  } else {
    u16x2 r = (mag + (u16x2)0x7f + ((mag >> 8) & (u16x2)1)) >> 8;
    r = __builtin_elementwise_min(r, (u16x2)0x7b);  // infinity and NaN -> 0x7b
    // bit 15 of mag + 0x3ff is set iff mag > 0x7c00 (NaN): no compare, no VCC
    const uint32_t nanb = as_u32(mag + (u16x2)0x3ffu) & 0x80008000u;
    return as_u32(r) | (nanb >> 13) | (sign & ~(nanb >> 8));  // NaN: 0x7b | 0x04 = 0x7f, no sign
  }
}
template <bool E4M3>
__device__ __forceinline__ uint32_t f8x4_add(uint32_t a, uint32_t b) {
  const uint32_t alo = f8x2_widen<E4M3>(a & 0x00ff00ffu), ahi = f8x2_widen<E4M3>((a >> 8) & 0x00ff00ffu);
  const uint32_t blo = f8x2_widen<E4M3>(b & 0x00ff00ffu), bhi = f8x2_widen<E4M3>((b >> 8) & 0x00ff00ffu);
  const f16x2 slo = __builtin_bit_cast(f16x2, alo) + __builtin_bit_cast(f16x2, blo);
  const f16x2 shi = __builtin_bit_cast(f16x2, ahi) + __builtin_bit_cast(f16x2, bhi);
  uint32_t r = f8x2_narrow<E4M3>(__builtin_bit_cast(uint32_t, slo)) |
               (f8x2_narrow<E4M3>(__builtin_bit_cast(uint32_t, shi)) << 8);
  if constexpr (E4M3) {  // byte-wise NaN mask: (code & 0x7f) == 0x7f in either input
    const uint32_t na = ((a & 0x7f7f7f7fu) + 0x01010101u) & 0x80808080u;
    const uint32_t nb = ((b & 0x7f7f7f7fu) + 0x01010101u) & 0x80808080u;
    const uint32_t n = na | nb, n7f = n - (n >> 7);  // 0x7f in every NaN byte
    r = (r & ~(n | n7f)) | n7f;
  }
  return r;
}
template <bool E4M3>
__device__ __forceinline__ u32x4 f8_pack_add(u32x4 a, u32x4 b) {
  return u32x4{f8x4_add<E4M3>(a.x, b.x), f8x4_add<E4M3>(a.y, b.y), f8x4_add<E4M3>(a.z, b.z),
               f8x4_add<E4M3>(a.w, b.w)};
}
// E4M3 sum on gfx950's fp8 conversion units: v_cvt_pk_f32_fp8 widens two
// codes exactly, v_pk_add_f32 adds exactly (4-bit significands, exponents
// 2^-9 .. 2^8), v_med3_f32 clamps to +-448 (satfinite) and v_cvt_pk_fp8_f32
// narrows RN-even.  One rounding of the exact sum equals the reference's
// fp8(RN_half(a + b)): a sum needing more than half's 11 bits has operands
// >= 8 binades apart, so the smaller one moves the result less than 2^-7 of
// the larger — never to or across an E4M3 rounding midpoint (checked
// exhaustively: all 65,536 code pairs, test_fp8_all_code_pairs).  NaN codes
// are patched with the byte-wise mask (med3 does not keep NaN).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t e4m3x4_add_cvt(uint32_t a, uint32_t b) {
  const f32x2 lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)a, false) + __builtin_amdgcn_cvt_pk_f32_fp8((int)b, false);
  const f32x2 hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)a, true) + __builtin_amdgcn_cvt_pk_f32_fp8((int)b, true);
  const float m = 448.0f;
  int r = __builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(lo.x, -m, m),
                                         __builtin_amdgcn_fmed3f(lo.y, -m, m), 0, false);
  r = __builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(hi.x, -m, m),
                                     __builtin_amdgcn_fmed3f(hi.y, -m, m), r, true);
  const uint32_t na = ((a & 0x7f7f7f7fu) + 0x01010101u) & 0x80808080u;
  const uint32_t nb = ((b & 0x7f7f7f7fu) + 0x01010101u) & 0x80808080u;
  const uint32_t n = na | nb, n7f = n - (n >> 7);
  return ((uint32_t)r & ~(n | n7f)) | n7f;
}
__device__ __forceinline__ u32x4 e4m3_pack_add(u32x4 a, u32x4 b) {
  return u32x4{e4m3x4_add_cvt(a.x, b.x), e4m3x4_add_cvt(a.y, b.y), e4m3x4_add_cvt(a.z, b.z),
               e4m3x4_add_cvt(a.w, b.w)};
}
__device__ __forceinline__ u32x4 pack_reduce(const FnSum<f8e4m3_t>&, u32x4 a, u32x4 b) {
#ifdef VCCL_F8_HALF_PAIRS
  return f8_pack_add<true>(a, b);
#else
  return e4m3_pack_add(a, b);
#endif
}
__device__ __forceinline__ u32x4 pack_reduce(const FnPreMulSum<f8e4m3_t>&, u32x4 a, u32x4 b) {
  return pack_reduce(FnSum<f8e4m3_t>(), a, b);
}
// E5M2 the same way (v_cvt_pk_f32_bf8 / v_cvt_pk_bf8_f32; 3-bit significands,
// so the f32 sum is exact and the single-rounding argument holds with margin),
// but narrowed WITHOUT a clamp: the converter rounds RN-even and returns the
// infinity code 0x7c for anything past max finite and a NaN code (magnitude
// > 0x7c) for NaN (probed on the box: tools/probe_fp8_cvt.hip,
// profiles/r01y/probe.log), so satfinite and the canonical NaN are byte-wise
// fix-ups on the result alone: 0x7c -> 0x7b (sign kept), NaN -> 0x7f.
__device__ __forceinline__ uint32_t e5m2x4_add_cvt(uint32_t a, uint32_t b) {
  const f32x2 lo = __builtin_amdgcn_cvt_pk_f32_bf8((int)a, false) + __builtin_amdgcn_cvt_pk_f32_bf8((int)b, false);
  const f32x2 hi = __builtin_amdgcn_cvt_pk_f32_bf8((int)a, true) + __builtin_amdgcn_cvt_pk_f32_bf8((int)b, true);
  int ri = __builtin_amdgcn_cvt_pk_bf8_f32(lo.x, lo.y, 0, false);
  ri = __builtin_amdgcn_cvt_pk_bf8_f32(hi.x, hi.y, ri, true);
  uint32_t r = (uint32_t)ri;
  const uint32_t mag = r & 0x7f7f7f7fu;
  const uint32_t inf = ~((mag ^ 0x7c7c7c7cu) + 0x7f7f7f7fu) & 0x80808080u;  // exact byte == 0x7c
  const uint32_t n = (mag + 0x03030303u) & 0x80808080u, n7f = n - (n >> 7);  // byte > 0x7c
  r -= inf >> 7;  // 0x7c -> 0x7b in those bytes (no borrow: the byte is >= 0x7c)
  return (r & ~(n | n7f)) | n7f;
}
// The default E5M2 sum (-DVCCL_F8_E5M2_ELEMENTWISE restores the per-element
// widen-by-shift / _Float16 / integer-narrowing form).  Every 1-byte kernel is
// power-bound, not VALU-bound, at config 2: on zero inputs E4M3, E5M2 and u8
// all run at 7.85-7.92 TB/s (0.98-0.99 of peak), on random bytes at 7.0-7.2
// (tools/rc_data.py, profiles/r02q).  This form issues 2.5x fewer VALU
// instructions per launch (25.8 M vs 65.4 M, E4M3 26.9 M; SQ_ACTIVE_INST_VALU
// 28.0 M vs 65.5 M quad-cycles, profiles/r02p/pmc_dtypes.log), so it draws
// less power: +5 % on a box where the per-element form ran at 0.80 of peak
// (profiles/r02p/ab_fp8.log, interleaved), -2 % on one where it ran at 0.89.
#ifndef VCCL_F8_E5M2_ELEMENTWISE
__device__ __forceinline__ u32x4 pack_reduce(const FnSum<f8e5m2_t>&, u32x4 a, u32x4 b) {
  return u32x4{e5m2x4_add_cvt(a.x, b.x), e5m2x4_add_cvt(a.y, b.y), e5m2x4_add_cvt(a.z, b.z),
               e5m2x4_add_cvt(a.w, b.w)};
}
__device__ __forceinline__ u32x4 pack_reduce(const FnPreMulSum<f8e5m2_t>&, u32x4 a, u32x4 b) {
  return pack_reduce(FnSum<f8e5m2_t>(), a, b);
}
#endif
// (f8_pack_add<false>, the E5M2 form, measured 6.2 TB/s and is unused.  An
// E4M3-shaped E5M2 sum — med3 clamp to +-57344 before narrowing, NaN patched
// from the input codes — was exact on all 65,536 pairs and 7-8 % slower,
// 6.52 vs 7.07 TB/s: ~10 more VALU per dword, profiles/r06e.)

template <class Fn>
__device__ __forceinline__ u32x4 pack_preop(const Fn& fn, u32x4 a) {
  using T = typename Fn::EltType;
  Pack16<T> x;
  x.v = a;
#pragma unroll
  for (int i = 0; i < (int)(16 / sizeof(T)); i++) x.e[i] = fn.preOp(x.e[i]);
  return x.v;
}
__device__ __forceinline__ u32x4 pack_preop(const FnPreMulSum<uint8_t>& fn, u32x4 a) {
  uint32_t s = 0x01010101u * fn.scalar;
  return u32x4{swar_mul_u8(a.x, s), swar_mul_u8(a.y, s), swar_mul_u8(a.z, s), swar_mul_u8(a.w, s)};
}
template <class Fn>
__device__ __forceinline__ u32x4 pack_postop(const Fn& fn, u32x4 a) {
  using T = typename Fn::EltType;
  Pack16<T> x;
  x.v = a;
#pragma unroll
  for (int i = 0; i < (int)(16 / sizeof(T)); i++) x.e[i] = fn.postOp(x.e[i]);
  return x.v;
}

}  // namespace vccl
