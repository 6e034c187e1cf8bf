// (devOp, ncclDataType_t) -> functor dispatch.
//
// Replaces the reference's generated function table (generate.py:141-167 ->
// host_table.cc / device_table.cu, 670 primary functions) with one C++ switch.
// Kernel element types follow generate.py:129-137 (equivalent_primary):
// signed integers run the unsigned kernel for every op; SumPostDiv exists only
// for integers (generate.py:107).  fp8 (generate.py:109-111, sm90+ in the
// reference) runs natively on gfx950's OCP E4M3 / E5M2 through half (ops.hpp).
#pragma once
#include "ops.hpp"

namespace vccl {

// ncclDataType_t values (nccl.h.in:239-252)
enum : int { T_I8 = 0, T_U8, T_I32, T_U32, T_I64, T_U64, T_F16, T_F32, T_F64, T_BF16, T_F8E4M3, T_F8E5M2 };
// ncclDevRedOp_t values (src/include/device.h:34-38)
enum : int { OP_SUM = 0, OP_PROD, OP_MINMAX, OP_PREMULSUM, OP_SUMPOSTDIV, OP_COPY = 15 };
// kernel element types
enum : int { K_U8 = 0, K_U32, K_U64, K_F16, K_F32, K_F64, K_BF16, K_F8E4M3, K_F8E5M2 };

__host__ __device__ inline int kernel_type_of(int devOp, int type) {
  int k;
  switch (type) {
    case T_I8: case T_U8: k = K_U8; break;
    case T_I32: case T_U32: k = K_U32; break;
    case T_I64: case T_U64: k = K_U64; break;
    case T_F16: k = K_F16; break;
    case T_F32: k = K_F32; break;
    case T_F64: k = K_F64; break;
    case T_BF16: k = K_BF16; break;
    case T_F8E4M3: k = K_F8E4M3; break;
    case T_F8E5M2: k = K_F8E5M2; break;
    default: return -1;
  }
  if (devOp == OP_SUMPOSTDIV && k >= K_F16) return -1;
  if (devOp == OP_COPY && k != K_U8) return -1;  // copies are byte copies (enqueue.cc:2400-2404)
  if (devOp < OP_SUM || (devOp > OP_SUMPOSTDIV && devOp != OP_COPY)) return -1;
  return k;
}

template <int K> struct KTypeOf;
template <> struct KTypeOf<K_U8> { using T = uint8_t; };
template <> struct KTypeOf<K_U32> { using T = uint32_t; };
template <> struct KTypeOf<K_U64> { using T = uint64_t; };
template <> struct KTypeOf<K_F16> { using T = _Float16; };
template <> struct KTypeOf<K_F32> { using T = float; };
template <> struct KTypeOf<K_F64> { using T = double; };
template <> struct KTypeOf<K_BF16> { using T = bf16_t; };
template <> struct KTypeOf<K_F8E4M3> { using T = f8e4m3_t; };
template <> struct KTypeOf<K_F8E5M2> { using T = f8e5m2_t; };

// Calls f.template operator()<Fn>() for the functor of devOp on element type T.
template <class T, class F>
inline bool dispatch_op(int devOp, F&& f) {
  switch (devOp) {
    case OP_SUM: f.template operator()<FnSum<T>>(); return true;
    case OP_PROD: f.template operator()<FnProd<T>>(); return true;
    case OP_MINMAX: f.template operator()<FnMinMax<T>>(); return true;
    case OP_PREMULSUM: f.template operator()<FnPreMulSum<T>>(); return true;
    case OP_COPY:
      if constexpr (sizeof(T) == 1) { f.template operator()<FnCopy<T>>(); return true; }
      return false;
    case OP_SUMPOSTDIV:
      if constexpr (!IsFloat<T>::value) { f.template operator()<FnSumPostDiv<T>>(); return true; }
      return false;
  }
  return false;
}

// Launch geometry shared by the launchers.
struct LaunchGeom {
  int block, unroll, grid, ntLoads, ntStores, order;
};

}  // namespace vccl
