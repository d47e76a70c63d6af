// Shared device helpers for the Qwen-Image-Edit MI355X (gfx950) kernels.
// bf16 is carried as raw 16-bit words (unsigned short) in memory; MFMA
// operands use the __bf16 ext-vector types the gfx950 builtins expect.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/qie.h"

typedef unsigned short bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;   // 16x16x32 / 32x32x16 operand
typedef __attribute__((ext_vector_type(4))) short s16x4_t;     // ds_read_tr16_b64 result
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) int i32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;

#define QIE_LDS __attribute__((address_space(3)))
#define QIE_GLOBAL __attribute__((address_space(1)))

// ---------------------------------------------------------------- bf16 <-> f32
__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((unsigned)h) << 16); }

// Round-to-nearest-even, NaN-preserving: a plain cast lowers to v_cvt_pk_bf16_f32
// on gfx950 (MI355X_MICROARCH.md, correctness boundaries).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
// round an fp32 value to the nearest bf16 and return it as fp32
__device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }

// two floats -> two RNE bf16 in one word: ONE v_cvt_pk_bf16_f32 with both operands (the scalar
// casts cost two conversions, a shift and an or)
typedef __attribute__((ext_vector_type(2))) float qie_f2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 qie_b2_t;
__device__ __forceinline__ unsigned pack2(float lo, float hi) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((qie_f2_t){lo, hi}, qie_b2_t));
}
// round two floats to bf16 and back (the pair form of rbf)
__device__ __forceinline__ void rbf2(float& a, float& b) {
  const unsigned p = pack2(a, b);
  a = __uint_as_float(p << 16);
  b = __uint_as_float(p & 0xffff0000u);
}
__device__ __forceinline__ float lo_f(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_f(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

// ---------------------------------------------------------------- reductions (wave64)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// reduce within aligned groups of G lanes (G power of two <= 64)
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float gelu_tanh_f(float x) {
  // torch gelu(approximate="tanh"): 0.5*x*(1+tanh(u)), u = sqrt(2/pi)*(x+0.044715*x^3).
  // Identity 0.5*(1+tanh(u)) = 1/(1+exp(-2u)): one v_exp_f32 + one v_rcp_f32
  // (relative error ~1e-7, far below the bf16 rounding of the result).
  // t = 2u log2(e) = x (c1 + c2 x^2): three VALU (mul, fma, mul) before the exp
  const float c1 = 2.0f * 0.7978845608028654f * 1.4426950408889634f;
  const float c2 = c1 * 0.044715f;
  const float t = x * __builtin_fmaf(c2, x * x, c1);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-t));
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }

// ---------------------------------------------------------------- launch helpers
#define QIE_CHECK_ARG(cond)            \
  do {                                 \
    if (!(cond)) return QIE_ERR_INVALID; \
  } while (0)

static inline int qie_last_error() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QIE_OK : (int)e;
}

// small by-value arrays for per-batch scalars (stream batch <= 16 rows)
struct QieBatchF {
  float v[QIE_MAX_BATCH];
};
struct QieBatchI {
  int v[QIE_MAX_BATCH];
};
