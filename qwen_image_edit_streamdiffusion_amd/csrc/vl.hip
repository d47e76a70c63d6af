// Qwen2.5-VL prompt-encoder pieces: row gather (token embedding, window
// permutation), rotate-half RoPE (3-D M-RoPE tables / 2-D vision tables), SwiGLU gating, erf GELU. The projections, RMSNorms and the
// attention products run on the GEMM / norm kernels of gemm.hip / norm.hip / vae.hip.
//
// Rounding points follow transformers' Qwen2_5_VLTextModel in bf16 [U: transformers 5.15
// models/qwen2_5_vl/modeling_qwen2_5_vl.py]: apply_multimodal_rotary_pos_emb computes
// q * cos + rotate_half(q) * sin in the activation dtype with cos / sin cast to it (three bf16
// roundings); Qwen2MLP is act(gate(x)) * up(x), each a bf16 tensor.
#include "qie_common.h"

namespace {

// out[i][:] = table[ids[i]][:], D % 8 == 0 (16-byte chunks)
__global__ void __launch_bounds__(256)
    embed_rows_kernel(const bf16_t* __restrict__ table, const int* __restrict__ ids, int rows, int D, int vocab,
                      bf16_t* __restrict__ out) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int nch = D >> 3;
  if (q >= (int64_t)rows * nch) return;
  const int r = (int)(q / nch), c = (int)(q - (int64_t)r * nch);
  const int id = min(max(ids[r], 0), vocab - 1);
  *(u32x4_t*)(out + (int64_t)r * D + c * 8) = *(const u32x4_t*)(table + (int64_t)id * D + c * 8);
}

// In place on heads [h0, h0 + nh) of each row (rotary width Dh, heads hs elements apart, row
// stride ld), with per-row tables cos / sin [rows][Dh] (the M-RoPE sections already merged):
//   bf16 tables (the language model): three bf16 roundings, as in the activation dtype
//     x[d]        <- bf16(bf16(x[d] cos[d])        + bf16(-x[d + Dh/2] sin[d]))
//     x[d + Dh/2] <- bf16(bf16(x[d + Dh/2] cos[d + Dh/2]) + bf16(x[d] sin[d + Dh/2]))
//   fp32 tables (the vision tower, apply_rotary_pos_emb_vision upcasts): fp32 products and sum,
//   one bf16 rounding (unfused, as torch evaluates q * cos + rotate_half(q) * sin).
template <bool F32TAB>
__global__ void __launch_bounds__(256)
    rope_half_kernel(bf16_t* __restrict__ x, int64_t ld, int rows, int h0, int nh, int Dh, int hs,
                     const void* __restrict__ cs_, const void* __restrict__ sn_) {
  const int half = Dh >> 1;
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= (int64_t)rows * nh * half) return;
  const int d = (int)(q % half);
  const int64_t rh = q / half;
  const int h = (int)(rh % nh), r = (int)(rh / nh);
  bf16_t* p = x + (int64_t)r * ld + (int64_t)(h0 + h) * hs;
  const float a = bf2f(p[d]), b = bf2f(p[d + half]);
  float lo, hi;
  if constexpr (F32TAB) {
    const float* cr = (const float*)cs_ + (int64_t)r * Dh;
    const float* sr = (const float*)sn_ + (int64_t)r * Dh;
    lo = __fadd_rn(__fmul_rn(a, cr[d]), __fmul_rn(-b, sr[d]));
    hi = __fadd_rn(__fmul_rn(b, cr[d + half]), __fmul_rn(a, sr[d + half]));
  } else {
    const bf16_t* cr = (const bf16_t*)cs_ + (int64_t)r * Dh;
    const bf16_t* sr = (const bf16_t*)sn_ + (int64_t)r * Dh;
    lo = rbf(rbf(a * bf2f(cr[d])) + rbf(-b * bf2f(sr[d])));
    hi = rbf(rbf(b * bf2f(cr[d + half])) + rbf(a * bf2f(sr[d + half])));
  }
  p[d] = f2bf(lo);
  p[d + half] = f2bf(hi);
}

// y = bf16(gelu_erf(x)) elementwise over [rows][n] (nn.GELU() default, on a bf16 tensor)
__global__ void __launch_bounds__(256)
    gelu_erf_kernel(bf16_t* __restrict__ x, int64_t ld, int rows, int n) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int nch = n >> 3;
  if (q >= (int64_t)rows * nch) return;
  const int r = (int)(q / nch), c = (int)(q - (int64_t)r * nch);
  bf16_t* p = x + (int64_t)r * ld + c * 8;
  const u32x4_t w = *(const u32x4_t*)p;
  const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
  uint32_t o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float a = lo_f(ww[k]), b = hi_f(ww[k]);
    o[k] = pack2(0.5f * a * (1.0f + erff(a * 0.70710678118654752f)), 0.5f * b * (1.0f + erff(b * 0.70710678118654752f)));
  }
  *(u32x4_t*)p = u32x4_t{o[0], o[1], o[2], o[3]};
}

// y[r][f] = bf16(bf16(silu(g)) * u), g = gu[r][f], u = gu[r][F + f] (packed gate | up GEMM output)
__global__ void __launch_bounds__(256)
    silu_mul_kernel(const bf16_t* __restrict__ gu, int64_t ldg, int rows, int F, bf16_t* __restrict__ y,
                    int64_t ldy) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int nch = F >> 3;
  if (q >= (int64_t)rows * nch) return;
  const int r = (int)(q / nch), c = (int)(q - (int64_t)r * nch);
  const u32x4_t g = *(const u32x4_t*)(gu + (int64_t)r * ldg + c * 8);
  const u32x4_t u = *(const u32x4_t*)(gu + (int64_t)r * ldg + F + c * 8);
  const uint32_t gw[4] = {g.x, g.y, g.z, g.w}, uw[4] = {u.x, u.y, u.z, u.w};
  uint32_t o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float g0 = lo_f(gw[k]), g1 = hi_f(gw[k]);
    const float s0 = rbf(g0 / (1.0f + expf(-g0))), s1 = rbf(g1 / (1.0f + expf(-g1)));
    o[k] = pack2(s0 * lo_f(uw[k]), s1 * hi_f(uw[k]));
  }
  *(u32x4_t*)(y + (int64_t)r * ldy + c * 8) = u32x4_t{o[0], o[1], o[2], o[3]};
}

}  // namespace

extern "C" int qie_embed_rows_bf16(const void* table, const int* ids_dev, int rows, int D, int vocab, void* out,
                                   qie_stream_t stream) {
  QIE_CHECK_ARG(table && ids_dev && out && rows > 0 && D > 0 && D % 8 == 0 && vocab > 0);
  QIE_CHECK_ARG(((uintptr_t)table % 16) == 0 && ((uintptr_t)out % 16) == 0);
  const int64_t n = (int64_t)rows * (D / 8);
  embed_rows_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      (const bf16_t*)table, ids_dev, rows, D, vocab, (bf16_t*)out);
  return qie_last_error();
}

extern "C" int qie_rope_half_bf16(void* x, int64_t ld, int rows, int h0, int nh, int head_dim, int head_stride,
                                  const void* cos_tab, const void* sin_tab, int tab_f32, qie_stream_t stream) {
  QIE_CHECK_ARG(x && cos_tab && sin_tab && rows > 0 && h0 >= 0 && nh > 0 && head_dim > 0 && head_dim % 2 == 0);
  QIE_CHECK_ARG(head_stride >= head_dim && ld >= (int64_t)(h0 + nh - 1) * head_stride + head_dim);
  const int64_t n = (int64_t)rows * nh * (head_dim / 2);
  const unsigned g = (unsigned)((n + 255) / 256);
  if (tab_f32)
    rope_half_kernel<true><<<g, 256, 0, (hipStream_t)stream>>>((bf16_t*)x, ld, rows, h0, nh, head_dim, head_stride,
                                                               cos_tab, sin_tab);
  else
    rope_half_kernel<false><<<g, 256, 0, (hipStream_t)stream>>>((bf16_t*)x, ld, rows, h0, nh, head_dim, head_stride,
                                                                cos_tab, sin_tab);
  return qie_last_error();
}

extern "C" int qie_gelu_erf_bf16(void* x, int64_t ld, int rows, int n, qie_stream_t stream) {
  QIE_CHECK_ARG(x && rows > 0 && n > 0 && n % 8 == 0 && ld >= n && ld % 8 == 0 && ((uintptr_t)x % 16) == 0);
  const int64_t t = (int64_t)rows * (n / 8);
  gelu_erf_kernel<<<(unsigned)((t + 255) / 256), 256, 0, (hipStream_t)stream>>>((bf16_t*)x, ld, rows, n);
  return qie_last_error();
}

extern "C" int qie_silu_mul_bf16(const void* gu, int64_t ldg, int rows, int F, void* y, int64_t ldy,
                                 qie_stream_t stream) {
  QIE_CHECK_ARG(gu && y && rows > 0 && F > 0 && F % 8 == 0 && ldg >= 2 * (int64_t)F && ldy >= F);
  QIE_CHECK_ARG(ldg % 8 == 0 && ldy % 8 == 0 && ((uintptr_t)gu % 16) == 0 && ((uintptr_t)y % 16) == 0);
  const int64_t n = (int64_t)rows * (F / 8);
  silu_mul_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>((const bf16_t*)gu, ldg, rows, F,
                                                                                 (bf16_t*)y, ldy);
  return qie_last_error();
}
