// Row-wise normalisation kernels (HBM-bound; one wave per row, 16-byte lanes).
//
//  * LayerNorm(no affine) + AdaLN _modulate of QwenImageTransformerBlock [U],
//    optionally emitting int8 + per-row scale for the Int8Linear path (the
//    quantisation prologue fused into the norm);
//  * RMSNorm with weight (txt_norm);
//  * per-head RMSNorm(128) of q/k + complex RoPE, in place on the
//    head-major joint QKV buffer;
//  * per-row int8 quantisation of GEMM inputs that are not produced by a norm
//    (attention output, GELU output).
// Every elementwise op mirrors the bf16 rounding points of the reference model
// (oracle/dit_ref.py); statistics are fp32.
#include "qie_common.h"

namespace {

constexpr int kMaxC = 8;  // 16-byte chunks per lane: D <= 64*8*8 = 4096

__device__ __forceinline__ void unpack8(const u32x4_t w, float f[8]) {
  f[0] = lo_f(w.x); f[1] = hi_f(w.x); f[2] = lo_f(w.y); f[3] = hi_f(w.y);
  f[4] = lo_f(w.z); f[5] = hi_f(w.z); f[6] = lo_f(w.w); f[7] = hi_f(w.w);
}
__device__ __forceinline__ u32x4_t pack8(const float f[8]) {
  return u32x4_t{pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7])};
}

// symmetric int8 of 8 values with a precomputed inverse scale; returns 8 bytes
__device__ __forceinline__ u32x2_t quant8(const float f[8], float inv) {
  unsigned w[2] = {0, 0};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float q = rintf(f[j] * inv);
    q = fminf(fmaxf(q, -127.f), 127.f);
    w[j >> 2] |= ((unsigned)((int)q & 0xff)) << (8 * (j & 3));
  }
  return u32x2_t{w[0], w[1]};
}

#ifndef QIE_LNMOD_YR  // y never aliases x / shift / scale: lets hipcc hoist chunk i+1's scale / shift
#define QIE_LNMOD_YR __restrict__  // loads above chunk i's store (one round trip per row, not six)
#endif
#ifndef QIE_LNMOD_PREFETCH
#define QIE_LNMOD_PREFETCH 0  // measured slower: 42.0 vs 39.3 us (register pressure), kept as a build option
#endif
#ifndef QIE_LNMOD_EXACT  // 1: chunk count per lane as a template argument where D = 512 * NC (no guards,
#define QIE_LNMOD_EXACT 1  // x kept packed: 102 -> fewer VGPRs, more waves in flight); 0: generic only
#endif
// NC: 16-byte chunks per lane (EXACT: every lane has exactly NC, D = 512 * NC); the bf16 path keeps
// x packed (4 VGPRs per chunk) and unpacks it for each pass; the int8 path also keeps the modulated
// values for the quantisation pass. Same arithmetic and order in every instantiation.
template <bool I8, int NC, bool EXACT>
__global__ void __launch_bounds__(256)
    ln_mod_kernel(const bf16_t* __restrict__ x, int64_t ldx, const bf16_t* __restrict__ shift,
                  const bf16_t* __restrict__ scale, int64_t mod_bstride, int rpb, void* QIE_LNMOD_YR y, int64_t ldy,
                  float* qscale, int rows, int D, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const int nch = D >> 3;
  const bf16_t* xr = x + (int64_t)row * ldx;
  u32x4_t raw[EXACT ? NC : 1];   // EXACT: x packed, unpacked again by each pass
  float xf[EXACT ? 1 : NC][8];   // generic: x unpacked once (fewer VGPRs for the guarded form)
  auto get = [&](int i, float f[8]) {
    if constexpr (EXACT) unpack8(raw[i], f);
    else
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = xf[i][j];
  };
  // int8: the modulated row for the quant pass -- packed (bf16-exact values) in the exact form,
  // as floats in the generic one (fewer VGPRs for each)
  u32x4_t vp[I8 && EXACT ? NC : 1];
  float vf[I8 && !EXACT ? NC : 1][8];
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = lane + 64 * i;
    if (EXACT || c < nch) {
      const u32x4_t w = *(const u32x4_t*)(xr + c * 8);
      float f[8];
      unpack8(w, f);
      if constexpr (EXACT) raw[i] = w;
      else
#pragma unroll
        for (int j = 0; j < 8; ++j) xf[i][j] = f[j];
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += f[j];
    }
  }
  const int b = row / rpb;
  const bf16_t* sh = shift + (int64_t)b * mod_bstride;
  const bf16_t* sc = scale + (int64_t)b * mod_bstride;
#if QIE_LNMOD_PREFETCH
  // scale / shift issued with x, under the two reductions: in the store loop below hipcc may not
  // move chunk i+1's loads above chunk i's store (y may alias them), one round trip per chunk
  u32x4_t scv[NC], shv[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = min(lane + 64 * i, nch - 1);
    scv[i] = *(const u32x4_t*)(sc + c * 8);
    shv[i] = *(const u32x4_t*)(sh + c * 8);
  }
#endif
  const float mean = wave_sum(sum) / (float)D;
  // the passes re-unpack x from the packed registers: without these fences hipcc keeps all 8 * NC
  // unpacked floats live across the reductions (CSE of the three unpacks)
  if constexpr (EXACT)
#pragma unroll
    for (int i = 0; i < NC; ++i) asm volatile("" : "+v"(raw[i]));
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i)
    if (EXACT || lane + 64 * i < nch) {
      float f[8];
      get(i, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = f[j] - mean;
        sq = __builtin_fmaf(d, d, sq);
      }
    }
  const float rstd = rsqrtf(wave_sum(sq) / (float)D + eps);
  if constexpr (EXACT)
#pragma unroll
    for (int i = 0; i < NC; ++i) asm volatile("" : "+v"(raw[i]));
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = lane + 64 * i;
    if (EXACT || c < nch) {
      float f[8], s8[8], h8[8];
      get(i, f);
#if QIE_LNMOD_PREFETCH
      unpack8(scv[i], s8);
      unpack8(shv[i], h8);
#else
      unpack8(*(const u32x4_t*)(sc + c * 8), s8);
      unpack8(*(const u32x4_t*)(sh + c * 8), h8);
#endif
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float n = rbf((f[j] - mean) * rstd);
        const float t = rbf(n * rbf(1.0f + s8[j]));
        f[j] = rbf(t + h8[j]);
        amax = fmaxf(amax, fabsf(f[j]));
      }
      if constexpr (I8 && EXACT) {
        vp[i] = pack8(f);  // exact: every f[j] is already a bf16 value
      } else if constexpr (I8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) vf[i][j] = f[j];
      } else {
        *(u32x4_t*)((bf16_t*)y + (int64_t)row * ldy + c * 8) = pack8(f);
      }
    }
  }
  if constexpr (I8) {
    amax = wave_max(amax);
    const float inv = amax > 0.f ? 127.0f / amax : 0.f;
    int8_t* qr = (int8_t*)y + (int64_t)row * ldy;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = lane + 64 * i;
      if (EXACT || c < nch) {
        if constexpr (EXACT) {
          float g[8];
          unpack8(vp[i], g);
          *(u32x2_t*)(qr + c * 8) = quant8(g, inv);
        } else {
          *(u32x2_t*)(qr + c * 8) = quant8(vf[i], inv);
        }
      }
    }
    if (lane == 0) qscale[row] = amax > 0.f ? amax / 127.0f : 1.0f;
  }
}

// one launch of ln_mod_kernel: the exact-chunk instantiation for D = 3072 / 3584 / 4096
template <bool I8>
void launch_ln_mod(const void* x, int64_t ldx, const void* shift, const void* scale, int64_t mod_bstride,
                   int rpb, void* y, int64_t ldy, float* qscale, int rows, int D, float eps, hipStream_t s) {
  const dim3 grid((rows + 3) / 4), block(256);
  const auto* xp = (const bf16_t*)x;
  const auto* shp = (const bf16_t*)shift;
  const auto* scp = (const bf16_t*)scale;
  if (QIE_LNMOD_EXACT && D == 512 * 6)
    ln_mod_kernel<I8, 6, true><<<grid, block, 0, s>>>(xp, ldx, shp, scp, mod_bstride, rpb, y, ldy, qscale, rows, D, eps);
  else if (QIE_LNMOD_EXACT && D == 512 * 7)
    ln_mod_kernel<I8, 7, true><<<grid, block, 0, s>>>(xp, ldx, shp, scp, mod_bstride, rpb, y, ldy, qscale, rows, D, eps);
  else if (QIE_LNMOD_EXACT && D == 512 * 8)
    ln_mod_kernel<I8, 8, true><<<grid, block, 0, s>>>(xp, ldx, shp, scp, mod_bstride, rpb, y, ldy, qscale, rows, D, eps);
  else
    ln_mod_kernel<I8, kMaxC, false><<<grid, block, 0, s>>>(xp, ldx, shp, scp, mod_bstride, rpb, y, ldy, qscale, rows, D,
                                                           eps);
}

__global__ void __launch_bounds__(256)
    rmsnorm_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                   int rows, int D, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const int nch = D >> 3;
  const bf16_t* xr = x + (int64_t)row * D;
  float v[kMaxC][8];
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      unpack8(*(const u32x4_t*)(xr + c * 8), v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) sq = __builtin_fmaf(v[i][j], v[i][j], sq);
    }
  }
  const float rstd = rsqrtf(wave_sum(sq) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < kMaxC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      float w8[8];
      unpack8(*(const u32x4_t*)(w + c * 8), w8);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = rbf(rbf(v[i][j] * rstd) * w8[j]);
      *(u32x4_t*)(y + (int64_t)row * D + c * 8) = pack8(v[i]);
    }
  }
}

// 16 lanes per 128-wide head row, 8 elements (4 complex pairs) per lane.
__global__ void __launch_bounds__(256)
    qk_norm_rope_kernel(bf16_t* __restrict__ qkv, int B, int H, int s_pad, int seg_start, int seg_len,
                        const bf16_t* __restrict__ wq, const bf16_t* __restrict__ wk,
                        const float* __restrict__ cos_tab, const float* __restrict__ sin_tab,
                        float eps, float q_scale) {
  const int64_t gr = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);  // global row id
  const int64_t total = (int64_t)2 * B * H * seg_len;
  if (gr >= total) return;
  const int l16 = threadIdx.x & 15;
  const int sl = (int)(gr % seg_len);
  const int64_t plane = gr / seg_len;  // (which*B + b)*H + h, which in {0,1}
  const int which = (int)(plane / ((int64_t)B * H));
  bf16_t* p = qkv + (plane * s_pad + seg_start + sl) * 128 + l16 * 8;
  float v[8];
  unpack8(*(const u32x4_t*)p, v);
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) sq = __builtin_fmaf(v[j], v[j], sq);
  sq = group_sum<16>(sq);
  const float rstd = rsqrtf(sq * (1.0f / 128.0f) + eps);
  float w8[8];
  unpack8(*(const u32x4_t*)((which == 0 ? wq : wk) + l16 * 8), w8);
  const f32x4_t cs = *(const f32x4_t*)(cos_tab + (int64_t)sl * 64 + l16 * 4);
  const f32x4_t sn = *(const f32x4_t*)(sin_tab + (int64_t)sl * 64 + l16 * 4);
  const float osc = which == 0 ? q_scale : 1.0f;  // folded in before the one rounding of the output
  float o[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float a = rbf(rbf(v[2 * j] * rstd) * w8[2 * j]);
    const float bb = rbf(rbf(v[2 * j + 1] * rstd) * w8[2 * j + 1]);
    o[2 * j] = __builtin_fmaf(a, cs[j], -(bb * sn[j])) * osc;
    o[2 * j + 1] = __builtin_fmaf(a, sn[j], bb * cs[j]) * osc;
  }
  *(u32x4_t*)p = pack8(o);
}

template <int MAXC>
__global__ void __launch_bounds__(256)
    quant_rows_kernel(const bf16_t* __restrict__ x, int64_t ldx, int8_t* __restrict__ q, int64_t ldq,
                      float* __restrict__ scale, int rows, int D) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const int nch = D >> 3;
  const bf16_t* xr = x + (int64_t)row * ldx;
  u32x4_t raw[MAXC];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      raw[i] = *(const u32x4_t*)(xr + c * 8);
      float f[8];
      unpack8(raw[i], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(f[j]));
    }
  }
  amax = wave_max(amax);
  const float inv = amax > 0.f ? 127.0f / amax : 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      float f[8];
      unpack8(raw[i], f);
      *(u32x2_t*)(q + (int64_t)row * ldq + c * 8) = quant8(f, inv);
    }
  }
  if (lane == 0) scale[row] = amax > 0.f ? amax / 127.0f : 1.0f;
}

// Two waves per row (D = 1024 * NCW, the int8 path's GELU output at D = 12288): each wave holds
// NCW chunks per lane (48 VGPRs of x at NCW = 12 instead of 96), the two wave maxima meet in LDS.
// amax is a max, so the result is bit-identical to quant_rows_kernel. Rows past `rows` still reach
// the barrier.
#ifndef QIE_QUANT_2W
#define QIE_QUANT_2W 1
#endif
template <int NCW>
__global__ void __launch_bounds__(256)
    quant_rows2_kernel(const bf16_t* __restrict__ x, int64_t ldx, int8_t* __restrict__ q, int64_t ldq,
                       float* __restrict__ scale, int rows) {
  __shared__ float wmax[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 2 + (wave >> 1), half = wave & 1;
  const bool valid = row < rows;
  const int c0 = half * 64 * NCW + lane;  // this lane's first chunk of the row
  const bf16_t* xr = x + (int64_t)(valid ? row : 0) * ldx;
  u32x4_t raw[NCW];
  float amax = 0.f;
  if (valid) {
#pragma unroll
    for (int i = 0; i < NCW; ++i) {
      raw[i] = *(const u32x4_t*)(xr + (c0 + 64 * i) * 8);
      float f[8];
      unpack8(raw[i], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(f[j]));
    }
  }
  amax = wave_max(amax);
  if (lane == 0) wmax[wave] = amax;
  __syncthreads();
  if (!valid) return;
  amax = fmaxf(wmax[wave & 2], wmax[(wave & 2) + 1]);
  const float inv = amax > 0.f ? 127.0f / amax : 0.f;
#pragma unroll
  for (int i = 0; i < NCW; ++i) {
    float f[8];
    unpack8(raw[i], f);
    *(u32x2_t*)(q + (int64_t)row * ldq + (c0 + 64 * i) * 8) = quant8(f, inv);
  }
  if (half == 0 && lane == 0) scale[row] = amax > 0.f ? amax / 127.0f : 1.0f;
}

}  // namespace

extern "C" int qie_layernorm_modulate_bf16(const void* x, int64_t ldx, const void* shift,
                                           const void* scale, int64_t mod_bstride,
                                           int rows_per_batch, void* y, int64_t ldy, int rows, int D,
                                           float eps, qie_stream_t stream) {
  QIE_CHECK_ARG(x && shift && scale && y && rows > 0 && rows_per_batch > 0);
  QIE_CHECK_ARG(D % 8 == 0 && D <= 64 * 8 * kMaxC && ldx % 8 == 0 && ldy % 8 == 0);
  QIE_CHECK_ARG(mod_bstride % 8 == 0);
  launch_ln_mod<false>(x, ldx, shift, scale, mod_bstride, rows_per_batch, y, ldy, nullptr, rows, D, eps,
                       (hipStream_t)stream);
  return qie_last_error();
}

extern "C" int qie_layernorm_modulate_i8(const void* x, int64_t ldx, const void* shift,
                                         const void* scale, int64_t mod_bstride,
                                         int rows_per_batch, void* q, int64_t ldq, float* qscale,
                                         int rows, int D, float eps, qie_stream_t stream) {
  QIE_CHECK_ARG(x && shift && scale && q && qscale && rows > 0 && rows_per_batch > 0);
  QIE_CHECK_ARG(D % 8 == 0 && D <= 64 * 8 * kMaxC && ldx % 8 == 0 && ldq % 8 == 0);
  QIE_CHECK_ARG(mod_bstride % 8 == 0);
  launch_ln_mod<true>(x, ldx, shift, scale, mod_bstride, rows_per_batch, q, ldq, qscale, rows, D, eps,
                      (hipStream_t)stream);
  return qie_last_error();
}

extern "C" int qie_rmsnorm_bf16(const void* x, const void* w, void* y, int rows, int D, float eps,
                                qie_stream_t stream) {
  QIE_CHECK_ARG(x && w && y && rows > 0 && D % 8 == 0 && D <= 64 * 8 * kMaxC);
  rmsnorm_kernel<<<(rows + 3) / 4, 256, 0, (hipStream_t)stream>>>(
      (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, rows, D, eps);
  return qie_last_error();
}

extern "C" int qie_qk_norm_rope_bf16(void* qkv, int batch, int heads, int head_dim, int s_pad,
                                     int seg_start, int seg_len, const void* wq, const void* wk,
                                     const float* cos_tab, const float* sin_tab, float eps,
                                     float q_scale, qie_stream_t stream) {
  QIE_CHECK_ARG(qkv && wq && wk && cos_tab && sin_tab && head_dim == 128);
  QIE_CHECK_ARG(batch > 0 && heads > 0 && seg_len >= 0 && seg_start >= 0 &&
                seg_start + seg_len <= s_pad);
  if (seg_len == 0) return QIE_OK;
  const int64_t rows = (int64_t)2 * batch * heads * seg_len;
  const int64_t blocks = (rows + 15) / 16;
  QIE_CHECK_ARG(blocks < (1ll << 31));
  qk_norm_rope_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(
      (bf16_t*)qkv, batch, heads, s_pad, seg_start, seg_len, (const bf16_t*)wq, (const bf16_t*)wk,
      cos_tab, sin_tab, eps, q_scale);
  return qie_last_error();
}

extern "C" int qie_quantize_rows_i8(const void* x, int64_t ldx, void* q, int64_t ldq, float* scale,
                                    int rows, int D, qie_stream_t stream) {
  QIE_CHECK_ARG(x && q && scale && rows > 0 && D % 8 == 0 && ldx % 8 == 0 && ldq % 8 == 0);
  hipStream_t s = (hipStream_t)stream;
  const int grid = (rows + 3) / 4;
  if (QIE_QUANT_2W && D == 1024 * 12)
    quant_rows2_kernel<12><<<(rows + 1) / 2, 256, 0, s>>>((const bf16_t*)x, ldx, (int8_t*)q, ldq, scale, rows);
  else if (D <= 64 * 8 * 8)
    quant_rows_kernel<8><<<grid, 256, 0, s>>>((const bf16_t*)x, ldx, (int8_t*)q, ldq, scale, rows, D);
  else if (D <= 64 * 8 * 24)
    quant_rows_kernel<24><<<grid, 256, 0, s>>>((const bf16_t*)x, ldx, (int8_t*)q, ldq, scale, rows, D);
  else
    return QIE_ERR_UNSUPPORTED;
  return qie_last_error();
}
