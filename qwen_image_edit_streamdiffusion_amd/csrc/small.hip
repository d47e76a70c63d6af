// Small / bandwidth-bound kernels of the denoise loop:
//   timestep sinusoid, SiLU, true-CFG combine + norm rescale,
//   FlowMatch Euler step with per-row dt, strided batch copy,
//   latent pack/unpack, and the skinny GEMV used for the AdaLN
//   modulation linears (img_mod/txt_mod 3072->18432 on SiLU(temb)),
//   which is weight-bandwidth bound (13.6 GB of weights per forward).
#include "qie_common.h"

namespace {

__global__ void timestep_kernel(const bf16_t* __restrict__ t, bf16_t* __restrict__ out, int B,
                                int dim) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * dim) return;
  const int b = i / dim, j = i % dim, half = dim / 2;
  const int k = j < half ? j : j - half;
  // exponent = -ln(10000) * k / half ; emb = exp(exponent) ; arg = 1000 * (t * emb)
  const float e = expf((-9.210340371976184f * (float)k) / (float)half);
  const float arg = 1000.0f * (bf2f(t[b]) * e);
  out[i] = f2bf(j < half ? cosf(arg) : sinf(arg));
}

__global__ void silu_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = f2bf(silu_f(bf2f(x[i])));
}

// one wave per token row, C channels (C <= 256)
__global__ void __launch_bounds__(256)
    cfg_kernel(const bf16_t* __restrict__ cond, int64_t cbs, const bf16_t* __restrict__ unc, int64_t ubs,
               bf16_t* __restrict__ out, int64_t obs, int rows, int C, float s) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  cond += blockIdx.y * cbs;
  unc += blockIdx.y * ubs;
  out += blockIdx.y * obs;
  const int lane = threadIdx.x & 63;
  float cb[4], comb[4];
  float cn = 0.f, nn = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ch = lane + 64 * i;
    cb[i] = comb[i] = 0.f;
    if (ch < C) {
      const float c = bf2f(cond[(int64_t)row * C + ch]);
      const float u = bf2f(unc[(int64_t)row * C + ch]);
      cb[i] = c;
      comb[i] = rbf(u + rbf(s * rbf(c - u)));
      cn = __builtin_fmaf(c, c, cn);
      nn = __builtin_fmaf(comb[i], comb[i], nn);
    }
  }
  cn = rbf(sqrtf(wave_sum(cn)));
  nn = rbf(sqrtf(wave_sum(nn)));
  const float ratio = rbf(cn / nn);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ch = lane + 64 * i;
    if (ch < C) out[(int64_t)row * C + ch] = f2bf(comb[i] * ratio);
  }
}

// out = bf16(x + bf16(dt[b] * v)); 8 elements per thread when aligned
__global__ void euler_kernel(const bf16_t* __restrict__ x, int64_t xs, const bf16_t* __restrict__ v,
                             int64_t vs, bf16_t* out, int64_t os, int64_t n, QieBatchF dt) {
  const int b = blockIdx.y;
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n) return;
  const float d = dt.v[b];
  const bf16_t* xr = x + b * xs + i;
  const bf16_t* vr = v + b * vs + i;
  bf16_t* orow = out + b * os + i;
  for (int j = 0; j < 8 && i + j < n; ++j) orow[j] = f2bf(bf2f(xr[j]) + rbf(d * bf2f(vr[j])));
}

__global__ void copy_kernel(const bf16_t* __restrict__ src, int64_t ss, bf16_t* dst, int64_t ds,
                            int64_t n) {
  const int b = blockIdx.y;
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n) return;
  const bf16_t* s = src + b * ss + i;
  bf16_t* d = dst + b * ds + i;
  if (i + 8 <= n && (((uintptr_t)s | (uintptr_t)d) & 15) == 0) {
    *(u32x4_t*)d = *(const u32x4_t*)s;
  } else {
    for (int j = 0; j < 8 && i + j < n; ++j) d[j] = s[j];
  }
}

// y[b][(i*(W/2)+j)][c*4 + di*2 + dj] = x[b][c][2i+di][2j+dj]
template <bool PACK>
__global__ void pack_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int B, int C, int H,
                            int W) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)B * C * H * W;
  if (idx >= total) return;
  const int w = idx % W;
  const int hh = (idx / W) % H;
  const int c = (idx / ((int64_t)W * H)) % C;
  const int b = idx / ((int64_t)W * H * C);
  const int64_t tok = (int64_t)(hh >> 1) * (W >> 1) + (w >> 1);
  const int64_t packed = ((int64_t)b * (H / 2) * (W / 2) + tok) * (4 * C) + c * 4 + (hh & 1) * 2 + (w & 1);
  if (PACK) y[packed] = x[idx];
  else y[idx] = x[packed];
}

// Skinny GEMV: y[m][n] = bf16(sum_k x[m][k] w[n][k] + bias[n]) for m < M <= MM.
// One wave computes 4 output columns; lanes stride K in 16-byte chunks. HBM-bound on W (the
// modulation matrices are 113 MB each): every lane issues all U x 4 of a K-slab's W loads before
// the first FMA, so a wave keeps U x 4 x 1 KB in flight instead of one row's 1 KB at a time
// (U = 1 measured best: 22.5 us vs 24.1 us for the one-load-per-row form, HBM-cold 113 MB; U = 3 and 6
// lose occupancy: 27 / 26 us).
#ifndef QIE_GEMV_U
#define QIE_GEMV_U 1
#endif
#ifndef QIE_GEMV_NT
#define QIE_GEMV_NT 1
#endif
template <int MM, int U = QIE_GEMV_U>
__global__ void __launch_bounds__(256)
    gemv_kernel(const bf16_t* __restrict__ x, int64_t ldx, const bf16_t* __restrict__ w,
                const bf16_t* __restrict__ bias, bf16_t* __restrict__ y, int64_t ldy, int M, int N,
                int K) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n0 = (blockIdx.x * 4 + wave) * 4;
  if (n0 >= N) return;
  const int nch = K >> 3;
  float acc[MM][4];
#pragma unroll
  for (int m = 0; m < MM; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[m][j] = 0.f;
  const bf16_t* wrow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) wrow[j] = w + (int64_t)min(n0 + j, N - 1) * K;
  for (int c0 = lane; c0 < nch; c0 += 64 * U) {
    u32x4_t ww[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = min(c0 + u * 64, nch - 1);  // clamped reload of a valid chunk; its FMAs are skipped
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const u32x4_t* p = (const u32x4_t*)(wrow[j] + c * 8);
        ww[u][j] = QIE_GEMV_NT ? __builtin_nontemporal_load(p) : *p;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + u * 64;
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        if (m < M && c < nch) {
          const u32x4_t xx = *(const u32x4_t*)(x + (int64_t)m * ldx + c * 8);
          const float xf[8] = {lo_f(xx.x), hi_f(xx.x), lo_f(xx.y), hi_f(xx.y),
                               lo_f(xx.z), hi_f(xx.z), lo_f(xx.w), hi_f(xx.w)};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const u32x4_t& q = ww[u][j];
            const float wf[8] = {lo_f(q.x), hi_f(q.x), lo_f(q.y), hi_f(q.y),
                                 lo_f(q.z), hi_f(q.z), lo_f(q.w), hi_f(q.w)};
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[m][j] = __builtin_fmaf(xf[e], wf[e], acc[m][j]);
          }
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MM; ++m) {
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[m][j] = wave_sum(acc[m][j]);
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (n0 + j < N) y[(int64_t)m * ldy + n0 + j] = f2bf(acc[m][j] + bf2f(bias[n0 + j]));
    }
  }
}

}  // namespace

extern "C" int qie_abi_version(void) { return QIE_ABI_VERSION; }

extern "C" const char* qie_strerror(int code) {
  switch (code) {
    case QIE_OK: return "ok";
    case QIE_ERR_INVALID: return "invalid argument (shape/stride/alignment/null)";
    case QIE_ERR_UNSUPPORTED: return "unsupported size";
    default: return hipGetErrorString((hipError_t)code);
  }
}

extern "C" int qie_timestep_embed_bf16(const void* t, void* out, int batch, int dim,
                                       qie_stream_t stream) {
  QIE_CHECK_ARG(t && out && batch > 0 && dim > 0 && dim % 2 == 0);
  const int n = batch * dim;
  timestep_kernel<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>((const bf16_t*)t, (bf16_t*)out,
                                                                    batch, dim);
  return qie_last_error();
}

extern "C" int qie_silu_bf16(const void* x, void* y, int64_t n, qie_stream_t stream) {
  QIE_CHECK_ARG(x && y && n > 0);
  silu_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>((const bf16_t*)x,
                                                                            (bf16_t*)y, n);
  return qie_last_error();
}

extern "C" int qie_cfg_combine_bf16(const void* cond, int64_t cond_bstride, const void* uncond,
                                    int64_t uncond_bstride, void* out, int64_t out_bstride, int batch,
                                    int rows, int C, float scale, qie_stream_t stream) {
  QIE_CHECK_ARG(cond && uncond && out && rows > 0 && C > 0 && C <= 256);
  QIE_CHECK_ARG(batch > 0 && batch < 65536);
  dim3 grid((rows + 3) / 4, batch);
  cfg_kernel<<<grid, 256, 0, (hipStream_t)stream>>>((const bf16_t*)cond, cond_bstride,
                                                    (const bf16_t*)uncond, uncond_bstride,
                                                    (bf16_t*)out, out_bstride, rows, C, scale);
  return qie_last_error();
}

extern "C" int qie_euler_step_bf16(const void* x, int64_t x_bstride, const void* v,
                                   int64_t v_bstride, void* out, int64_t out_bstride, int batch,
                                   int64_t n, const float* dt_host, qie_stream_t stream) {
  QIE_CHECK_ARG(x && v && out && dt_host && batch > 0 && batch <= QIE_MAX_BATCH && n > 0);
  QieBatchF dt{};
  for (int i = 0; i < batch; ++i) dt.v[i] = dt_host[i];
  const int64_t threads = (n + 7) / 8;
  dim3 grid((unsigned)((threads + 255) / 256), batch);
  euler_kernel<<<grid, 256, 0, (hipStream_t)stream>>>((const bf16_t*)x, x_bstride, (const bf16_t*)v,
                                                      v_bstride, (bf16_t*)out, out_bstride, n, dt);
  return qie_last_error();
}

extern "C" int qie_copy_bf16(const void* src, int64_t src_bstride, void* dst, int64_t dst_bstride,
                             int batch, int64_t n, qie_stream_t stream) {
  QIE_CHECK_ARG(src && dst && batch > 0 && n > 0 && batch < 65536);
  const int64_t threads = (n + 7) / 8;
  dim3 grid((unsigned)((threads + 255) / 256), batch);
  copy_kernel<<<grid, 256, 0, (hipStream_t)stream>>>((const bf16_t*)src, src_bstride, (bf16_t*)dst,
                                                     dst_bstride, n);
  return qie_last_error();
}

extern "C" int qie_pack_latents_bf16(const void* x, void* y, int batch, int C, int H, int W,
                                     qie_stream_t stream) {
  QIE_CHECK_ARG(x && y && batch > 0 && C > 0 && H % 2 == 0 && W % 2 == 0 && H > 0 && W > 0);
  const int64_t total = (int64_t)batch * C * H * W;
  pack_kernel<true><<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      (const bf16_t*)x, (bf16_t*)y, batch, C, H, W);
  return qie_last_error();
}

extern "C" int qie_unpack_latents_bf16(const void* x, void* y, int batch, int C, int H, int W,
                                       qie_stream_t stream) {
  QIE_CHECK_ARG(x && y && batch > 0 && C > 0 && H % 2 == 0 && W % 2 == 0 && H > 0 && W > 0);
  const int64_t total = (int64_t)batch * C * H * W;
  pack_kernel<false><<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      (const bf16_t*)x, (bf16_t*)y, batch, C, H, W);
  return qie_last_error();
}

extern "C" int qie_gemv_bf16(const void* x, int64_t ldx, const void* w, const void* bias, void* y,
                             int64_t ldy, int M, int N, int K, qie_stream_t stream) {
  QIE_CHECK_ARG(x && w && bias && y && M > 0 && M <= 16 && N > 0 && K % 8 == 0 && ldx % 8 == 0);
  QIE_CHECK_ARG(((uintptr_t)x % 16) == 0 && ((uintptr_t)w % 16) == 0);
  hipStream_t s = (hipStream_t)stream;
  const int grid = (N + 15) / 16;
  const bf16_t *xb = (const bf16_t*)x, *wb = (const bf16_t*)w, *bb = (const bf16_t*)bias;
  bf16_t* yb = (bf16_t*)y;
  if (M <= 1) gemv_kernel<1><<<grid, 256, 0, s>>>(xb, ldx, wb, bb, yb, ldy, M, N, K);
  else if (M <= 2) gemv_kernel<2><<<grid, 256, 0, s>>>(xb, ldx, wb, bb, yb, ldy, M, N, K);
  else if (M <= 4) gemv_kernel<4><<<grid, 256, 0, s>>>(xb, ldx, wb, bb, yb, ldy, M, N, K);
  else if (M <= 8) gemv_kernel<8><<<grid, 256, 0, s>>>(xb, ldx, wb, bb, yb, ldy, M, N, K);
  else gemv_kernel<16><<<grid, 256, 0, s>>>(xb, ldx, wb, bb, yb, ldy, M, N, K);
  return qie_last_error();
}
