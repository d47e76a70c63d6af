// VAE decoder (AutoencoderKLQwenImage on one frame) -- the memory-bound pieces
// around the implicit-GEMM convolutions of gemm.hip (qie_conv2d_bf16). Activations are NHWC bf16
// ([pixels][channels], channels contiguous), so every per-pixel channel reduction is one
// contiguous row and every convolution is a GEMM over K = (tap, channel).
//
// Rounding points follow the bf16 module graph of diffusers' QwenImage VAE [U] (restated in
// oracle/vae_ref.py): F.normalize (bf16 norm, bf16 quotient), * sqrt(C), * gamma, SiLU, each
// rounded to bf16; the latent de-normalisation `latents / (1/std) + mean` in bf16.
#include <type_traits>

#include "qie_common.h"

namespace {

// ---- latents in: packed [B][(h/2)(w/2)][64] -> NHWC [B][h][w][16] (pipeline _unpack_latents),
// z = bf16(bf16(l / sinv) + mean) per channel, then post_quant_conv (1x1x1, 16 -> 16, bias):
// y[o] = bf16(sum_c W[o][c] z[c] + b[o]) in fp32. One thread per latent pixel.
__global__ void __launch_bounds__(256)
    latents_in_kernel(const bf16_t* __restrict__ packed, int B, int h, int w, const bf16_t* __restrict__ sinv,
                      const bf16_t* __restrict__ mean, const bf16_t* __restrict__ W, const bf16_t* __restrict__ b,
                      bf16_t* __restrict__ y) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= (int64_t)B * h * w) return;
  const int bi = (int)(p / ((int64_t)h * w));
  const int rem = (int)(p - (int64_t)bi * h * w);
  const int yy = rem / w, xx = rem - yy * w;
  const int i = yy >> 1, dy = yy & 1, j = xx >> 1, dx = xx & 1;
  const bf16_t* src = packed + (((int64_t)bi * (h / 2) + i) * (w / 2) + j) * 64 + dy * 2 + dx;
  float z[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) z[c] = rbf(rbf(bf2f(src[c * 4]) / bf2f(sinv[c])) + bf2f(mean[c]));
  u32x4_t o[2];
  uint32_t* ow = (uint32_t*)o;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float a[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int oc = 2 * q + t;
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) acc = __builtin_fmaf(bf2f(W[oc * 16 + c]), z[c], acc);
      a[t] = acc + bf2f(b[oc]);
    }
    ow[q] = pack2(a[0], a[1]);
  }
  u32x4_t* dst = (u32x4_t*)(y + p * 16);
  dst[0] = o[0];
  dst[1] = o[1];
}

// ---- QwenImageRMS_norm (+ SiLU): per pixel, y = bf16(bf16(bf16(x / bf16(max(|x|_2, 1e-12))) *
// sqrt(C)) * gamma), then optionally bf16(silu(y)). G lanes per pixel (8 channels, one 16-byte
// load each; C <= 8 G), 64 / G pixels per wave: every lane of the wave moves bytes.
template <bool SILU, int G>
__global__ void __launch_bounds__(256)
    rms_norm_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ gamma, bf16_t* __restrict__ y,
                    int64_t P, int C, float scale) {
  const int64_t p = ((int64_t)blockIdx.x * 256 + threadIdx.x) / G;
  const int gl = threadIdx.x & (G - 1);
  const bool act = p < P && gl * 8 < C;
  const bf16_t* xr = x + p * C;
  u32x4_t raw = {0, 0, 0, 0};
  if (act) raw = *(const u32x4_t*)(xr + gl * 8);
  const uint32_t w4[4] = {raw.x, raw.y, raw.z, raw.w};
  float v[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = lo_f(w4[k]);
    v[2 * k + 1] = hi_f(w4[k]);
  }
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) ss = __builtin_fmaf(v[k], v[k], ss);
  ss = group_sum<G>(ss);
  const float d = fmaxf(rbf(sqrtf(ss)), 1e-12f);
  if (!act) return;
  u32x4_t graw = *(const u32x4_t*)(gamma + gl * 8);
  const uint32_t g4[4] = {graw.x, graw.y, graw.z, graw.w};
  uint32_t o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float r[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const float g = t ? hi_f(g4[k]) : lo_f(g4[k]);
      float u = rbf(rbf(rbf(v[2 * k + t] / d) * scale) * g);
      if (SILU) u = u * __builtin_amdgcn_rcpf(1.0f + __expf(-u));
      r[t] = u;
    }
    o[k] = pack2(r[0], r[1]);
  }
  *(u32x4_t*)(y + p * C + gl * 8) = u32x4_t{o[0], o[1], o[2], o[3]};
}

// ---- softmax over rows of fp32 scores: P = bf16(exp(scale (s - max)) / sum) for columns < N,
// zeros in [N, ldp) (the K padding of the P.V GEMM). One workgroup per row, N % 4 == 0: pass 1
// keeps a per-thread online (max, sum) over its float4s, merged across the workgroup; pass 2
// re-reads the row (L2-resident, <= 64 KiB) and writes P.
__device__ __forceinline__ void ml_merge(float& m, float& l, float m2, float l2) {
  const float mn = fmaxf(m, m2);
  l = (m == -INFINITY ? 0.f : l * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : l2 * __expf(m2 - mn));
  m = mn;
}

__global__ void __launch_bounds__(256)
    softmax_rows_kernel(const float* __restrict__ s, int64_t lds, bf16_t* __restrict__ p, int64_t ldp, int Nall,
                        float scale, int causal, const int* __restrict__ ranges, int period) {
  const int64_t row = blockIdx.x;
  const int rr = (int)(row % period);  // row within its head (head-batched score blocks)
  // Keys [c0, c1) of row r: all Nall; causal (the text encoder's decoder mask) 0..r; ranges (the
  // vision tower's window / per-image blocks) ranges[2r] .. ranges[2r+1]. Other columns are 0.
  int c0 = 0, c1 = Nall;
  if (causal) c1 = min(Nall, rr + 1);
  if (ranges) {
    c0 = max(ranges[2 * rr], 0);
    c1 = min(ranges[2 * rr + 1], Nall);
  }
  const float* sr = s + row * lds;
  __shared__ float red_m[4], red_l[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float m = -INFINITY, l = 0.f;  // in scaled units
  for (int c = (c0 & ~3) + tid * 4; c < c1; c += 1024) {
    f32x4_t t = *(const f32x4_t*)(sr + c);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c + k < c0 || c + k >= c1) t[k] = -INFINITY;  // the chunks straddling the range ends
    const float tm = fmaxf(fmaxf(t[0], t[1]), fmaxf(t[2], t[3])) * scale;
    float tl = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) tl += __expf(__builtin_fmaf(t[k], scale, -tm));
    ml_merge(m, l, tm, tl);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ml_merge(m, l, __shfl_xor(m, o, 64), __shfl_xor(l, o, 64));
  if (lane == 0) {
    red_m[wave] = m;
    red_l[wave] = l;
  }
  __syncthreads();
  m = red_m[0];
  l = red_l[0];
  for (int w = 1; w < 4; ++w) ml_merge(m, l, red_m[w], red_l[w]);
  const float inv = 1.0f / l;
  bf16_t* pr = p + row * ldp;
  for (int c = tid * 4; c < ldp; c += 1024) {
    float e[4] = {0.f, 0.f, 0.f, 0.f};
    if (c + 3 >= c0 && c < c1) {
      const f32x4_t t = *(const f32x4_t*)(sr + c);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (c + k >= c0 && c + k < c1) e[k] = __expf(t[k] * scale - m) * inv;
    }
    *(u32x2_t*)(pr + c) = u32x2_t{pack2(e[0], e[1]), pack2(e[2], e[3])};
  }
}

// ---- bf16 transpose: y[c][r] = x[r][c] for a [R][C] block with row stride ldx; 64x64 LDS tiles
__global__ void __launch_bounds__(256)
    transpose_kernel(const bf16_t* __restrict__ x, int64_t ldx, bf16_t* __restrict__ y, int64_t ldy, int R, int C) {
  __shared__ bf16_t t[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, c = c0 + tx;
    t[i][tx] = (r < R && c < C) ? x[(int64_t)r * ldx + c] : (bf16_t)0;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, r = r0 + tx;
    if (c < C && r < R) y[(int64_t)c * ldy + r] = t[tx][i];
  }
}

// ---- image out: conv_out result [P][ldx] bf16 (channels 0..2) -> decode's clamp(-1, 1), then
// the image processor's (x / 2 + 0.5).clamp(0, 1) on bf16 and (v * 255).round() -> uint8 RGB.
__global__ void __launch_bounds__(256)
    rgb_out_kernel(const bf16_t* __restrict__ x, int64_t ldx, uint8_t* __restrict__ rgb, int64_t P) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = fminf(fmaxf(bf2f(x[p * ldx + c]), -1.0f), 1.0f);
    const float u = fminf(fmaxf(rbf(v * 0.5f + 0.5f), 0.0f), 1.0f);
    rgb[p * 3 + c] = (uint8_t)rintf(u * 255.0f);
  }
}

// ---- image in (encoder): uint8 RGB [P][3] -> the image processor's bf16(2 (v / 255) - 1), NHWC
// with the channels padded to 8 (zeros) for the conv gather's 16-byte chunks.
__global__ void __launch_bounds__(256)
    rgb_in_kernel(const uint8_t* __restrict__ rgb, bf16_t* __restrict__ y, int64_t P) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  float v[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) v[c] = 2.0f * ((float)rgb[p * 3 + c] / 255.0f) - 1.0f;
  *(u32x4_t*)(y + p * 8) = u32x4_t{pack2(v[0], v[1]), pack2(v[2], 0.f), 0u, 0u};
}

// ---- latents out (encoder): quant_conv output NHWC [B][h][w][ldx] -> mode (channels 0..15 = mu)
// -> bf16(bf16(mu - mean) / std) -> packed [B][(h/2)(w/2)][64] (pipeline _encode_vae_image,
// _pack_latents). One thread per packed element.
__global__ void __launch_bounds__(256)
    latents_out_kernel(const bf16_t* __restrict__ x, int64_t ldx, int B, int h, int w, const bf16_t* __restrict__ mean,
                       const bf16_t* __restrict__ stdv, bf16_t* __restrict__ packed) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)B * h * w * 16;
  if (q >= total) return;
  const int ch = (int)(q & 63);
  const int64_t tok = q >> 6;
  const int c = ch >> 2, dy = (ch >> 1) & 1, dx = ch & 1;
  const int bi = (int)(tok / ((h / 2) * (w / 2)));
  const int r = (int)(tok - (int64_t)bi * (h / 2) * (w / 2));
  const int i = r / (w / 2), j = r - i * (w / 2);
  const int64_t pix = ((int64_t)bi * h + 2 * i + dy) * w + 2 * j + dx;
  const float mu = bf2f(x[pix * ldx + c]);
  packed[q] = f2bf(rbf(mu - bf2f(mean[c])) / bf2f(stdv[c]));
}

}  // namespace

extern "C" int qie_vae_latents_in_bf16(const void* packed, int batch, int h, int w, const void* sinv,
                                       const void* mean, const void* pq_w, const void* pq_b, void* y,
                                       qie_stream_t stream) {
  QIE_CHECK_ARG(packed && sinv && mean && pq_w && pq_b && y && batch > 0 && h > 0 && w > 0);
  QIE_CHECK_ARG(h % 2 == 0 && w % 2 == 0 && ((uintptr_t)y % 16) == 0);
  const int64_t P = (int64_t)batch * h * w;
  latents_in_kernel<<<(unsigned)((P + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      (const bf16_t*)packed, batch, h, w, (const bf16_t*)sinv, (const bf16_t*)mean, (const bf16_t*)pq_w,
      (const bf16_t*)pq_b, (bf16_t*)y);
  return qie_last_error();
}

extern "C" int qie_vae_rms_norm_bf16(const void* x, const void* gamma, void* y, int64_t pixels, int C,
                                     int silu, qie_stream_t stream) {
  QIE_CHECK_ARG(x && gamma && y && pixels > 0 && C > 0 && C % 8 == 0 && C <= 512);
  QIE_CHECK_ARG(((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0 && ((uintptr_t)gamma % 16) == 0);
  const float scale = sqrtf((float)C);
  const hipStream_t st = (hipStream_t)stream;
  const bf16_t *xb = (const bf16_t*)x, *gb = (const bf16_t*)gamma;
  bf16_t* yb = (bf16_t*)y;
  auto launch = [&](auto g_t) {
    constexpr int G = decltype(g_t)::value;
    const unsigned grid = (unsigned)((pixels * G + 255) / 256);
    if (silu) rms_norm_kernel<true, G><<<grid, 256, 0, st>>>(xb, gb, yb, pixels, C, scale);
    else rms_norm_kernel<false, G><<<grid, 256, 0, st>>>(xb, gb, yb, pixels, C, scale);
  };
  if (C <= 128) launch(std::integral_constant<int, 16>{});
  else if (C <= 256) launch(std::integral_constant<int, 32>{});
  else launch(std::integral_constant<int, 64>{});
  return qie_last_error();
}

extern "C" int qie_softmax_rows_f32_bf16(const float* s, int64_t lds, void* p, int64_t ldp, int rows, int N,
                                         float scale, int causal, qie_stream_t stream) {
  QIE_CHECK_ARG(s && p && rows > 0 && N > 0 && N % 4 == 0 && lds >= N && lds % 4 == 0);
  QIE_CHECK_ARG(ldp >= N && ldp % 4 == 0 && ((uintptr_t)s % 16) == 0 && ((uintptr_t)p % 8) == 0);
  softmax_rows_kernel<<<rows, 256, 0, (hipStream_t)stream>>>(s, lds, (bf16_t*)p, ldp, N, scale, causal, nullptr,
                                                              rows);
  return qie_last_error();
}

extern "C" int qie_softmax_rows_ranged_f32_bf16(const float* s, int64_t lds, void* p, int64_t ldp, int rows, int N,
                                                float scale, const int* ranges_dev, int period, qie_stream_t stream) {
  QIE_CHECK_ARG(s && p && ranges_dev && rows > 0 && N > 0 && N % 4 == 0 && lds >= N && lds % 4 == 0);
  QIE_CHECK_ARG(period > 0 && rows % period == 0);
  QIE_CHECK_ARG(ldp >= N && ldp % 4 == 0 && ((uintptr_t)s % 16) == 0 && ((uintptr_t)p % 8) == 0);
  softmax_rows_kernel<<<rows, 256, 0, (hipStream_t)stream>>>(s, lds, (bf16_t*)p, ldp, N, scale, 0, ranges_dev,
                                                              period);
  return qie_last_error();
}

extern "C" int qie_transpose_bf16(const void* x, int64_t ldx, void* y, int64_t ldy, int R, int C,
                                  qie_stream_t stream) {
  QIE_CHECK_ARG(x && y && R > 0 && C > 0 && ldx >= C && ldy >= R);
  const dim3 grid((C + 63) / 64, (R + 63) / 64);
  transpose_kernel<<<grid, 256, 0, (hipStream_t)stream>>>((const bf16_t*)x, ldx, (bf16_t*)y, ldy, R, C);
  return qie_last_error();
}

extern "C" int qie_vae_rgb_out(const void* x, int64_t ldx, void* rgb, int64_t pixels, qie_stream_t stream) {
  QIE_CHECK_ARG(x && rgb && pixels > 0 && ldx >= 3);
  rgb_out_kernel<<<(unsigned)((pixels + 255) / 256), 256, 0, (hipStream_t)stream>>>((const bf16_t*)x, ldx,
                                                                                     (uint8_t*)rgb, pixels);
  return qie_last_error();
}

extern "C" int qie_vae_rgb_in(const void* rgb, void* y, int64_t pixels, qie_stream_t stream) {
  QIE_CHECK_ARG(rgb && y && pixels > 0 && ((uintptr_t)y % 16) == 0);
  rgb_in_kernel<<<(unsigned)((pixels + 255) / 256), 256, 0, (hipStream_t)stream>>>((const uint8_t*)rgb, (bf16_t*)y,
                                                                                    pixels);
  return qie_last_error();
}

extern "C" int qie_vae_latents_out_bf16(const void* x, int64_t ldx, int batch, int h, int w, const void* mean,
                                        const void* stdv, void* packed, qie_stream_t stream) {
  QIE_CHECK_ARG(x && mean && stdv && packed && batch > 0 && h > 0 && w > 0 && h % 2 == 0 && w % 2 == 0);
  QIE_CHECK_ARG(ldx >= 16);
  const int64_t total = (int64_t)batch * h * w * 16;
  latents_out_kernel<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      (const bf16_t*)x, ldx, batch, h, w, (const bf16_t*)mean, (const bf16_t*)stdv, (bf16_t*)packed);
  return qie_last_error();
}
