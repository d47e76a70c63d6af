// Shared pieces of the MFMA GEMM family (gemm.hip: the DiT linears; conv.hip: the VAE
// convolutions): epilogue arguments and arithmetic, LDS tile staging and swizzle, the XCD-aware
// block remap, MFMA wrappers and the LDS-DMA piece. gfx950 only.
#pragma once
#include <algorithm>
#include <type_traits>

#include "qie_common.h"

namespace {

constexpr int kRowBytes = 128;  // one LDS tile row = 64 bf16 or 128 int8 of K

// EPI_QKV_NR: EPI_QKV + the per-head RMSNorm of q and k and their RoPE (gemm_pp only)
// EPI_RES: out = bf16(out + bf16(acc + bias)) (the VAE ResidualBlock's x + h; conv_kernel only)
// EPI_NORM: out = RMS_norm(bf16(acc + bias)) * gamma (+ SiLU) per pixel over all N channels (the VAE
// ResidualBlock's norm2 folded into conv1; conv_halo_kernel with one wave across N only)
enum Epi { EPI_BIAS = 0, EPI_GELU = 1, EPI_GATE_RES = 2, EPI_QKV = 3, EPI_PARTIAL = 4, EPI_QKV_NR = 5, EPI_RES = 6,
           EPI_NORM = 7 };

struct EpiArgs {
  void* out;          // y / resid / qkv base
  int64_t ldo;        // row stride (elements) of y / resid
  const bf16_t* bias;
  const bf16_t* gate;
  int64_t gate_bstride;
  int rows_per_batch;
  // qkv scatter
  int seq_offset, batch, heads, head_dim, s_pad;
  // int8 scales
  const float* sx;
  const float* sw;
  // split-K partial sums (EPI_PARTIAL): [splits][M][N] fp32 (bf16) or int32 (int8)
  void* ws;
  // EPI_QKV_NR: RMSNorm weights of q / k (head_dim), RoPE cos / sin [rows_per_batch][head_dim/2]
  const bf16_t* nq;
  const bf16_t* nk;
  const float* rcos;
  const float* rsin;
  float eps;
  float qscale;  // EPI_QKV_NR: factor on q (1, or scale*log2(e) for qie_attention_fwd_log2q_bf16)
  // head-batched products (gemm_kernel, blockIdx.z = batch entry): byte strides of x / w / out,
  // w advancing once per `group` entries (grouped-query attention shares k / v across a group)
  int64_t bsx_b, bsw_b, bso_b;
  int group;
  // EPI_NORM: per-channel gamma, sqrt(N), SiLU after the norm
  const bf16_t* ngamma;
  float nscale;
  int nsilu;
};

__device__ __forceinline__ int swz_chunk(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// Stage a [ROWS][128 B] tile: wave-instruction i of wave w fills 8 rows (1 KiB).
template <int ROWS, int NWAVE>
__device__ __forceinline__ void stage_tile(const char* __restrict__ g, int64_t ld_bytes, int rows_valid,
                                           char QIE_LDS* lds, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < ROWS / 8 / NWAVE; ++i) {
    const int blk = wave + i * NWAVE;
    const int r = blk * 8 + (lane >> 3);
    const int c = swz_chunk(r, lane & 7);
    const int gr = r < rows_valid ? r : rows_valid - 1;
    const char* src = g + (int64_t)gr * ld_bytes + (c << 4);
    __builtin_amdgcn_global_load_lds((const void*)src, (QIE_LDS void*)(lds + blk * 1024), 16, 0, 0);
  }
}

// bijective XCD remap (cdna_hip_programming.md §5, "XCD swizzle must be bijective")
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

template <bool I8>
struct MfmaOp;
template <>
struct MfmaOp<false> {
  typedef bf16x8_t frag;
  typedef f32x4_t acc;
  static __device__ __forceinline__ acc mma(frag a, frag b, acc c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ float tof(float v) { return v; }
};
template <>
struct MfmaOp<true> {
  typedef i32x4_t frag;
  typedef i32x4_t acc;
  static __device__ __forceinline__ acc mma(frag a, frag b, acc c) {
    return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  }
};

template <bool I8>
__device__ __forceinline__ float acc_val(const typename MfmaOp<I8>::acc& a, int r, float s) {
  if constexpr (I8) return (float)a[r] * s;
  else return a[r];
}

// Epilogue for 4 consecutive columns n..n+3 of row m.
template <int EPI, bool I8>
__device__ __forceinline__ void epilogue4(const EpiArgs& e, int m, int n, const float v_in[4]) {
  float v[4];
  const u32x2_t bw = *(const u32x2_t*)(e.bias + n);
  const float b4[4] = {lo_f(bw.x), hi_f(bw.x), lo_f(bw.y), hi_f(bw.y)};
  if constexpr (I8) {
    const float sx = e.sx[m];
    const f32x4_t sw = *(const f32x4_t*)(e.sw + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = rbf(__builtin_fmaf(v_in[j], sx * sw[j], b4[j]));
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = rbf(v_in[j] + b4[j]);
  }
  if constexpr (EPI == EPI_BIAS || EPI == EPI_GELU) {
    if constexpr (EPI == EPI_GELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = gelu_tanh_f(v[j]);
    }
    bf16_t* y = (bf16_t*)e.out + (int64_t)m * e.ldo + n;
    *(u32x2_t*)y = u32x2_t{pack2(v[0], v[1]), pack2(v[2], v[3])};
  } else if constexpr (EPI == EPI_RES) {
    bf16_t* x = (bf16_t*)e.out + (int64_t)m * e.ldo + n;
    const u32x2_t xw = *(const u32x2_t*)x;
    *(u32x2_t*)x = u32x2_t{pack2(lo_f(xw.x) + v[0], hi_f(xw.x) + v[1]), pack2(lo_f(xw.y) + v[2], hi_f(xw.y) + v[3])};
  } else if constexpr (EPI == EPI_GATE_RES) {
    const int b = m / e.rows_per_batch;
    const u32x2_t gw = *(const u32x2_t*)(e.gate + (int64_t)b * e.gate_bstride + n);
    bf16_t* x = (bf16_t*)e.out + (int64_t)m * e.ldo + n;
    const u32x2_t xw = *(const u32x2_t*)x;
    const float g4[4] = {lo_f(gw.x), hi_f(gw.x), lo_f(gw.y), hi_f(gw.y)};
    const float x4[4] = {lo_f(xw.x), hi_f(xw.x), lo_f(xw.y), hi_f(xw.y)};
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = x4[j] + rbf(g4[j] * v[j]);
    *(u32x2_t*)x = u32x2_t{pack2(o[0], o[1]), pack2(o[2], o[3])};
  } else {  // EPI_QKV
    const int hd = e.heads * e.head_dim;
    const int which = n / hd;
    const int hn = n - which * hd;
    const int h = hn / e.head_dim;
    const int d = hn - h * e.head_dim;
    const int b = m / e.rows_per_batch;
    const int s = e.seq_offset + (m - b * e.rows_per_batch);
    const int64_t off = ((((int64_t)which * e.batch + b) * e.heads + h) * e.s_pad + s) * e.head_dim + d;
    bf16_t* y = (bf16_t*)e.out + off;
    *(u32x2_t*)y = u32x2_t{pack2(v[0], v[1]), pack2(v[2], v[3])};
  }
}

// The per-column (bias, int8 weight scales) and per-row (int8 activation scales) operands of a
// wave's 128 x (16 NT) accumulator block, loaded ONCE before its stores: read inside the store
// loop, hipcc may not move them above an earlier store to `out` (possible alias), and every
// 16-byte store then waits (vmcnt(0)) for its own completion before the next operand load -- 32
// serialised store round trips per wave in the 128x128 form.
template <bool I8, int NT>
struct EpiCols {
  u32x2_t bw[NT];
  f32x4_t sw[I8 ? NT : 1];
  float sx[I8 ? 8 : 1];
};
template <bool I8, int NT>
__device__ __forceinline__ void epi_cols_load(EpiCols<I8, NT>& c, const EpiArgs& e, int M, int N, int mrow0,
                                              int ncol0, int lane) {
  const int g = lane >> 4, fr = lane & 15;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = min(ncol0 + j * 16 + g * 4, N - 4);
    c.bw[j] = *(const u32x2_t*)(e.bias + n);
    if constexpr (I8) c.sw[j] = *(const f32x4_t*)(e.sw + n);
  }
  if constexpr (I8) {
#pragma unroll
    for (int i = 0; i < 8; ++i) c.sx[i] = e.sx[min(mrow0 + i * 16 + fr, M - 1)];
  }
}
// epi_pre on preloaded operands: accumulator tile (i, j) of the block, the same arithmetic
template <int EPI, bool I8, int NT>
__device__ __forceinline__ u32x2_t epi_pre_c(const EpiCols<I8, NT>& c, int i, int j,
                                             const typename MfmaOp<I8>::acc& a) {
  const u32x2_t bw = c.bw[j];
  const float b4[4] = {lo_f(bw.x), hi_f(bw.x), lo_f(bw.y), hi_f(bw.y)};
  float v[4];
  if constexpr (I8) {
    const float sx = c.sx[i];
    const f32x4_t sw = c.sw[j];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = __builtin_fmaf((float)a[k], sx * sw[k], b4[k]);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = a[k] + b4[k];
  }
  rbf2(v[0], v[1]);  // the module output's bf16 rounding, two values per conversion
  rbf2(v[2], v[3]);
  if constexpr (EPI == EPI_GELU) {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = gelu_tanh_f(v[k]);
  }
  return u32x2_t{pack2(v[0], v[1]), pack2(v[2], v[3])};
}

// Post-swap part: 8 consecutive bf16 columns n..n+7 of row m (16-byte aligned, host-checked).
template <int EPI>
__device__ __forceinline__ void epi_store8(const EpiArgs& e, int m, int n, u32x4_t v) {
  if constexpr (EPI == EPI_BIAS || EPI == EPI_GELU) {
    *(u32x4_t*)((bf16_t*)e.out + (int64_t)m * e.ldo + n) = v;
  } else if constexpr (EPI == EPI_GATE_RES) {
    const int b = m / e.rows_per_batch;
    const u32x4_t gw = *(const u32x4_t*)(e.gate + (int64_t)b * e.gate_bstride + n);
    bf16_t* x = (bf16_t*)e.out + (int64_t)m * e.ldo + n;
    const u32x4_t xw = *(const u32x4_t*)x;
    const uint32_t vv[4] = {v.x, v.y, v.z, v.w}, gg[4] = {gw.x, gw.y, gw.z, gw.w},
                   xx[4] = {xw.x, xw.y, xw.z, xw.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      o[k] = pack2(lo_f(xx[k]) + rbf(lo_f(gg[k]) * lo_f(vv[k])), hi_f(xx[k]) + rbf(hi_f(gg[k]) * hi_f(vv[k])));
    *(u32x4_t*)x = u32x4_t{o[0], o[1], o[2], o[3]};
  } else {  // EPI_QKV: 8 columns stay inside one head (head_dim % 8 == 0)
    const int hd = e.heads * e.head_dim;
    const int which = n / hd;
    const int hn = n - which * hd;
    const int h = hn / e.head_dim;
    const int d = hn - h * e.head_dim;
    const int b = m / e.rows_per_batch;
    const int s = e.seq_offset + (m - b * e.rows_per_batch);
    const int64_t off = ((((int64_t)which * e.batch + b) * e.heads + h) * e.s_pad + s) * e.head_dim + d;
    *(u32x4_t*)((bf16_t*)e.out + off) = v;
  }
}

template <bool I8>
struct Mma4;
template <>
struct Mma4<false> {
  static __device__ __forceinline__ void acc(f32x4_t& c, const bf16x8_t& a, const bf16x8_t& b) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  }
  static __device__ __forceinline__ void init(f32x4_t& c, const bf16x8_t& a, const bf16x8_t& b) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
  }
};
template <>
struct Mma4<true> {
  static __device__ __forceinline__ void acc(i32x4_t& c, const i32x4_t& a, const i32x4_t& b) {
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  }
  static __device__ __forceinline__ void init(i32x4_t& c, const i32x4_t& a, const i32x4_t& b) {
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
  }
};

// Raw buffer descriptor (base, stride 0, num_records, dword3 0x00020000) in SGPRs.
__device__ __forceinline__ i32x4_t pp_rsrc(const char* base, int bytes) {
  const uint64_t p = (uint64_t)base;
  return i32x4_t{__builtin_amdgcn_readfirstlane((int)(uint32_t)p),
                 __builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32)),
                 __builtin_amdgcn_readfirstlane(bytes), 0x00020000};
}

// One 1-KiB LDS-DMA piece (buffer_load_dwordx4 ... lds) as inline asm: hipcc does not count it, so
// it adds no conservative vmcnt(0) before LDS reads it cannot prove disjoint from the DMA target
// (the loops' own counted waits cover it). M0 is declared clobbered.
__device__ __forceinline__ void lds_dma(const i32x4_t& r, const char QIE_LDS* dst, uint32_t voff, int soff) {
  const int lds = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)dst);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
               :
               : "v"(voff), "s"(r), "s"(lds), "s"(soff)
               : "memory", "m0");
}

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

EpiArgs make_epi(void* out, int64_t ldo, const void* bias) {
  EpiArgs e{};
  e.out = out;
  e.ldo = ldo;
  e.bias = (const bf16_t*)bias;
  e.rows_per_batch = 1;
  e.group = 1;
  return e;
}


// CU count of the current device (persistent kernels launch one work-group per CU)
int cu_count() {
  static int g_cu_count = 0;
  if (g_cu_count == 0) {
    int dev = 0, cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cu <= 0)
      cu = 256;
    g_cu_count = cu;
  }
  return g_cu_count;
}

}  // namespace
