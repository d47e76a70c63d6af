// MFMA GEMM family for the DiT linears: y = epilogue(x[M,K] . W[N,K]^T + bias).
//
// Replaces the cuBLAS(Lt) GEMMs that diffusers' nn.Linear layers run inside
// QwenImageTransformerBlock [U] -- the 68.7 %
// of DiT FLOPs that are linear.
//
// Kernels, all gfx950-only (cdna_hip_programming.md §5):
//   gemm_pp_kernel (big shapes: M, N >= 256, >= 160 tiles, aligned output) -- 256x256 tile,
//     8 waves in two ping-pong groups, 64-wide K tiles of whole 128-byte lines double buffered
//     by LDS-DMA, asm MFMAs with in-place accumulators, permlane16-widened 16-byte epilogue
//     stores. See its section below.
//   gemm_ring_kernel (the previous big-shape kernel, build with -DQIE_GEMM_PP=0) -- the same tile
//     with a 4-slot ring of 32-wide K slices (64-byte rows), fragments of slice k+1 read into
//     registers during slice k.
//   gemm_kernel (everything else: text-stream rows, small N) -- BMxBN tile, 2-stage:
//     * both operands are K-contiguous (activation rows, nn.Linear weight rows),
//       staged global -> LDS with 16-byte global_load_lds (LDS-DMA), one 128-byte
//       K-row per tile row (BK = 64 bf16 or 128 int8), double buffered;
//     * LDS image XOR-swizzled at 16-byte granularity, chunk' = chunk ^ ((row>>1)&7):
//       conflict-free for the ds_read_b128 lane groups; the swizzle is applied on the
//       per-lane GLOBAL address (LDS-DMA writes are lane-linear, rule 21);
// Common: MFMA 16x16x32 bf16 (or 16x16x64 i8) with the WEIGHT tile as the A operand and the
// activation tile as B, so each lane owns 4 consecutive output columns of one row; XCD-aware
// bijective block remap + grouped tile order so the 32 CUs of one XCD share L2-resident tiles.
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

// ---- wide epilogue (gemm_ring): lanes of one 16x16 MFMA tile hold 4 consecutive columns of one
// row (column group g = lane>>4). One v_permlane16_swap per dword between tiles j and j+1 gives
// every lane 8 consecutive columns: g0 <- tile j cols 0-7, g1 <- tile j+1 cols 0-7, g2 <- tile j
// cols 8-15, g3 <- tile j+1 cols 8-15 -> one 16-byte store per lane per tile pair, 64 contiguous
// bytes per row (cdna_hip_programming.md T21, adapted from permlane32 to the 16x16 layout).
// Pre-swap part: bias (+ int8 scales), bf16 rounding, activation, packed to 4 bf16.
template <int EPI, bool I8>
__device__ __forceinline__ u32x2_t epi_pre(const EpiArgs& e, int m, int n,
                                           const typename MfmaOp<I8>::acc& a) {
  const u32x2_t bw = *(const u32x2_t*)(e.bias + n);
  const float b4[4] = {lo_f(bw.x), hi_f(bw.x), lo_f(bw.y), hi_f(bw.y)};
  float v[4];
  if constexpr (I8) {
    const float sx = e.sx[m];
    const f32x4_t sw = *(const f32x4_t*)(e.sw + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = rbf(__builtin_fmaf((float)a[j], sx * sw[j], b4[j]));
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = rbf(a[j] + b4[j]);
  }
  if constexpr (EPI == EPI_GELU) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = gelu_tanh_f(v[j]);
  }
  return u32x2_t{pack2(v[0], v[1]), pack2(v[2], v[3])};
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

template <int BM, int BN, int WM, int WN, int EPI, bool I8>
__global__ void __launch_bounds__(WM* WN * 64)
    gemm_kernel(const char* __restrict__ X, int64_t ldx_b, const char* __restrict__ W, int64_t ldw_b,
                int M, int N, int K_bytes, EpiArgs e) {
  using Op = MfmaOp<I8>;
  if (const int bz = blockIdx.z) {  // head-batched launch (gridDim.z == 1 otherwise)
    X += bz * e.bsx_b;
    W += (bz / e.group) * e.bsw_b;
    e.out = (char*)e.out + bz * e.bso_b;
    e.ws = (char*)e.ws + bz * e.bso_b;
  }
  constexpr int NWAVE = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MT = TM / 16, NTL = TN / 16;
  constexpr int A_BYTES = BM * kRowBytes, W_BYTES = BN * kRowBytes;
  constexpr int STAGE = A_BYTES + W_BYTES;
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * STAGE];
  char QIE_LDS* smem = (char QIE_LDS*)smem_raw;

  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  const int wgid = xcd_remap(blockIdx.x, nwg);
  // grouped order: GROUP tile-rows at a time, n fastest within the group
  constexpr int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int gid = wgid / per_group;
  const int first_m = gid * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (wgid % per_group) % gsz;
  const int tn = (wgid % per_group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave / WN, wn = wave % WN;

  // split-K: blockIdx.y selects a K range of K_bytes (gridDim.y == 1 otherwise)
  const int64_t koff = (int64_t)blockIdx.y * K_bytes;
  const char* xg = X + (int64_t)m0 * ldx_b + koff;
  const char* wg = W + (int64_t)n0 * ldw_b + koff;
  const int m_valid = M - m0, n_valid = N - n0;

  typename Op::acc acc[MT][NTL];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j) acc[i][j] = typename Op::acc{0, 0, 0, 0};

  const int nk = K_bytes / kRowBytes;
  stage_tile<BM, NWAVE>(xg, ldx_b, m_valid, smem, wave, lane);
  stage_tile<BN, NWAVE>(wg, ldw_b, n_valid, smem + A_BYTES, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // per-lane fragment offsets (the swizzle term depends only on lane&15)
  const int fr = lane & 15;
  const int sw = (fr >> 1) & 7;
  const int a_row = wm * TM + fr;
  const int w_row = wn * TN + fr;

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      char QIE_LDS* nb = smem + (cur ^ 1) * STAGE;
      stage_tile<BM, NWAVE>(xg + (int64_t)(kt + 1) * kRowBytes, ldx_b, m_valid, nb, wave, lane);
      stage_tile<BN, NWAVE>(wg + (int64_t)(kt + 1) * kRowBytes, ldw_b, n_valid, nb + A_BYTES, wave, lane);
    }
    const char QIE_LDS* at = smem + cur * STAGE;
    const char QIE_LDS* wt = at + A_BYTES;
    // (an explicit two-register-set read pipeline measured 10-15 % slower at 252
    //  VGPRs; hipcc's own lgkmcnt ladder with 2 waves/SIMD does better here)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int cofs = ((kk * 4 + (lane >> 4)) ^ sw) << 4;
      typename Op::frag wf[NTL], af[MT];
#pragma unroll
      for (int j = 0; j < NTL; ++j)
        wf[j] = *(const typename Op::frag QIE_LDS*)(wt + (w_row + j * 16) * kRowBytes + cofs);
#pragma unroll
      for (int i = 0; i < MT; ++i)
        af[i] = *(const typename Op::frag QIE_LDS*)(at + (a_row + i * 16) * kRowBytes + cofs);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j) acc[i][j] = Op::mma(wf[j], af[i], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: acc[i][j][r] -> row m = m0 + wm*TM + i*16 + (lane&15),
  //                           col n = n0 + wn*TN + j*16 + (lane>>4)*4 + r
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = m0 + wm * TM + i * 16 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < NTL; ++j) {
      const int n = n0 + wn * TN + j * 16 + (lane >> 4) * 4;
      if (n >= N) continue;
      if constexpr (EPI == EPI_PARTIAL) {  // raw fp32 / int32 partial sums, 16 bytes per lane
        *(typename Op::acc*)((char*)e.ws + (((int64_t)blockIdx.y * M + m) * N + n) * 4) = acc[i][j];
      } else {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc_val<I8>(acc[i][j], r, 1.0f);
        epilogue4<EPI, I8>(e, m, n, v);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// gemm_ring: 256x256 block tile; NT=4: 8 waves (2 per SIMD) of 128x64, NT=8: 4 waves of 128x128
// (8x8 MFMA 16x16 tiles = 256 accumulator registers = the whole AGPR half of the file).
//   * K advances in 64-byte slices (32 bf16 / 64 int8 = one MFMA K-step) through a 4-slot
//     LDS ring filled by LDS-DMA (buffer_load ... lds) three slices ahead;
//   * the fragments of slice k+1 are read into the second register set while the 64 MFMAs of
//     slice k run: after every 4th MFMA one ds_read_b128, after every 8th one 1-KiB DMA piece,
//     so LDS latency is covered by the wave's own MFMA stream instead of a second wave;
//   * the MFMAs are inline asm with the accumulator tied in place ("+a"): the 256 accumulators
//     exactly fill the AGPRs and hipcc's allocator otherwise rotates them through VGPR copies;
//     being volatile they also pin the interleave above (hipcc keeps memory ops in order
//     around them) -- the waits for the fragment reads are still hipcc's own (lgkmcnt);
//   * one barrier per slice, counted vmcnt(8) keeps the newest slice in flight.
// LDS rows are 64 B (4 x 16-byte chunks); chunk' = chunk ^ 3*((row>>3)&1) is conflict-free for
// the ds_read_b128 lane groups {0-3,12-15,20-27} / {4-11,16-19,28-31} (MI355X_MICROARCH §LDS)
// of the 16-row fragment read.
constexpr int k4RowBytes = 64;
constexpr int k4Tile = 256 * k4RowBytes;  // one operand slice, 16 KiB
constexpr int k4Stage = 2 * k4Tile;       // X + W slice, 32 KiB
#ifndef QIE_RING_DEPTH  // 4 (5 slots, 160 KiB) measured -1 % vs 3
#define QIE_RING_DEPTH 3
#endif
constexpr int kRingD = QIE_RING_DEPTH;  // K slices in flight ahead of the one being multiplied
constexpr int k4Slots = kRingD + 1;     // LDS ring slots (4: 128 KiB, 5: 160 KiB)
// 4 = the 8-wave form (measured +3..7.5 % over the 2-stage kernel on the DiT GEMMs, bitwise equal);
// 8 = the 4-wave form, 5 % slower: one wave per SIMD exposes each LDS-DMA piece's issue cost
#ifndef QIE_RING_NT  // 8: the 4-wave form (see above)
#define QIE_RING_NT 4
#endif
constexpr int kRingNT = QIE_RING_NT;
#ifndef QIE_PP_LEAN  // gemm_pp: DMA pieces through pp_dma_lean (no hand-saved M0, no leading s_nop): +2-4 % A/B
#define QIE_PP_LEAN 1
#endif
#ifndef QIE_W4_LEAN  // gemm_w4: 1 = DMA pieces without the hand-saved M0 / leading s_nop (pp_dma_lean)
#define QIE_W4_LEAN 1
#endif
#ifndef QIE_W4_ABL  // timing ablations of gemm_w4 (wrong results): 1 no DMA in the loop, 2 no vmcnt at the barrier, 4 (w4s) loads from tile 0 only
#define QIE_W4_ABL 0
#endif
#ifndef QIE_W4_DMA  // gemm_w4: where the 16 DMA pieces of tile k+2 go in stage B (see the kernel)
#define QIE_W4_DMA 1
#endif
#ifndef QIE_GEMM_W4  // big plain / GELU / residual / QKV shapes: 1 gemm_w4_kernel (4 waves of 128x128, LDS-DMA),
                     // 2 gemm_w4s_kernel (VGPR-staged), 3 gemm_w4l_kernel (the library's schedule), 0 gemm_pp
#define QIE_GEMM_W4 4
#endif
#ifndef QIE_GEMM_PP  // 1: gemm_pp_kernel for the big shapes (+14 % over gemm_ring in A/B); 0: gemm_ring
#define QIE_GEMM_PP 1
#endif
#ifndef QIE_SPLITK_PP  // 1: split-K partials on gemm_pp tiles (256x256), 0: on gemm_kernel<128,128>
#define QIE_SPLITK_PP 1
#endif
#ifndef QIE_PP_ABL  // diagnostic ablations of gemm_pp (wrong results): 1 no DMA, 2 no LDS reads
#define QIE_PP_ABL 0
#endif

#ifdef QIE_GEMM_STAMP
// diagnostic build only (tools/gemm_stamp.hip): sums over waves of per-slice cycles
__device__ unsigned long long g_gstamp[4];
#endif

__device__ __forceinline__ int swz4(int row) { return ((row >> 3) & 1) * 3; }

// per-lane byte offsets of the PPW 1-KiB pieces a wave stages per operand slice
template <int NWAVE>
__device__ __forceinline__ void stage4_offsets(int64_t ld_bytes, int rows_valid, int wave, int lane,
                                               uint32_t* off) {
#pragma unroll
  for (int i = 0; i < 16 / NWAVE; ++i) {
    const int r = (wave + i * NWAVE) * 16 + (lane >> 2);  // 16 rows (1 KiB) per wave-instruction
    const int c = (lane & 3) ^ swz4(r);
    const int gr = r < rows_valid ? r : rows_valid - 1;
    off[i] = (uint32_t)(gr * ld_bytes) + (c << 4);
  }
}

// buffer descriptor over [base, base + bytes) (wave-uniform inputs only); kept out of the kernel
// body so the host pass, which has no AMDGPU builtin types, still emits the launch stub
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const char* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, bytes, 0x00020000);
}
__device__ __forceinline__ void dma_piece(const __amdgpu_buffer_rsrc_t& r, char QIE_LDS* dst, uint32_t voff,
                                          int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (QIE_LDS void*)dst, 16, voff, soff, 0, 0);
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

// Epilogue of a wave's 128 x (16 NT) accumulator block at output (mrow0, ncol0) -- rows
// mrow0 + 16i + (lane & 15), four consecutive columns per lane and tile. Every lane takes part
// in the permlane16 swaps, after which a lane holds 8 consecutive columns of one row; rows/columns
// past M/N are clamped for the loads and skipped for the store (N % 8 == 0, host-checked).
// EPI_QKV / EPI_QKV_NR with head_dim == 128 (host-checked for NR): the wave's 64 columns lie in
// one head of one of q/k/v, so the scatter address is computed once per wave and row. EPI_QKV_NR
// also applies the per-head RMSNorm (fp32 sum of squares over the head's 128 columns: the wave's
// 64 + its partner wave's 64, exchanged through `smem`) and the RoPE rotation of q and k, with
// the rounding points of qie_qk_norm_rope_bf16; it needs every wave of the workgroup here.
#ifndef QIE_NR_HOIST  // QKV + norm + RoPE epilogue: RoPE table loads of 4 row groups ahead of their stores
#define QIE_NR_HOIST 1
#endif
#ifndef QIE_GATE_UNIFORM  // gated-residual epilogue: one gate load + 8-row residual round trip
#define QIE_GATE_UNIFORM 1
#endif
// LDS_OK: the workgroup's LDS is free here (false in gemm_w4p, whose slots hold the next tile): the
// QKV + norm + RoPE form then loads its RoPE rows from the fp32 tables into registers instead.
template <int NT, int EPI, bool I8, bool LDS_OK = true>
__device__ __forceinline__ void ring_epilogue(typename MfmaOp<I8>::acc (&acc)[8][NT], const EpiArgs& e, int M,
                                              int N, int mrow0, int ncol0, int lane, char QIE_LDS* smem) {
  // MFMA D -> VALU read hazard (the MFMAs are inline asm, so hipcc pads nothing): 23 wait states
  // behind the last MFMA, then EVERY accumulator is redefined by an (empty) asm statement, so no
  // read of one -- an epilogue read, or a copy the register allocator makes on its own -- can be
  // placed above the nops, inside the tail of the MFMA stream, right behind the asm MFMA that
  // wrote the register (hipcc did exactly that for the register-heavy QKV + norm + RoPE form:
  // stale reads no hazard pass knew about)
  asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if constexpr (NT == 8)
      asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]), "+a"(acc[i][4]),
                   "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));
    else
      asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][NT - 1]));
  }
  const int g = lane >> 4, fr = lane & 15;
  if constexpr (EPI == EPI_PARTIAL) {  // raw fp32 / int32 partial sums of split blockIdx.y
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mrow0 + i * 16 + fr;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = ncol0 + j * 16 + g * 4;
        if (m < M && n < N) *(typename MfmaOp<I8>::acc*)((char*)e.ws + (((int64_t)blockIdx.y * M + m) * N + n) * 4) = acc[i][j];
      }
    }
    return;
  }
  EpiCols<I8, NT> cols;
  epi_cols_load<I8, NT>(cols, e, M, N, mrow0, ncol0, lane);
  constexpr bool QKV = EPI == EPI_QKV || EPI == EPI_QKV_NR;
  if constexpr (QKV && (NT == 4 || NT == 8)) {
    // NT == 4: the wave's 64 columns are one half of a head (its partner wave holds the other);
    // NT == 8: the wave's 128 columns are one whole head
    if (EPI == EPI_QKV_NR || e.head_dim == 128) {
      const int hd = e.heads * 128;
      const int which = ncol0 / hd;
      const int h = (ncol0 - which * hd) >> 7;
      const int dbase = ncol0 & 127;               // 0 or 64 (NT == 4), 0 (NT == 8)
      const int dl = (g & 1) * 16 + (g >> 1) * 8;  // the lane's column offset inside a 32-col pair
      // the lane's 8 consecutive bf16 of row i, column pair jp (bias added, rounded)
      auto cols8 = [&](int i, int jp) -> u32x4_t {
        const int mc = min(mrow0 + i * 16 + fr, M - 1);
        const int nb = ncol0 + jp * 32;
        u32x2_t a = epi_pre_c<EPI, I8, NT>(cols, i, 2 * jp, acc[i][2 * jp]);
        u32x2_t b = epi_pre_c<EPI, I8, NT>(cols, i, 2 * jp + 1, acc[i][2 * jp + 1]);
        const auto sx = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
        return u32x4_t{sx[0], sy[0], sx[1], sy[1]};
      };
      auto row_ptr = [&](int m) -> bf16_t* {
        const int b = m / e.rows_per_batch;
        const int s = e.seq_offset + (m - b * e.rows_per_batch);
        return (bf16_t*)e.out + ((((int64_t)which * e.batch + b) * e.heads + h) * e.s_pad + s) * 128 + dbase + dl;
      };
      bool done = false;
      if constexpr (EPI == EPI_QKV_NR) {
        if (which < 2) {
          // register path (NT == 8, no LDS): the RoPE row of row group i (its 4 column pairs) is
          // loaded one group ahead of its use, group 0 before pass 1, under its arithmetic
          auto rope_row = [&](int i, f32x4_t (&cs)[4], f32x4_t (&sn)[4]) {
            const int64_t o = (int64_t)(min(mrow0 + i * 16 + fr, M - 1) % e.rows_per_batch) * 64 + (dl >> 1);
#pragma unroll
            for (int jp = 0; jp < 4; ++jp) {
              cs[jp] = *(const f32x4_t*)(e.rcos + o + jp * 16);
              sn[jp] = *(const f32x4_t*)(e.rsin + o + jp * 16);
            }
          };
          f32x4_t rcs[2][4], rsn[2][4];
          if constexpr (NT == 8 && !LDS_OK) rope_row(0, rcs[0], rsn[0]);
          // pass 1: sum of squares of the rounded values over each 64-column half of the head
          // (the same order in both forms), the two halves added last
          auto half_ss = [&](int i, int hh) {
            float t = 0.f;
#pragma unroll
            for (int jp = 2 * hh; jp < 2 * hh + 2; ++jp) {
              const u32x4_t v = cols8(i, jp);
              const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                const float lo = lo_f(w4[k]), hi = hi_f(w4[k]);
                t += lo * lo + hi * hi;
              }
            }
            t += __shfl_xor(t, 16, 64);
            t += __shfl_xor(t, 32, 64);
            return t;
          };
          float ss[8];
          if constexpr (NT == 8) {
#pragma unroll
            for (int i = 0; i < 8; ++i) ss[i] = rsqrtf((half_ss(i, 0) + half_ss(i, 1)) * (1.0f / 128.0f) + e.eps);
          } else {  // the partner wave's half through LDS
#pragma unroll
            for (int i = 0; i < 8; ++i) ss[i] = half_ss(i, 0);
            const int wave = threadIdx.x >> 6;
            float QIE_LDS* red = (float QIE_LDS*)smem;
            if (g == 0) {
#pragma unroll
              for (int i = 0; i < 8; ++i) red[wave * 128 + i * 16 + fr] = ss[i];
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 8; ++i) ss[i] = rsqrtf((ss[i] + red[(wave ^ 1) * 128 + i * 16 + fr]) * (1.0f / 128.0f) + e.eps);
          }
          const bf16_t* nw = which == 0 ? e.nq : e.nk;
          const float osc = which == 0 ? e.qscale : 1.0f;
          if constexpr (NT == 8 && !LDS_OK) {
            u32x4_t wwv[4];
#pragma unroll
            for (int jp = 0; jp < 4; ++jp) wwv[jp] = *(const u32x4_t*)(nw + jp * 32 + dl);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              if (i < 7) rope_row(i + 1, rcs[(i + 1) & 1], rsn[(i + 1) & 1]);
              const int m = mrow0 + i * 16 + fr;
#pragma unroll
              for (int jp = 0; jp < 4; ++jp) {
                const uint32_t wv[4] = {wwv[jp].x, wwv[jp].y, wwv[jp].z, wwv[jp].w};
                const f32x4_t cs = rcs[i & 1][jp], sn = rsn[i & 1][jp];
                const u32x4_t v = cols8(i, jp);
                const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
                uint32_t o[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                  const float x0 = rbf(rbf(lo_f(w4[k]) * ss[i]) * lo_f(wv[k]));
                  const float x1 = rbf(rbf(hi_f(w4[k]) * ss[i]) * hi_f(wv[k]));
                  o[k] = pack2((x0 * cs[k] - x1 * sn[k]) * osc, (x0 * sn[k] + x1 * cs[k]) * osc);
                }
                if (m < M) *(u32x4_t*)(row_ptr(m) + jp * 32) = u32x4_t{o[0], o[1], o[2], o[3]};
              }
            }
            return;
          }
          if constexpr (NT == 8) {
            // the work-group's 256 RoPE rows (cos | sin, 512 B of fp32 each) staged into the free
            // LDS slots in one round trip by LDS-DMA (32 KiB pieces per wave), chunks XOR-swizzled by
            // the row so the 16 rows of a ds_read_b128 lane group hit 16 different banks; then
            // pass 2 reads them from LDS -- instead of 8 row-group round trips to L2 per wave, each
            // held behind the previous group's stores (possible alias with the qkv buffer)
            const int m0w = mrow0 & ~255, wave = threadIdx.x >> 6;
#pragma unroll 1
            for (int p = 0; p < 32; ++p) {
              const int P = wave * 32 + p, r = 2 * P + (lane >> 5), q = lane & 31;
              const int sl = min(m0w + r, M - 1) % e.rows_per_batch;
              const float* src = (q < 16 ? e.rcos : e.rsin) + (int64_t)sl * 64 + (((q & 15) ^ (r & 15)) << 2);
              __builtin_amdgcn_global_load_lds((const void*)src, (QIE_LDS void*)(smem + P * 1024), 16, 0, 0);
            }
            u32x4_t wwv[4];
#pragma unroll
            for (int jp = 0; jp < 4; ++jp) wwv[jp] = *(const u32x4_t*)(nw + jp * 32 + dl);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            const int rl0 = (mrow0 & 255) + fr;  // the lane's row in the work-group tile, row group 0
#pragma unroll
            for (int jp = 0; jp < 4; ++jp) {
              const int d0 = jp * 32 + dl;
              const uint32_t wv[4] = {wwv[jp].x, wwv[jp].y, wwv[jp].z, wwv[jp].w};
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                const int m = mrow0 + i * 16 + fr, rl = rl0 + i * 16;
                const char QIE_LDS* rrow = smem + rl * 512 + (((d0 >> 3) ^ (rl & 15)) << 4);
                const f32x4_t cs = *(const f32x4_t QIE_LDS*)rrow;
                const f32x4_t sn = *(const f32x4_t QIE_LDS*)(rrow + 256);
                const u32x4_t v = cols8(i, jp);
                const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
                uint32_t o[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                  const float x0 = rbf(rbf(lo_f(w4[k]) * ss[i]) * lo_f(wv[k]));
                  const float x1 = rbf(rbf(hi_f(w4[k]) * ss[i]) * hi_f(wv[k]));
                  o[k] = pack2((x0 * cs[k] - x1 * sn[k]) * osc, (x0 * sn[k] + x1 * cs[k]) * osc);
                }
                if (m < M) *(u32x4_t*)(row_ptr(m) + jp * 32) = u32x4_t{o[0], o[1], o[2], o[3]};
              }
            }
            return;
          }
          // pass 2: recompute the rounded values, RMSNorm (two bf16 roundings) and rotate
#pragma unroll
          for (int jp = 0; jp < NT / 2; ++jp) {
            const int d0 = dbase + jp * 32 + dl;
            const u32x4_t ww = *(const u32x4_t*)(nw + d0);
            const uint32_t wv[4] = {ww.x, ww.y, ww.z, ww.w};
#if QIE_NR_HOIST
            // the RoPE rows of 4 row groups loaded before their stores: hipcc may not move a table
            // load above a store to the qkv buffer (possible alias), so in loop order every row's
            // cos/sin would be a separate round trip
#pragma unroll
            for (int i4 = 0; i4 < 8; i4 += 4) {
              f32x4_t csv[4], snv[4];
#pragma unroll
              for (int ii = 0; ii < 4; ++ii) {
                const int sl = min(mrow0 + (i4 + ii) * 16 + fr, M - 1) % e.rows_per_batch;
                csv[ii] = *(const f32x4_t*)(e.rcos + (int64_t)sl * 64 + (d0 >> 1));
                snv[ii] = *(const f32x4_t*)(e.rsin + (int64_t)sl * 64 + (d0 >> 1));
              }
#pragma unroll
              for (int ii = 0; ii < 4; ++ii) {
                const int i = i4 + ii;
                const int m = mrow0 + i * 16 + fr;
                const f32x4_t cs = csv[ii], sn = snv[ii];
#else
            {
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                const int m = mrow0 + i * 16 + fr;
                const int sl = min(m, M - 1) % e.rows_per_batch;  // row of the segment's RoPE table
                const f32x4_t cs = *(const f32x4_t*)(e.rcos + (int64_t)sl * 64 + (d0 >> 1));
                const f32x4_t sn = *(const f32x4_t*)(e.rsin + (int64_t)sl * 64 + (d0 >> 1));
#endif
              const u32x4_t v = cols8(i, jp);
              const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
              uint32_t o[4];
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                const float x0 = rbf(rbf(lo_f(w4[k]) * ss[i]) * lo_f(wv[k]));
                const float x1 = rbf(rbf(hi_f(w4[k]) * ss[i]) * hi_f(wv[k]));
                o[k] = pack2((x0 * cs[k] - x1 * sn[k]) * osc, (x0 * sn[k] + x1 * cs[k]) * osc);
              }
              if (m < M) *(u32x4_t*)(row_ptr(m) + jp * 32) = u32x4_t{o[0], o[1], o[2], o[3]};
              }
            }
          }
          done = true;
        }
      }
      if (!done) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int m = mrow0 + i * 16 + fr;
          u32x4_t v[NT / 2];
#pragma unroll
          for (int jp = 0; jp < NT / 2; ++jp) v[jp] = cols8(i, jp);
          if (m < M) {
            bf16_t* row = row_ptr(m);
#pragma unroll
            for (int jp = 0; jp < NT / 2; ++jp) *(u32x4_t*)(row + 32 * jp) = v[jp];
          }
        }
      }
      return;
    }
  }
  if constexpr (EPI == EPI_GATE_RES && NT == 4) {
#if QIE_GATE_UNIFORM
    // the wave's 128 rows in one batch (wave-uniform; always so for the image rows, S_img % 128 ==
    // 0): one gate vector for all of them, so the residual loads of all 8 row groups fit the
    // registers the 4-row form spends on residual + gate, and go out in one round trip
    const int b0 = min(mrow0, M - 1) / e.rows_per_batch;
    if (b0 == min(mrow0 + 127, M - 1) / e.rows_per_batch) {
      u32x4_t gv[2], xv[8][2];
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int n = min(ncol0 + jp * 32 + (g & 1) * 16 + (g >> 1) * 8, N - 8);
        gv[jp] = *(const u32x4_t*)(e.gate + (int64_t)b0 * e.gate_bstride + n);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int mc = min(mrow0 + i * 16 + fr, M - 1);
          xv[i][jp] = *(const u32x4_t*)((const bf16_t*)e.out + (int64_t)mc * e.ldo + n);
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = mrow0 + i * 16 + fr;
        const int mc = min(m, M - 1);
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          const int nb = ncol0 + jp * 32;
          u32x2_t a = epi_pre_c<EPI, I8, NT>(cols, i, 2 * jp, acc[i][2 * jp]);
          u32x2_t b = epi_pre_c<EPI, I8, NT>(cols, i, 2 * jp + 1, acc[i][2 * jp + 1]);
          const auto sx = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
          const auto sy = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
          const uint32_t vv[4] = {sx[0], sy[0], sx[1], sy[1]};
          const uint32_t gg[4] = {gv[jp].x, gv[jp].y, gv[jp].z, gv[jp].w};
          const uint32_t xx[4] = {xv[i][jp].x, xv[i][jp].y, xv[i][jp].z, xv[i][jp].w};
          uint32_t o[4];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            o[k] = pack2(lo_f(xx[k]) + rbf(lo_f(gg[k]) * lo_f(vv[k])), hi_f(xx[k]) + rbf(hi_f(gg[k]) * hi_f(vv[k])));
          const int n = nb + (g & 1) * 16 + (g >> 1) * 8;
          if (m < M && n < N) *(u32x4_t*)((bf16_t*)e.out + (int64_t)m * e.ldo + n) = u32x4_t{o[0], o[1], o[2], o[3]};
        }
      }
      return;
    }
#endif
    // x is read and written in place, so hipcc cannot hoist a later row's residual load above an
    // earlier row's store: issue the residual and gate loads of 4 rows first, then combine and
    // store (one round trip per 4 rows instead of one per 16-byte chunk)
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      u32x4_t xv[4][2], gv[4][2];
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int mc = min(mrow0 + (4 * h2 + ii) * 16 + fr, M - 1);
        const int b = mc / e.rows_per_batch;
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          const int n = min(ncol0 + jp * 32 + (g & 1) * 16 + (g >> 1) * 8, N - 8);
          xv[ii][jp] = *(const u32x4_t*)((const bf16_t*)e.out + (int64_t)mc * e.ldo + n);
          gv[ii][jp] = *(const u32x4_t*)(e.gate + (int64_t)b * e.gate_bstride + n);
        }
      }
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int i = 4 * h2 + ii;
        const int m = mrow0 + i * 16 + fr;
        const int mc = min(m, M - 1);
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          const int nb = ncol0 + jp * 32;
          u32x2_t a = epi_pre_c<EPI, I8, NT>(cols, i, 2 * jp, acc[i][2 * jp]);
          u32x2_t b = epi_pre_c<EPI, I8, NT>(cols, i, 2 * jp + 1, acc[i][2 * jp + 1]);
          const auto sx = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
          const auto sy = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
          const uint32_t vv[4] = {sx[0], sy[0], sx[1], sy[1]};
          const uint32_t gg[4] = {gv[ii][jp].x, gv[ii][jp].y, gv[ii][jp].z, gv[ii][jp].w};
          const uint32_t xx[4] = {xv[ii][jp].x, xv[ii][jp].y, xv[ii][jp].z, xv[ii][jp].w};
          uint32_t o[4];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            o[k] = pack2(lo_f(xx[k]) + rbf(lo_f(gg[k]) * lo_f(vv[k])), hi_f(xx[k]) + rbf(hi_f(gg[k]) * hi_f(vv[k])));
          const int n = nb + (g & 1) * 16 + (g >> 1) * 8;
          if (m < M && n < N) *(u32x4_t*)((bf16_t*)e.out + (int64_t)m * e.ldo + n) = u32x4_t{o[0], o[1], o[2], o[3]};
        }
      }
    }
    return;
  }
  if constexpr (EPI != EPI_QKV_NR && EPI != EPI_PARTIAL) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mrow0 + i * 16 + fr;
      const int mc = min(m, M - 1);
#pragma unroll
      for (int jp = 0; jp < NT / 2; ++jp) {
        const int nb = ncol0 + jp * 32;
        u32x2_t a = epi_pre_c<EPI, I8, NT>(cols, i, 2 * jp, acc[i][2 * jp]);
        u32x2_t b = epi_pre_c<EPI, I8, NT>(cols, i, 2 * jp + 1, acc[i][2 * jp + 1]);
        const auto sx = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
        const int n = nb + (g & 1) * 16 + (g >> 1) * 8;
#ifdef QIE_EPI_ABL  // timing ablation (wrong results): 1 compute but do not store, 2 store without computing
        if constexpr (QIE_EPI_ABL == 1) {
          u32x4_t v = u32x4_t{sx[0], sy[0], sx[1], sy[1]};
          asm volatile("" ::"v"(v));
        } else if (m < M && n < N) {
          epi_store8<EPI>(e, m, n, u32x4_t{(uint32_t)m, (uint32_t)n, 0u, 0u});
        }
#else
        if (m < M && n < N) epi_store8<EPI>(e, m, n, u32x4_t{sx[0], sy[0], sx[1], sy[1]});
#endif
      }
    }
  }
}

// NT = 16-column MFMA tiles per wave: 8 -> 4 waves (2x2, 128x128 per wave, one wave per SIMD);
// 4 -> 8 waves (2x4, 128x64 per wave, two per SIMD: a wave's DMA issue hides behind its partner)
template <int NT, int EPI, bool I8>
__global__ void __launch_bounds__(NT == 8 ? 256 : 512, 1)
    gemm_ring_kernel(const char* __restrict__ X, int64_t ldx_b, const char* __restrict__ W, int64_t ldw_b,
                  int M, int N, int K_bytes, EpiArgs e) {
  using frag = typename MfmaOp<I8>::frag;
  using accT = typename MfmaOp<I8>::acc;
  __shared__ __attribute__((aligned(16))) char smem_raw[k4Slots * k4Stage];
  char QIE_LDS* smem = (char QIE_LDS*)smem_raw;

  const int tiles_m = (M + 255) >> 8, tiles_n = (N + 255) >> 8;
  const int nwg = tiles_m * tiles_n;
  const int wgid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int first_m = (wgid / per_group) * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (wgid % per_group) % gsz;
  const int tn = (wgid % per_group) / gsz;
  const int m0 = tm * 256, n0 = tn * 256;

  constexpr int WN = 256 / (NT * 16), NWAVE = 2 * WN, PPW = 16 / NWAVE;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int m_valid = M - m0, n_valid = N - n0;
  const int nk = K_bytes / k4RowBytes;  // host guarantees nk >= 4

  // buffer descriptors over this block's operand rows (wave-uniform); per-lane row offsets in
  // 32-bit VGPRs, the K position in the scalar offset
  const auto xr = make_rsrc(X + (int64_t)m0 * ldx_b, (int)(min(m_valid, 256) * ldx_b));
  const auto wr = make_rsrc(W + (int64_t)n0 * ldw_b, (int)(min(n_valid, 256) * ldw_b));
  uint32_t xo[PPW], wo[PPW];
  stage4_offsets<NWAVE>(ldx_b, m_valid, wave, lane, xo);
  stage4_offsets<NWAVE>(ldw_b, n_valid, wave, lane, wo);
  // DMA piece p (0..2*PPW-1) of slice kt: p < PPW -> X rows, else W rows
  auto dma = [&](int kt, int p) {
    const bool isw = p >= PPW;
    const int pi = isw ? p - PPW : p;
    char QIE_LDS* dst = smem + (kt % k4Slots) * k4Stage + (isw ? k4Tile : 0) +
                        (wave + pi * NWAVE) * 1024;
    if (isw) dma_piece(wr, dst, wo[pi], kt * k4RowBytes);
    else dma_piece(xr, dst, xo[pi], kt * k4RowBytes);
  };

  // fragment r of a slice: r < 8 -> W rows wn*16*NT + 16r + fr, else X rows wm*128 + 16(r-8) + fr
  const int fr = lane & 15;
  const int cofs = ((lane >> 4) ^ swz4(fr)) << 4;
  const int a_off = (wm * 128 + fr) * k4RowBytes + cofs;
  const int w_off = k4Tile + (wn * NT * 16 + fr) * k4RowBytes + cofs;
  auto ldfrag = [&](int kt, int r) -> frag {
    const char QIE_LDS* base = smem + (kt % k4Slots) * k4Stage;
    return *(const frag QIE_LDS*)(base + (r < 8 ? w_off + r * 16 * k4RowBytes
                                                 : a_off + (r - 8) * 16 * k4RowBytes));
  };

  accT acc[8][NT];
  frag af[2][8], wf[2][NT];

  // slice kt: 64 MFMAs on register set CUR; interleaved reads of slice kt+1 into set CUR^1 and
  // DMA of slice kt+3 into the slot last read by slice kt-2 (consumed before this barrier)
#ifdef QIE_GEMM_STAMP
  unsigned long long st_wait = 0, st_body = 0, st_n = 0;
#endif
  // W: slices allowed to stay in flight when slice kt+1 must have landed
  auto wait_bar = [&](auto n_t) {
    constexpr int n = decltype(n_t)::value;
    static_assert(n == 0 || n == 4 || n == 8 || n == 12 || n == 16, "vmcnt");
    if constexpr (n == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (n == 4) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    else if constexpr (n == 8) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    else if constexpr (n == 12) asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  };
  auto slice = [&](auto ph_t, auto cur_t, auto init_t, auto read_t, auto dma_t, auto w_t, int kt) {
    constexpr int PH = decltype(ph_t)::value;  // MFMA index (mod 8) after which a DMA piece goes
    constexpr int CUR = decltype(cur_t)::value;
    constexpr bool INIT = decltype(init_t)::value, READ = decltype(read_t)::value;
    constexpr bool DMA = decltype(dma_t)::value;
    constexpr int W = decltype(w_t)::value;
#ifdef QIE_GEMM_STAMP
    const unsigned long long ta = __builtin_amdgcn_s_memtime();
#endif
    if constexpr (READ) wait_bar(std::integral_constant<int, W * 2 * PPW>{});  // slice kt+1 landed
#pragma unroll
    for (int q = 0; q < 8 * NT; ++q) {
      const int i = q / NT, j = q % NT;
      if constexpr (INIT) Mma4<I8>::init(acc[i][j], wf[CUR][j], af[CUR][i]);
      else Mma4<I8>::acc(acc[i][j], wf[CUR][j], af[CUR][i]);
      if constexpr (READ) {
        // W fragments of slice kt+1 early (row 0 of the next slice needs all 8); the A
        // fragment of row i right after row i's last MFMA, so it can reuse row i's registers
        if ((q & 3) == 1 && q < 4 * NT) wf[CUR ^ 1][q >> 2] = ldfrag(kt + 1, q >> 2);
        if (j == NT - 1) af[CUR ^ 1][i] = ldfrag(kt + 1, 8 + i);
      }
      if constexpr (DMA) {
        if ((q & 7) == PH) dma(kt + kRingD, q >> 3);
      }
#ifdef QIE_GEMM_STAMP
      if (q == 0) st_wait += __builtin_amdgcn_s_memtime() - ta;
#endif
    }
#ifdef QIE_GEMM_STAMP
    st_body += __builtin_amdgcn_s_memtime() - ta;
    st_n += 1;
#endif
  };
  using T = std::true_type;
  using F = std::false_type;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  using W0 = std::integral_constant<int, 0>;
  using W1 = std::integral_constant<int, 1>;
  using W2 = std::integral_constant<int, 2>;
  using WD = std::integral_constant<int, kRingD - 2>;  // steady state: slices kt+2 .. kt+D-1

  // K loop; `ph` = MFMA index (mod 8) after which each LDS-DMA piece is issued (staggering it
  // between the two waves of a SIMD measured -1 %, so both use the same position)
  auto kloop = [&](auto ph) {
    // prologue: slices 0 .. D-1 in flight, slice 0 landed, its fragments read
  #pragma unroll
    for (int d = 0; d < kRingD; ++d)
  #pragma unroll
      for (int p = 0; p < 2 * PPW; ++p) dma(d, p);
    wait_bar(std::integral_constant<int, (kRingD - 1) * 2 * PPW>{});
  #pragma unroll
    for (int r = 0; r < NT; ++r) wf[0][r] = ldfrag(0, r);
  #pragma unroll
    for (int r = 0; r < 8; ++r) af[0][r] = ldfrag(0, 8 + r);
    slice(ph, I0{}, T{}, T{}, T{}, WD{}, 0);  // slice 0 (host: nk >= kRingD + 2)
    int kt = 1;
    for (; kt + 1 + kRingD < nk; kt += 2) {  // steady state: slices kt, kt+1 stage kt+D, kt+1+D
      slice(ph, I1{}, F{}, T{}, T{}, WD{}, kt);
      slice(ph, I0{}, F{}, T{}, T{}, WD{}, kt + 1);
    }
    // tail: nk is even (host: K_bytes % 128 == 0), so exactly D or D+1 (whichever is odd) slices
    // remain, register set 1 first (a data-dependent branch here makes hipcc spill AGPRs)
    if constexpr (kRingD == 3) {  // slices nk-3 .. nk-1
      slice(ph, I1{}, F{}, T{}, F{}, W1{}, kt);      // reads nk-2, everything staged
      slice(ph, I0{}, F{}, T{}, F{}, W0{}, kt + 1);  // reads nk-1
      slice(ph, I1{}, F{}, F{}, F{}, W0{}, kt + 2);
    } else {  // kRingD == 4: slices nk-5 .. nk-1
      slice(ph, I1{}, F{}, T{}, T{}, W2{}, kt);      // stages the last slice nk-1
      slice(ph, I0{}, F{}, T{}, F{}, W2{}, kt + 1);
      slice(ph, I1{}, F{}, T{}, F{}, W1{}, kt + 2);
      slice(ph, I0{}, F{}, T{}, F{}, W0{}, kt + 3);
      slice(ph, I1{}, F{}, F{}, F{}, W0{}, kt + 4);
    }
  };
  kloop(std::integral_constant<int, 3>{});
#ifdef QIE_GEMM_STAMP
  if (lane == 0) {
    atomicAdd(&g_gstamp[0], st_wait);
    atomicAdd(&g_gstamp[1], st_body);
    atomicAdd(&g_gstamp[2], st_n);
  }
#endif
  ring_epilogue<NT, EPI, I8>(acc, e, M, N, m0 + wm * 128, n0 + wn * NT * 16, lane, smem);
}

// ---------------------------------------------------------------------------------------------
// gemm_pp: the 256x256 tile with its two wave groups in ping-pong and full-line K tiles
// (cdna_hip_programming.md §5 "256² 8-phase template" / T3-T5, MI355X_MICROARCH.md "Two waves
// per SIMD"). Measured on the ring form: with its LDS-DMA removed the same MFMA + LDS-read loop
// runs 1.3-1.4x faster, i.e. the 64-byte-row slices (every 1-KiB DMA piece touching 16 half-used
// 128-byte lines) bound it. Here:
//   * K advances in 64-wide tiles of 128-byte LDS rows (8 rows x 128 B per DMA piece: whole
//     lines), double buffered: 2 x [X 256 rows | W 256 rows] = 128 KiB; row chunks XOR-swizzled
//     chunk ^ ((row >> 1) & 7) (conflict-free ds_read_b128, applied on the source address);
//   * waves 0-3 (group 0 = output rows 0-127) and 4-7 (group 1 = rows 128-255) put one wave of
//     each group on every SIMD; group 1 runs one workgroup barrier behind group 0, so between two
//     barriers one wave of every SIMD runs a 16-MFMA cluster while its partner reads the next
//     cluster's fragments and issues DMA pieces (whose issue cost hides under the partner's
//     MFMAs);
//   * per tile and wave 4 sections (m-half, k-step): (0,0) (0,1) (1,0) (1,1); the 8 W fragments
//     are read in sections 0-1 and kept, 4 X fragments per section;
//   * staging: X(k+1) in sections 0-1 of tile k (its buffer's X rows were last read in section 3
//     of tile k-1), W(k+2) in sections 2-3 of tile k (this buffer's W rows were last read in
//     section 1 of tile k); section 3 waits vmcnt(4) = everything but W(k+2) -> tile k+1 landed;
//   * every loader section ends with lgkmcnt(0) BEFORE its barrier, so each read has retired
//     before the barrier behind which the next DMA into its rows is issued (WAR), and each wave's
//     pieces of tile k+1 have landed before the barrier that precedes any read of it (RAW);
//   * DMA pieces are inline asm: hipcc does not count them, so it adds no conservative vmcnt(0)
//     before the LDS reads; the waits above are the only ones.
__device__ __forceinline__ i32x4_t pp_rsrc(const char* base, int bytes) {
  const uint64_t p = (uint64_t)base;
  return i32x4_t{__builtin_amdgcn_readfirstlane((int)(uint32_t)p),
                 __builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32)),
                 __builtin_amdgcn_readfirstlane(bytes), 0x00020000};
}
// one 1-KiB buffer_load_dwordx4 ... lds piece; M0 saved/set/restored inside the statement, s_nop 4
// covers a just-readfirstlane'd SGPR operand (cdna_hip_programming.md §5.7)
__device__ __forceinline__ void pp_dma(const i32x4_t& r, const char QIE_LDS* dst, uint32_t voff, int soff) {
  unsigned keep;
  const int lds = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)dst);
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(r), "s"(lds), "s"(soff)
      : "memory");
}

// the same piece for a loop where every operand is SALU-computed (no fresh readfirstlane): no
// leading s_nop, and M0 declared clobbered instead of saved / restored by hand
__device__ __forceinline__ void pp_dma_lean(const i32x4_t& r, const char QIE_LDS* dst, uint32_t voff, int soff) {
  const int lds = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)dst);
  asm volatile(
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %1, %3 offen lds"
      :
      : "v"(voff), "s"(r), "s"(lds), "s"(soff)
      : "memory", "m0");
}

constexpr int kPPTile = 256 * kRowBytes;  // one operand of one K tile, 32 KiB
#ifndef QIE_PP_XRING  // X tiles in flight + 1: 2 -> 128 KiB of LDS, 3 -> all 160 KiB
#define QIE_PP_XRING 2
#endif
constexpr int kPPX = QIE_PP_XRING;        // X slots; W always has 2
constexpr int kPPXA = kPPX - 1;           // X(k + kPPXA) is staged during tile k

template <int EPI, bool I8>
__global__ void __launch_bounds__(512, 2)
    gemm_pp_kernel(const char* __restrict__ X, int64_t ldx_b, const char* __restrict__ W, int64_t ldw_b,
                   int M, int N, int K_bytes, EpiArgs e) {
  using frag = typename MfmaOp<I8>::frag;
  using accT = typename MfmaOp<I8>::acc;
  constexpr int NT = 4, NWAVE = 8, PPO = 4;  // PPO: DMA pieces per wave per operand tile
  __shared__ __attribute__((aligned(16))) char smem_raw[(kPPX + 2) * kPPTile];
  char QIE_LDS* smem = (char QIE_LDS*)smem_raw;

  const int tiles_m = (M + 255) >> 8, tiles_n = (N + 255) >> 8;
  const int nwg = tiles_m * tiles_n;
  const int wgid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int first_m = (wgid / per_group) * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (wgid % per_group) % gsz;
  const int tn = (wgid % per_group) / gsz;
  const int m0 = tm * 256, n0 = tn * 256;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 2, wn = wave & 3;  // wm is also the ping-pong group
  const int m_valid = M - m0, n_valid = N - n0;
  const int nk = K_bytes / kRowBytes;  // host guarantees nk >= 3

  // split-K (EPI_PARTIAL): blockIdx.y selects a K range of K_bytes (gridDim.y == 1 otherwise)
  const int64_t koff = (int64_t)blockIdx.y * K_bytes;
  const i32x4_t xr = pp_rsrc(X + (int64_t)m0 * ldx_b + koff, (int)(min(m_valid, 256) * ldx_b - koff));
  const i32x4_t wr = pp_rsrc(W + (int64_t)n0 * ldw_b + koff, (int)(min(n_valid, 256) * ldw_b - koff));
  // piece i of an operand tile: rows 8 (wave + 8 i) .. +7, lane -> row + (lane >> 3), swizzled chunk
  uint32_t xo[PPO], wo[PPO];
#pragma unroll
  for (int i = 0; i < PPO; ++i) {
    const int r = (wave + i * NWAVE) * 8 + (lane >> 3);
    const int c = swz_chunk(r, lane & 7);
    xo[i] = (uint32_t)(min(r, m_valid - 1) * ldx_b) + (c << 4);
    wo[i] = (uint32_t)(min(r, n_valid - 1) * ldw_b) + (c << 4);
  }
  // LDS: X slots [0, kPPX) (tile kt in slot kt % kPPX), then two W slots (tile kt in kt & 1)
  auto xslot = [&](int kt) { return smem + (kt % kPPX) * kPPTile; };
  auto wslot = [&](int kt) { return smem + (kPPX + (kt & 1)) * kPPTile; };
  auto dmaX = [&](int kt, int i) {
    if constexpr (QIE_PP_LEAN) pp_dma_lean(xr, xslot(kt) + (wave + i * NWAVE) * 1024, xo[i], kt * kRowBytes);
    else pp_dma(xr, xslot(kt) + (wave + i * NWAVE) * 1024, xo[i], kt * kRowBytes);
  };
  auto dmaW = [&](int kt, int i) {
    if constexpr (QIE_PP_LEAN) pp_dma_lean(wr, wslot(kt) + (wave + i * NWAVE) * 1024, wo[i], kt * kRowBytes);
    else pp_dma(wr, wslot(kt) + (wave + i * NWAVE) * 1024, wo[i], kt * kRowBytes);
  };

  // fragment of k-step ks: lane reads row (lane & 15) of its 16-row block, chunk 4 ks + (lane >> 4)
  const int fr = lane & 15;
  const int a_row = wm * 128 + fr, w_row = wn * NT * 16 + fr;
  const int sw = (fr >> 1) & 7;  // swz_chunk term; (row + 16 i) >> 1 & 7 == row >> 1 & 7
  auto ldX = [&](int kt, int i, int ks) -> frag {
    return *(const frag QIE_LDS*)(xslot(kt) + (a_row + 16 * i) * kRowBytes + (((4 * ks + (lane >> 4)) ^ sw) << 4));
  };
  auto ldW = [&](int kt, int j, int ks) -> frag {
    return *(const frag QIE_LDS*)(wslot(kt) + (w_row + 16 * j) * kRowBytes + (((4 * ks + (lane >> 4)) ^ sw) << 4));
  };

  accT acc[8][NT];
  frag wf[2][NT], af[4];

  // loader-section end: lgkmcnt(0) and, when n >= 0, vmcnt(n), then the barrier
  auto ld_end = [&](auto n_t) {
    constexpr int n = decltype(n_t)::value;
    static_assert(n == -1 || n == 0 || n == 4 || n == 8, "vmcnt");
    if constexpr (n == -1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (n == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (n == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  // section (MH, KS) of tile kt. DX: stage X(kt+1) pieces 2 KS, 2 KS + 1 (sections MH = 0);
  // DW: stage W(kt+2) pieces 2 KS, 2 KS + 1 (sections MH = 1); VM: vmcnt of section (1, 1)
  auto section = [&](auto mh_t, auto ks_t, auto init_t, auto dx_t, auto dw_t, auto vm_t, int kt) {
    constexpr int MH = decltype(mh_t)::value, KS = decltype(ks_t)::value;
    constexpr bool INIT = decltype(init_t)::value && KS == 0;
    constexpr bool DX = decltype(dx_t)::value, DW = decltype(dw_t)::value;
    if constexpr (!(QIE_PP_ABL & 2) || decltype(init_t)::value) {
      if constexpr (MH == 0) {
#pragma unroll
        for (int j = 0; j < NT; ++j) wf[KS][j] = ldW(kt, j, KS);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = ldX(kt, 4 * MH + i, KS);
    }
    if constexpr (!(QIE_PP_ABL & 1)) {
      if constexpr (DX) {
        dmaX(kt + kPPXA, 2 * KS);
        dmaX(kt + kPPXA, 2 * KS + 1);
      }
      if constexpr (DW) {
        dmaW(kt + 2, 2 * KS);
        dmaW(kt + 2, 2 * KS + 1);
      }
    }
    if constexpr (MH == 1 && KS == 1) ld_end(vm_t);
    else ld_end(std::integral_constant<int, -1>{});
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        if constexpr (INIT) Mma4<I8>::init(acc[4 * MH + i][j], wf[KS][j], af[i]);
        else Mma4<I8>::acc(acc[4 * MH + i][j], wf[KS][j], af[i]);
      }
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_barrier" ::: "memory");
  };
  using T = std::true_type;
  using F = std::false_type;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using VNone = std::integral_constant<int, -1>;
  using V0 = std::integral_constant<int, 0>;
  using V4 = std::integral_constant<int, 4>;
  // tile kt: X(kt+1) if DX, W(kt+2) if DW; section (1,1) waits for tile kt+1
  auto tile = [&](auto init_t, auto dx_t, auto dw_t, auto vm_t, int kt) {
    section(I0{}, I0{}, init_t, dx_t, F{}, VNone{}, kt);
    section(I0{}, I1{}, init_t, dx_t, F{}, VNone{}, kt);
    section(I1{}, I0{}, init_t, F{}, dw_t, VNone{}, kt);
    section(I1{}, I1{}, init_t, F{}, dw_t, vm_t, kt);
  };

  // prologue (2 X slots): W(0), X(0), W(1); (3 X slots): X(0), W(0), X(1), W(1); wait for tile 0;
  // group 1 one barrier behind. Steady tile k stages X(k + kPPXA) and W(k + 2) and waits for
  // everything but its own pieces (vmcnt VS) -> tile k+1 has landed.
  using VS = std::integral_constant<int, kPPXA == 1 ? 4 : 8>;
  if constexpr (kPPXA == 1) {
#pragma unroll
    for (int i = 0; i < PPO; ++i) dmaW(0, i);
#pragma unroll
    for (int i = 0; i < PPO; ++i) dmaX(0, i);
  } else {
#pragma unroll
    for (int i = 0; i < PPO; ++i) dmaX(0, i);
#pragma unroll
    for (int i = 0; i < PPO; ++i) dmaW(0, i);
#pragma unroll
    for (int i = 0; i < PPO; ++i) dmaX(1, i);
  }
#pragma unroll
  for (int i = 0; i < PPO; ++i) dmaW(1, i);
  ld_end(VS{});
  if (wm == 1) asm volatile("s_barrier" ::: "memory");

  tile(T{}, T{}, T{}, VS{}, 0);
  int kt = 1;
  for (; kt < nk - 2; ++kt) tile(F{}, T{}, T{}, VS{}, kt);
  if constexpr (kPPXA == 1) tile(F{}, T{}, F{}, V0{}, kt);  // nk-2: stages X(nk-1), waits for it
  else tile(F{}, F{}, F{}, V0{}, kt);                       // nk-2: waits for tile nk-1
  tile(F{}, F{}, F{}, VNone{}, kt + 1);                     // nk-1
  if (wm == 0) asm volatile("s_barrier" ::: "memory");  // every wave passes the same barrier count

  ring_epilogue<NT, EPI, I8>(acc, e, M, N, m0 + wm * 128, n0 + wn * NT * 16, lane, smem);
}

// ---------------------------------------------------------------------------------------------
// gemm_w4: the 256x256 tile as FOUR waves of 128x128 -- one wave per SIMD, 8x8 16x16 MFMA tiles
// = 256 AGPR accumulators -- on the 64-wide K tiles of 128-byte LDS rows that gemm_pp uses.
// Why (profiles/r07_gemm_vs_hipblaslt_pmc.json): the library kernel with this shape runs one
// wave per SIMD that is parked 6 % of its cycles and reads 1/3 less LDS per MFMA (128x128 wave
// tile: 16 fragments per 64 MFMAs instead of 12 per 32), where gemm_pp's two ping-pong waves
// park 31 %. Per K tile (two k-steps, 128 MFMAs per wave):
//   stage A: 64 MFMAs of k-step 0 (fragment set 0), the k-step 1 fragments of the same tile read
//            into set 1 between them (one ds_read_b128 per 4 MFMAs);
//   barrier: vmcnt(0) lgkmcnt(0) -> this wave's DMA pieces of tile k+1 have landed and its reads
//            of tile k have retired; after the barrier that holds for every wave, so
//   stage B: 64 MFMAs of k-step 1 (set 1), the k-step 0 fragments of tile k+1 read into set 0
//            and the 16 DMA pieces of tile k+2 issued into tile k's slot (one per 4 MFMAs).
// Two slots of [X 256 rows | W 256 rows] x 128 B = 128 KiB; one barrier per 128 MFMAs.
template <int EPI, bool I8>
__global__ void __launch_bounds__(256, 1)
    gemm_w4_kernel(const char* __restrict__ X, int64_t ldx_b, const char* __restrict__ W, int64_t ldw_b,
                   int M, int N, int K_bytes, EpiArgs e) {
  using frag = typename MfmaOp<I8>::frag;
  using accT = typename MfmaOp<I8>::acc;
  constexpr int NWAVE = 4, PPO = 8;  // PPO: DMA pieces per wave per operand tile (32 pieces / 4 waves)
  __shared__ __attribute__((aligned(16))) char smem_raw[4 * kPPTile];
  char QIE_LDS* smem = (char QIE_LDS*)smem_raw;

  const int tiles_m = (M + 255) >> 8, tiles_n = (N + 255) >> 8;
  const int nwg = tiles_m * tiles_n;
  const int wgid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int first_m = (wgid / per_group) * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (wgid % per_group) % gsz;
  const int tn = (wgid % per_group) / gsz;
  const int m0 = tm * 256, n0 = tn * 256;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int m_valid = M - m0, n_valid = N - n0;
  const int nk = K_bytes / kRowBytes;  // host guarantees nk >= 3

  const int64_t koff = (int64_t)blockIdx.y * K_bytes;  // split-K range (gridDim.y == 1 otherwise)
  const i32x4_t xr = pp_rsrc(X + (int64_t)m0 * ldx_b + koff, (int)(min(m_valid, 256) * ldx_b - koff));
  const i32x4_t wr = pp_rsrc(W + (int64_t)n0 * ldw_b + koff, (int)(min(n_valid, 256) * ldw_b - koff));
  // piece i of an operand tile: rows 8 (wave + 4 i) .. +7, lane -> row + (lane >> 3), swizzled chunk
  uint32_t xo[PPO], wo[PPO];
#pragma unroll
  for (int i = 0; i < PPO; ++i) {
    const int r = (wave + i * NWAVE) * 8 + (lane >> 3);
    const int c = swz_chunk(r, lane & 7);
    xo[i] = (uint32_t)(min(r, m_valid - 1) * ldx_b) + (c << 4);
    wo[i] = (uint32_t)(min(r, n_valid - 1) * ldw_b) + (c << 4);
  }
  // slot s = kt & 1: X tile at s * 2 * kPPTile, W tile right after it
  auto xslot = [&](int kt) { return smem + (kt & 1) * 2 * kPPTile; };
  auto wslot = [&](int kt) { return smem + (kt & 1) * 2 * kPPTile + kPPTile; };
  // DMA piece p (0..15) of tile kt: p < 8 -> X piece p, else W piece p - 8
  auto dma = [&](int kt, int p) {
    if constexpr (QIE_W4_LEAN) {
      if (p < PPO) pp_dma_lean(xr, xslot(kt) + (wave + p * NWAVE) * 1024, xo[p], kt * kRowBytes);
      else pp_dma_lean(wr, wslot(kt) + (wave + (p - PPO) * NWAVE) * 1024, wo[p - PPO], kt * kRowBytes);
    } else {
      if (p < PPO) pp_dma(xr, xslot(kt) + (wave + p * NWAVE) * 1024, xo[p], kt * kRowBytes);
      else pp_dma(wr, wslot(kt) + (wave + (p - PPO) * NWAVE) * 1024, wo[p - PPO], kt * kRowBytes);
    }
  };

  const int fr = lane & 15;
  const int sw = (fr >> 1) & 7;
  const int a_row = wm * 128 + fr, w_row = wn * 128 + fr;
  // fragment r (0..15) of k-step ks of tile kt: r < 8 -> W rows w_row + 16 r, else X rows a_row + 16 (r - 8)
  auto ldfrag = [&](int kt, int ks, int r) -> frag {
    const int cofs = ((4 * ks + (lane >> 4)) ^ sw) << 4;
    if (r < 8) return *(const frag QIE_LDS*)(wslot(kt) + (w_row + 16 * r) * kRowBytes + cofs);
    return *(const frag QIE_LDS*)(xslot(kt) + (a_row + 16 * (r - 8)) * kRowBytes + cofs);
  };

  accT acc[8][8];
  frag wf[2][8], af[2][8];

  // one k-step: 64 MFMAs on set CUR (row i = q / 8, column tile j = q % 8); RD: read k-step
  // (rkt, rks) into set CUR ^ 1 (fragment q / 4 after MFMA q, q % 4 == 1); DM: DMA tile dkt
  // (piece q / 4 after MFMA q, q % 4 == 3)
  auto kstep = [&](auto cur_t, auto init_t, auto rd_t, auto dm_t, int rkt, int rks, int dkt) {
    constexpr int CUR = decltype(cur_t)::value;
    constexpr bool INIT = decltype(init_t)::value, RD = decltype(rd_t)::value, DM = decltype(dm_t)::value;
#pragma unroll
    for (int q = 0; q < 64; ++q) {
      const int i = q >> 3, j = q & 7;
      if constexpr (INIT) Mma4<I8>::init(acc[i][j], wf[CUR][j], af[CUR][i]);
      else Mma4<I8>::acc(acc[i][j], wf[CUR][j], af[CUR][i]);
      if constexpr (RD) {
        if ((q & 3) == 1) {
          const int r = q >> 2;
          if (r < 8) wf[CUR ^ 1][r] = ldfrag(rkt, rks, r);
          else af[CUR ^ 1][r - 8] = ldfrag(rkt, rks, r);
        }
      }
      if constexpr (DM && !(QIE_W4_ABL & 1)) {  // QIE_W4_DMA: 0 spread (1 per 4 MFMAs), 1 burst (1 per MFMA), 2 (1 per 2)
        if constexpr (QIE_W4_DMA == 0) {
          if ((q & 3) == 3) dma(dkt, q >> 2);
        } else if constexpr (QIE_W4_DMA == 1) {
          if (q < 16) dma(dkt, q);
        } else {
          if ((q & 1) == 1 && q < 32) dma(dkt, q >> 1);
        }
      }
    }
  };
  using T = std::true_type;
  using F = std::false_type;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  auto bar = [&]() {
    if constexpr (QIE_W4_ABL & 2) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // timing only
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };

  // prologue: tiles 0 and 1 in flight, tile 0 landed, its k-step 0 fragments read
#pragma unroll
  for (int p = 0; p < 2 * PPO; ++p) dma(0, p);
#pragma unroll
  for (int p = 0; p < 2 * PPO; ++p) dma(1, p);
  asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
#pragma unroll
  for (int r = 0; r < 8; ++r) wf[0][r] = ldfrag(0, 0, r);
#pragma unroll
  for (int r = 0; r < 8; ++r) af[0][r] = ldfrag(0, 0, 8 + r);

  // tile 0 (INIT), tiles 1 .. nk-3 (steady), nk-2 (no DMA), nk-1 (no reads ahead)
  kstep(I0{}, T{}, T{}, F{}, 0, 1, 0);
  bar();
  kstep(I1{}, F{}, T{}, T{}, 1, 0, 2);
  int kt = 1;
  for (; kt < nk - 2; ++kt) {
    kstep(I0{}, F{}, T{}, F{}, kt, 1, 0);
    bar();
    kstep(I1{}, F{}, T{}, T{}, kt + 1, 0, kt + 2);
  }
  kstep(I0{}, F{}, T{}, F{}, kt, 1, 0);  // nk-2
  bar();
  kstep(I1{}, F{}, T{}, F{}, kt + 1, 0, 0);
  kstep(I0{}, F{}, T{}, F{}, kt + 1, 1, 0);  // nk-1
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  kstep(I1{}, F{}, F{}, F{}, 0, 0, 0);

  ring_epilogue<8, EPI, I8>(acc, e, M, N, m0 + wm * 128, n0 + wn * 128, lane, smem);
}

// gemm_w4s: gemm_w4 with the operand tiles staged through VGPRs instead of LDS-DMA (the
// library's form): every thread loads its 16 x 16 B of tile k+3 with buffer_load_dwordx4 (64
// VGPRs) while tile k computes, and writes tile k+2 from the registers into the slot freed by
// the mid-tile barrier. The LDS layout (128-byte rows, XOR-swizzled chunks) is gemm_w4's; the
// ablation there showed the DMA issue itself as the cost (0.80 ms without it vs 0.93 ms).
template <int EPI, bool I8>
__global__ void __launch_bounds__(256, 1)
    gemm_w4s_kernel(const char* __restrict__ X, int64_t ldx_b, const char* __restrict__ W, int64_t ldw_b,
                    int M, int N, int K_bytes, EpiArgs e) {
  using frag = typename MfmaOp<I8>::frag;
  using accT = typename MfmaOp<I8>::acc;
  typedef unsigned int g4_t __attribute__((ext_vector_type(4)));
  constexpr int NWAVE = 4, PPO = 8;
  __shared__ __attribute__((aligned(16))) char smem_raw[4 * kPPTile];
  char QIE_LDS* smem = (char QIE_LDS*)smem_raw;

  const int tiles_m = (M + 255) >> 8, tiles_n = (N + 255) >> 8;
  const int nwg = tiles_m * tiles_n;
  const int wgid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int first_m = (wgid / per_group) * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (wgid % per_group) % gsz;
  const int tn = (wgid % per_group) / gsz;
  const int m0 = tm * 256, n0 = tn * 256;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int m_valid = M - m0, n_valid = N - n0;
  const int nk = K_bytes / kRowBytes;  // host guarantees nk >= 3

  const int64_t koff = (int64_t)blockIdx.y * K_bytes;
  auto mk = [](const char* base, int bytes) {
    const uint64_t p = (uint64_t)base;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)p);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                             __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
  };
  const auto xr = mk(X + (int64_t)m0 * ldx_b + koff, (int)(min(m_valid, 256) * ldx_b - koff));
  const auto wr = mk(W + (int64_t)n0 * ldw_b + koff, (int)(min(n_valid, 256) * ldw_b - koff));
  uint32_t xo[PPO], wo[PPO];
#pragma unroll
  for (int i = 0; i < PPO; ++i) {
    const int r = (wave + i * NWAVE) * 8 + (lane >> 3);
    const int c = swz_chunk(r, lane & 7);
    xo[i] = (uint32_t)(min(r, m_valid - 1) * ldx_b) + (c << 4);
    wo[i] = (uint32_t)(min(r, n_valid - 1) * ldw_b) + (c << 4);
  }
  auto xslot = [&](int kt) { return smem + (kt & 1) * 2 * kPPTile; };
  auto wslot = [&](int kt) { return smem + (kt & 1) * 2 * kPPTile + kPPTile; };
  g4_t g[2 * PPO];
  auto gload = [&](int kt, int p) {
    if constexpr (QIE_W4_ABL & 4) kt = 0;  // timing ablation: every load re-reads tile 0 (L2-resident)
    if (p < PPO) g[p] = __builtin_amdgcn_raw_buffer_load_b128(xr, xo[p], kt * kRowBytes, 0);
    else g[p] = __builtin_amdgcn_raw_buffer_load_b128(wr, wo[p - PPO], kt * kRowBytes, 0);
  };
  auto gstore = [&](int kt, int p) {
    char QIE_LDS* dst = (p < PPO ? xslot(kt) + (wave + p * NWAVE) * 1024
                                 : wslot(kt) + (wave + (p - PPO) * NWAVE) * 1024) + lane * 16;
    *(g4_t QIE_LDS*)dst = g[p];
  };

  const int fr = lane & 15;
  const int sw = (fr >> 1) & 7;
  const int a_row = wm * 128 + fr, w_row = wn * 128 + fr;
  auto ldfrag = [&](int kt, int ks, int r) -> frag {
    const int cofs = ((4 * ks + (lane >> 4)) ^ sw) << 4;
    if (r < 8) return *(const frag QIE_LDS*)(wslot(kt) + (w_row + 16 * r) * kRowBytes + cofs);
    return *(const frag QIE_LDS*)(xslot(kt) + (a_row + 16 * (r - 8)) * kRowBytes + cofs);
  };

  accT acc[8][8];
  frag wf[2][8], af[2][8];
  // one k-step on set CUR; RD: read (rkt, rks) into CUR ^ 1; ST: write half H (8 pieces) of tile
  // skt from g; LD: then reload that half of g with tile lkt. Stage A (CUR 0) moves half 1, stage
  // B (CUR 1) half 0, so each stage carries 16 fragment reads and 8 tile stores: tile j's half 0
  // is stored in stage B of tile j-2, its half 1 in stage A of tile j-1 (slot j & 1 is free from
  // the barrier of tile j-2 on), and both are visible after the barrier of tile j-1.
  auto kstep = [&](auto cur_t, auto init_t, auto rd_t, auto st_t, auto ld_t, int rkt, int rks, int skt, int lkt) {
    constexpr int CUR = decltype(cur_t)::value;
    constexpr int H = CUR ^ 1;
    constexpr bool INIT = decltype(init_t)::value, RD = decltype(rd_t)::value;
    constexpr bool ST = decltype(st_t)::value, LD = decltype(ld_t)::value;
#pragma unroll
    for (int q = 0; q < 64; ++q) {
      const int i = q >> 3, j = q & 7;
      if constexpr (INIT) Mma4<I8>::init(acc[i][j], wf[CUR][j], af[CUR][i]);
      else Mma4<I8>::acc(acc[i][j], wf[CUR][j], af[CUR][i]);
      if constexpr (RD) {
        if ((q & 3) == 1) {
          const int r = q >> 2;
          if (r < 8) wf[CUR ^ 1][r] = ldfrag(rkt, rks, r);
          else af[CUR ^ 1][r - 8] = ldfrag(rkt, rks, r);
        }
      }
      if constexpr (ST) {
        if ((q & 7) == 3) gstore(skt, 8 * H + (q >> 3));
      }
      if constexpr (LD) {
        if ((q & 7) == 7) gload(lkt, 8 * H + (q >> 3));
      }
    }
  };
  using T = std::true_type;
  using F = std::false_type;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  // this wave's LDS stores / reads retired, then the barrier: no vmcnt, so the register loads
  // stay in flight across it (hipcc's own counted waits guard their use in the stores)
  auto bar = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  // prologue: tile 0 and half 0 of tile 1 into LDS; g = [tile 2 half 0 | tile 1 half 1]
#pragma unroll
  for (int p = 0; p < 2 * PPO; ++p) gload(0, p);
#pragma unroll
  for (int p = 0; p < 2 * PPO; ++p) gstore(0, p);
#pragma unroll
  for (int p = 0; p < 2 * PPO; ++p) gload(1, p);
#pragma unroll
  for (int p = 0; p < PPO; ++p) gstore(1, p);
#pragma unroll
  for (int p = 0; p < PPO; ++p) gload(2, p);
  bar();
#pragma unroll
  for (int r = 0; r < 8; ++r) wf[0][r] = ldfrag(0, 0, r);
#pragma unroll
  for (int r = 0; r < 8; ++r) af[0][r] = ldfrag(0, 0, 8 + r);

  // tile kt: A = k-step 0, stores tile kt+1 half 1, loads tile kt+2 half 1; barrier;
  //          B = k-step 1, reads tile kt+1 k-step 0, stores tile kt+2 half 0, loads tile kt+3 half 0
  int kt = 0;
  if (nk > 3) {
    kstep(I0{}, T{}, T{}, T{}, T{}, 0, 1, 1, 2);
    bar();
    kstep(I1{}, F{}, T{}, T{}, T{}, 1, 0, 2, 3);
    for (kt = 1; kt < nk - 3; ++kt) {
      kstep(I0{}, F{}, T{}, T{}, T{}, kt, 1, kt + 1, kt + 2);
      bar();
      kstep(I1{}, F{}, T{}, T{}, T{}, kt + 1, 0, kt + 2, kt + 3);
    }
    kstep(I0{}, F{}, T{}, T{}, T{}, kt, 1, kt + 1, kt + 2);  // nk-3
  } else {
    kstep(I0{}, T{}, T{}, T{}, T{}, 0, 1, 1, 2);  // nk == 3: tile 0 is nk-3
  }
  bar();
  kstep(I1{}, F{}, T{}, T{}, F{}, kt + 1, 0, kt + 2, 0);
  ++kt;  // nk-2
  kstep(I0{}, F{}, T{}, T{}, F{}, kt, 1, kt + 1, 0);
  bar();
  kstep(I1{}, F{}, T{}, F{}, F{}, kt + 1, 0, 0, 0);
  ++kt;  // nk-1
  kstep(I0{}, F{}, T{}, F{}, F{}, kt, 1, 0, 0);
  kstep(I1{}, F{}, F{}, F{}, F{}, 0, 0, 0, 0);

  ring_epilogue<8, EPI, I8>(acc, e, M, N, m0 + wm * 128, n0 + wn * 128, lane, smem);
}

// ---------------------------------------------------------------------------------------------
// gemm_w4l: gemm_w4's tile (4 waves of 128x128, 256 AGPR accumulators) and LDS image (two slots
// of [X 256 rows | W 256 rows] x 128 B, XOR-swizzled chunks, filled by LDS-DMA) on the schedule of
// the library's fastest kernel for these shapes (hipBLASLt's MT256x256x64 MI16x16 DirectToLds
// PGR2 kernel, studied in its disassembly). The difference to gemm_w4 is where the time goes:
// every fragment of a whole 64-wide K tile is held in VGPRs (2 sets x 16 x 4 = 128 VGPRs), and
// the k-step 1 fragments are read one per MFMA at the START of the tile, so the tile's LDS slot
// is free early and the 16 DMA pieces of tile kt+2 spread over the other ~90 MFMAs instead of
// bursting. Per tile kt (128 MFMAs per wave; set 0 = the k-step 0 fragments, already in flight):
//   phase A (k-step 0): set 1 read behind MFMAs 0-15 (lgkmcnt(7) before MFMA 0, lgkmcnt(8) before
//     MFMA 8 retire set 0); at MFMA QB1 `lgkmcnt(0); s_barrier` -- every wave has read all of
//     tile kt -- then the 8 X pieces of tile kt+2 into tile kt's slot, one per DS1 MFMAs;
//   phase B (k-step 1, set 1): the 8 W pieces of tile kt+2, one per DS2 MFMAs; at MFMA 64 + QB2
//     `vmcnt(16); s_barrier` -- this wave's pieces of tile kt+1 (issued a whole tile earlier)
//     have landed, and after the barrier everyone's -- then set 0 of tile kt+1, one per MFMA.
// Two barriers per 128 MFMAs. The reads are inline asm with hand-counted lgkmcnt waits (hipcc
// counts neither them nor the DMA pieces, so it adds no waits of its own in the loop).
#ifndef QIE_W4L_QB1  // MFMA of phase A after which the slot-free barrier sits
#define QIE_W4L_QB1 24
#endif
#ifndef QIE_W4L_DS1  // MFMAs between the X pieces (phase A)
#define QIE_W4L_DS1 3
#endif
#ifndef QIE_W4L_DS2  // MFMAs between the W pieces (phase B)
#define QIE_W4L_DS2 5
#endif
#ifndef QIE_W4L_QB2  // MFMA of phase B after which the tile-landed barrier sits (then 16 reads)
#define QIE_W4L_QB2 48
#endif
#ifndef QIE_W4L_PRIO  // s_setprio 3 over the MFMA runs, 0 before each barrier (the library's form)
#define QIE_W4L_PRIO 1
#endif

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

#ifndef QIE_W4L_XAUX  // cache bits of the X / W pieces: 0 none, 1 sc0 sc1, 2 nt, 3 sc1, 4 sc0
#define QIE_W4L_XAUX 0
#endif
#ifndef QIE_W4L_WAUX
#define QIE_W4L_WAUX 0
#endif
#ifndef QIE_W4L_ABL  // timing ablations (wrong results): 1 no DMA in the loop, 2 no vmcnt wait, 4 no W DMA, 8 no X DMA
#define QIE_W4L_ABL 0
#endif
template <int AUX>
__device__ __forceinline__ void w4l_dma(const i32x4_t& r, const char QIE_LDS* dst, uint32_t voff, int soff) {
  const int lds = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)dst);
#define QIE_W4L_DMA_ASM(BITS)                                                           \
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen" BITS " lds" \
               :                                                                        \
               : "v"(voff), "s"(r), "s"(lds), "s"(soff)                                 \
               : "memory", "m0")
  if constexpr (AUX == 1) QIE_W4L_DMA_ASM(" sc0 sc1");
  else if constexpr (AUX == 2) QIE_W4L_DMA_ASM(" nt");
  else if constexpr (AUX == 3) QIE_W4L_DMA_ASM(" sc1");
  else if constexpr (AUX == 4) QIE_W4L_DMA_ASM(" sc0");
  else QIE_W4L_DMA_ASM("");
#undef QIE_W4L_DMA_ASM
}

#ifndef QIE_W4L_UNIFORM  // 1: the 16 pieces evenly over MFMAs QB1+1 .. 64+QB2-2 (QIE_W4L_ALT: X, W alternating)
#define QIE_W4L_UNIFORM 1
#endif
#ifndef QIE_W4L_ALT
#define QIE_W4L_ALT 0
#endif
// piece k (0..15) goes after MFMA g_k = QB1 + 1 + k * span / 16 of the tile's 128
__host__ __device__ constexpr int w4l_piece(int g) {
  constexpr int first = QIE_W4L_QB1 + 1, span = 64 + QIE_W4L_QB2 - 1 - first;
  for (int k = 0; k < 16; ++k)
    if (first + k * span / 16 == g) return k;
  return -1;
}

template <int OFF, class FR>
__device__ __forceinline__ void w4l_read(FR& f, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f) : "v"(addr), "i"(OFF));
}

template <int EPI, bool I8>
__global__ void __launch_bounds__(256, 1)
    gemm_w4l_kernel(const char* __restrict__ X, int64_t ldx_b, const char* __restrict__ W, int64_t ldw_b,
                    int M, int N, int K_bytes, EpiArgs e) {
  using frag = typename MfmaOp<I8>::frag;
  using accT = typename MfmaOp<I8>::acc;
  constexpr int NWAVE = 4, PPO = 8;  // PPO: DMA pieces per wave per operand tile
  constexpr int kSlot = 2 * kPPTile;  // 64 KiB: X tile then W tile
  static_assert(QIE_W4L_QB1 >= 16 && (QIE_W4L_UNIFORM || QIE_W4L_QB1 + 1 + 7 * QIE_W4L_DS1 < 64), "phase A placement");
  static_assert(QIE_W4L_UNIFORM || 1 + 7 * QIE_W4L_DS2 < QIE_W4L_QB2, "phase B placement");
  static_assert(QIE_W4L_QB2 + 16 <= 64, "phase B reads");
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * kSlot];
  char QIE_LDS* smem = (char QIE_LDS*)smem_raw;

  const int tiles_m = (M + 255) >> 8, tiles_n = (N + 255) >> 8;
  const int nwg = tiles_m * tiles_n;
  const int wgid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int first_m = (wgid / per_group) * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (wgid % per_group) % gsz;
  const int tn = (wgid % per_group) / gsz;
  const int m0 = tm * 256, n0 = tn * 256;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int m_valid = M - m0, n_valid = N - n0;
  const int nk = K_bytes / kRowBytes;  // host guarantees nk >= 3

  const int64_t koff = (int64_t)blockIdx.y * K_bytes;  // split-K range (gridDim.y == 1 otherwise)
  const i32x4_t xr = pp_rsrc(X + (int64_t)m0 * ldx_b + koff, (int)(min(m_valid, 256) * ldx_b - koff));
  const i32x4_t wr = pp_rsrc(W + (int64_t)n0 * ldw_b + koff, (int)(min(n_valid, 256) * ldw_b - koff));
  // piece p of an operand tile: rows 8 (wave + 4 p) .. +7, lane -> row + (lane >> 3), swizzled chunk
  uint32_t xo[PPO], wo[PPO];
#pragma unroll
  for (int i = 0; i < PPO; ++i) {
    const int r = (wave + i * NWAVE) * 8 + (lane >> 3);
    const int c = swz_chunk(r, lane & 7);
    xo[i] = (uint32_t)(min(r, m_valid - 1) * ldx_b) + (c << 4);
    wo[i] = (uint32_t)(min(r, n_valid - 1) * ldw_b) + (c << 4);
  }
  auto dmaX = [&](int kt, int p) {
    w4l_dma<QIE_W4L_XAUX>(xr, smem + (kt & 1) * kSlot + (wave + p * NWAVE) * 1024, xo[p], kt * kRowBytes);
  };
  auto dmaW = [&](int kt, int p) {
    w4l_dma<QIE_W4L_WAUX>(wr, smem + (kt & 1) * kSlot + kPPTile + (wave + p * NWAVE) * 1024, wo[p], kt * kRowBytes);
  };

  // piece k of the uniform schedule: X pieces 0..7 then W (or alternating with QIE_W4L_ALT)
  auto dma_piece_k = [&](int kt, int k) {
    const bool is_x = QIE_W4L_ALT ? (k & 1) == 0 : k < PPO;
    const int p = QIE_W4L_ALT ? k >> 1 : (k & (PPO - 1));
    if (is_x) {
      if constexpr (!(QIE_W4L_ABL & 9)) dmaX(kt, p);
    } else {
      if constexpr (!(QIE_W4L_ABL & 5)) dmaW(kt, p);
    }
  };
  // fragment read addresses: fragment r of a set sits 16 rows (2 KiB) after fragment r - 1, and
  // k-step 1's chunk is k-step 0's ^ 4; the slot bit (64 KiB) is toggled per tile
  const int fr = lane & 15;
  const int sw = (fr >> 1) & 7;
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const uint32_t c0 = (uint32_t)(((lane >> 4) ^ sw) << 4), c1 = (uint32_t)(((4 + (lane >> 4)) ^ sw) << 4);
  uint32_t xa0 = lds0 + (wm * 128 + fr) * kRowBytes + c0;
  uint32_t wa0 = lds0 + kPPTile + (wn * 128 + fr) * kRowBytes + c0;
  uint32_t xa1 = (lds0 + kSlot + (wm * 128 + fr) * kRowBytes + c1);           // slot 1: toggled at tile 0
  uint32_t wa1 = (lds0 + kSlot + kPPTile + (wn * 128 + fr) * kRowBytes + c1);

  accT acc[8][8];
  frag wf[2][8], af[2][8];

  // the 16 reads of one set in the order the MFMAs consume them: W0, X0, W1..W7, X1..X7
  auto rd = [&](auto set_t, auto r_t) {
    constexpr int S = decltype(set_t)::value, R = decltype(r_t)::value;
    const uint32_t xa = S ? xa1 : xa0, wa = S ? wa1 : wa0;
    if constexpr (R == 0) w4l_read<0>(wf[S][0], wa);
    else if constexpr (R == 1) w4l_read<0>(af[S][0], xa);
    else if constexpr (R < 9) w4l_read<2048 * (R - 1)>(wf[S][R - 1], wa);
    else w4l_read<2048 * (R - 8)>(af[S][R - 8], xa);
  };
  auto prio = [&](auto p_t) {
    if constexpr (QIE_W4L_PRIO) __builtin_amdgcn_s_setprio(decltype(p_t)::value);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I3 = std::integral_constant<int, 3>;

  // one K tile. INIT: first tile (accumulators start at 0); DMA: stage tile kt+2; NEXT: read set 0
  // of tile kt+1 at the end
  auto tile = [&](auto init_t, auto dma_t, auto next_t, int kt) {
    constexpr bool INIT = decltype(init_t)::value, DMA = decltype(dma_t)::value, NEXT = decltype(next_t)::value;
    xa1 ^= (uint32_t)kSlot;
    wa1 ^= (uint32_t)kSlot;
    // ---- phase A: k-step 0 on set 0
    static_for<0, 64>([&](auto q_t) {
      constexpr int q = decltype(q_t)::value;
      constexpr int i = q >> 3, j = q & 7;
      if constexpr (q == 0) asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory");
      if constexpr (q == 8) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      if constexpr (INIT) Mma4<I8>::init(acc[i][j], wf[0][j], af[0][i]);
      else Mma4<I8>::acc(acc[i][j], wf[0][j], af[0][i]);
      if constexpr (q < 16) rd(I1{}, q_t);
      if constexpr (q == QIE_W4L_QB1) {
        prio(I0{});
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        prio(I3{});
      }
      if constexpr (DMA && QIE_W4L_UNIFORM) {
        constexpr int k = w4l_piece(q);
        if constexpr (k >= 0) dma_piece_k(kt + 2, k);
      } else if constexpr (DMA && !(QIE_W4L_ABL & 9) && q > QIE_W4L_QB1 && (q - QIE_W4L_QB1 - 1) % QIE_W4L_DS1 == 0 &&
                           (q - QIE_W4L_QB1 - 1) / QIE_W4L_DS1 < PPO)
        dmaX(kt + 2, (q - QIE_W4L_QB1 - 1) / QIE_W4L_DS1);
    });
    // ---- phase B: k-step 1 on set 1
    if constexpr (NEXT) {
      xa0 ^= (uint32_t)kSlot;
      wa0 ^= (uint32_t)kSlot;
    }
    static_for<0, 64>([&](auto q_t) {
      constexpr int q = decltype(q_t)::value;
      constexpr int i = q >> 3, j = q & 7;
      Mma4<I8>::acc(acc[i][j], wf[1][j], af[1][i]);
      if constexpr (DMA && QIE_W4L_UNIFORM) {
        constexpr int k = w4l_piece(64 + q);
        if constexpr (k >= 0) dma_piece_k(kt + 2, k);
      } else if constexpr (DMA && !(QIE_W4L_ABL & 5) && q >= 1 && (q - 1) % QIE_W4L_DS2 == 0 &&
                           (q - 1) / QIE_W4L_DS2 < PPO)
        dmaW(kt + 2, (q - 1) / QIE_W4L_DS2);
      if constexpr (NEXT && q == QIE_W4L_QB2) {
        prio(I0{});
        if constexpr (QIE_W4L_ABL & 15) asm volatile("s_barrier" ::: "memory");
        else if constexpr (DMA) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        prio(I3{});
      }
      if constexpr (NEXT && q >= QIE_W4L_QB2 && q < QIE_W4L_QB2 + 16) rd(I0{}, std::integral_constant<int, q - QIE_W4L_QB2>{});
    });
    prio(I0{});
  };
  using T = std::true_type;
  using F = std::false_type;

  // prologue: tiles 0 and 1 in flight, tile 0 landed everywhere, set 0 of tile 0 read
#pragma unroll
  for (int p = 0; p < PPO; ++p) dmaX(0, p);
#pragma unroll
  for (int p = 0; p < PPO; ++p) dmaW(0, p);
#pragma unroll
  for (int p = 0; p < PPO; ++p) dmaX(1, p);
#pragma unroll
  for (int p = 0; p < PPO; ++p) dmaW(1, p);
  asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  static_for<0, 16>([&](auto r_t) { rd(I0{}, r_t); });
  prio(I3{});

  tile(T{}, T{}, T{}, 0);
  int kt = 1;
  for (; kt < nk - 2; ++kt) tile(F{}, T{}, T{}, kt);
  tile(F{}, F{}, T{}, kt);      // nk-2: nothing left to stage, reads tile nk-1
  tile(F{}, F{}, F{}, kt + 1);  // nk-1
  asm volatile("s_barrier" ::: "memory");  // no wave's epilogue LDS use overlaps another's reads

  if (QIE_W4L_ABL & 16) {  // timing ablation: the epilogue only for a never-seen ldo (no stores)
    if (e.ldo != -12345) return;
  }
  ring_epilogue<8, EPI, I8>(acc, e, M, N, m0 + wm * 128, n0 + wn * 128, lane, smem);
}

// ---------------------------------------------------------------------------------------------
// gemm_w4p: gemm_w4l as a persistent kernel -- one work-group per CU walks the output tiles
// b, b + G, b + 2G, ... (the same tile order and XCD placement as one work-group per tile) and
// runs ONE K-tile pipeline across tile boundaries: the last two K tiles of tile t stage K tiles 0
// and 1 of tile t+1 and read its first fragment set, so tile t's epilogue (bias / GELU / gated
// residual and the 128 KiB of stores) runs while the next tile's operands are already landing,
// and the next tile starts on fragments in registers instead of on a cold prologue.
// Row / column offsets of the DMA pieces are those of a full 256-row tile; rows past M or N lie
// past the buffer descriptor's range and read as zeros (never stored). EPI_QKV_NR takes its RoPE
// rows straight from the tables here (ring_epilogue's LDS_OK = false): the LDS holds the next tile.
#ifndef QIE_W4P_GROUP  // 0: by output width (below); else a fixed group size
#define QIE_W4P_GROUP 0
#endif
static int g_cu_count = 0;

template <int EPI, bool I8>
__global__ void __launch_bounds__(256, 1)
    gemm_w4p_kernel(const char* __restrict__ X, int64_t ldx_b, const char* __restrict__ W, int64_t ldw_b,
                    int M, int N, int K_bytes, EpiArgs e) {
  static_assert(EPI != EPI_PARTIAL, "w4p epilogues");
  using frag = typename MfmaOp<I8>::frag;
  using accT = typename MfmaOp<I8>::acc;
  constexpr int NWAVE = 4, PPO = 8;
  constexpr int kSlot = 2 * kPPTile;
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * kSlot];
  char QIE_LDS* smem = (char QIE_LDS*)smem_raw;

  const int tiles_m = (M + 255) >> 8, tiles_n = (N + 255) >> 8;
  const int nwg = tiles_m * tiles_n;
  const int nk = K_bytes / kRowBytes;  // host guarantees nk >= 3
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;

  struct TileRef {
    int m0, n0;
    i32x4_t xr, wr;
  };
  auto tile_of = [&](int vb) {
    const int wgid = xcd_remap(vb, nwg);
    // M tiles per group of the tile order: 4 for the narrow outputs (N = 3072: down-proj 0.855 ->
    // 0.838 ms, out-proj equal), 8 for the wide ones (up / QKV: 8 best by 0.5-1 %)
    const int GROUP = QIE_W4P_GROUP ? QIE_W4P_GROUP : (tiles_n <= 16 ? 4 : 8);
    const int per_group = GROUP * tiles_n;
    const int first_m = (wgid / per_group) * GROUP;
    const int gsz = min(tiles_m - first_m, GROUP);
    TileRef t;
    t.m0 = (first_m + (wgid % per_group) % gsz) * 256;
    t.n0 = ((wgid % per_group) / gsz) * 256;
    t.xr = pp_rsrc(X + (int64_t)t.m0 * ldx_b, (int)(min(M - t.m0, 256) * ldx_b));
    t.wr = pp_rsrc(W + (int64_t)t.n0 * ldw_b, (int)(min(N - t.n0, 256) * ldw_b));
    return t;
  };
  uint32_t xo[PPO], wo[PPO];
#pragma unroll
  for (int i = 0; i < PPO; ++i) {
    const int r = (wave + i * NWAVE) * 8 + (lane >> 3);
    const int c = swz_chunk(r, lane & 7);
    xo[i] = (uint32_t)(r * ldx_b) + (c << 4);
    wo[i] = (uint32_t)(r * ldw_b) + (c << 4);
  }
  // piece k (0..15) of K tile dkt of tile tr into LDS slot sl: X pieces 0..7, then W
  auto dma_piece = [&](const TileRef& tr, int sl, int dkt, int k) {
    if (k < PPO)
      w4l_dma<QIE_W4L_XAUX>(tr.xr, smem + sl * kSlot + (wave + k * NWAVE) * 1024, xo[k], dkt * kRowBytes);
    else
      w4l_dma<QIE_W4L_WAUX>(tr.wr, smem + sl * kSlot + kPPTile + (wave + (k - PPO) * NWAVE) * 1024, wo[k - PPO],
                            dkt * kRowBytes);
  };

  const int fr = lane & 15;
  const int sw = (fr >> 1) & 7;
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const uint32_t c0 = (uint32_t)(((lane >> 4) ^ sw) << 4), c1 = (uint32_t)(((4 + (lane >> 4)) ^ sw) << 4);
  uint32_t xa0 = lds0 + (wm * 128 + fr) * kRowBytes + c0;
  uint32_t wa0 = lds0 + kPPTile + (wn * 128 + fr) * kRowBytes + c0;
  uint32_t xa1 = (lds0 + kSlot + (wm * 128 + fr) * kRowBytes + c1);
  uint32_t wa1 = (lds0 + kSlot + kPPTile + (wn * 128 + fr) * kRowBytes + c1);

  accT acc[8][8];
  frag wf[2][8], af[2][8];
  auto rd = [&](auto set_t, auto r_t) {
    constexpr int S = decltype(set_t)::value, R = decltype(r_t)::value;
    const uint32_t xa = S ? xa1 : xa0, wa = S ? wa1 : wa0;
    if constexpr (R == 0) w4l_read<0>(wf[S][0], wa);
    else if constexpr (R == 1) w4l_read<0>(af[S][0], xa);
    else if constexpr (R < 9) w4l_read<2048 * (R - 1)>(wf[S][R - 1], wa);
    else w4l_read<2048 * (R - 8)>(af[S][R - 8], xa);
  };
  auto prio = [&](auto p_t) {
    if constexpr (QIE_W4L_PRIO) __builtin_amdgcn_s_setprio(decltype(p_t)::value);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I3 = std::integral_constant<int, 3>;

  // one K tile in slot sl: INIT (first K tile of an output tile), DMA (stage K tile dkt of tile
  // dsrc into slot sl), NEXT (read set 0 of the following K tile, in slot sl ^ 1)
  auto ktile = [&](auto init_t, auto dma_t, auto next_t, int sl, const TileRef& dsrc, int dkt) {
    constexpr bool INIT = decltype(init_t)::value, DMA = decltype(dma_t)::value, NEXT = decltype(next_t)::value;
    xa1 ^= (uint32_t)kSlot;
    wa1 ^= (uint32_t)kSlot;
    static_for<0, 64>([&](auto q_t) {
      constexpr int q = decltype(q_t)::value;
      constexpr int i = q >> 3, j = q & 7;
      if constexpr (q == 0) asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory");
      if constexpr (q == 8) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      if constexpr (INIT) Mma4<I8>::init(acc[i][j], wf[0][j], af[0][i]);
      else Mma4<I8>::acc(acc[i][j], wf[0][j], af[0][i]);
      if constexpr (q < 16) rd(I1{}, q_t);
      if constexpr (q == QIE_W4L_QB1) {
        prio(I0{});
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        prio(I3{});
      }
      if constexpr (DMA) {
        constexpr int k = w4l_piece(q);
        if constexpr (k >= 0) dma_piece(dsrc, sl, dkt, k);
      }
    });
    if constexpr (NEXT) {
      xa0 ^= (uint32_t)kSlot;
      wa0 ^= (uint32_t)kSlot;
    }
    static_for<0, 64>([&](auto q_t) {
      constexpr int q = decltype(q_t)::value;
      constexpr int i = q >> 3, j = q & 7;
      Mma4<I8>::acc(acc[i][j], wf[1][j], af[1][i]);
      if constexpr (DMA) {
        constexpr int k = w4l_piece(64 + q);
        if constexpr (k >= 0) dma_piece(dsrc, sl, dkt, k);
      }
      if constexpr (NEXT && q == QIE_W4L_QB2) {
        prio(I0{});
        if constexpr (DMA) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        prio(I3{});
      }
      if constexpr (NEXT && q >= QIE_W4L_QB2 && q < QIE_W4L_QB2 + 16) rd(I0{}, std::integral_constant<int, q - QIE_W4L_QB2>{});
    });
    prio(I0{});
  };
  using T = std::true_type;
  using F = std::false_type;

  int vb = blockIdx.x;
  TileRef cur = tile_of(vb);
  // prologue of the first tile: K tiles 0 and 1 in flight, 0 landed everywhere, set 0 read
#pragma unroll
  for (int k = 0; k < 16; ++k) dma_piece(cur, 0, 0, k);
#pragma unroll
  for (int k = 0; k < 16; ++k) dma_piece(cur, 1, 1, k);
  asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  static_for<0, 16>([&](auto r_t) { rd(I0{}, r_t); });
  prio(I3{});
  int g = 0;  // flat K-tile count of this work-group: K tile kt of the current tile is in slot (g + kt) & 1
  while (true) {
    const int vbn = vb + (int)gridDim.x;
    const bool has_next = vbn < nwg;
    const TileRef nxt = tile_of(has_next ? vbn : vb);
    // one code path for every tile (the accumulators must not meet at a branch: hipcc then
    // shuffles all 256 through VGPRs and scratch); the last tile of the work-group re-stages its
    // own K tiles 0 and 1 as a stand-in "next" tile and drains them before it exits
    ktile(T{}, T{}, T{}, g & 1, cur, 2);
    int kt = 1;
    for (; kt < nk - 2; ++kt) ktile(F{}, T{}, T{}, (g + kt) & 1, cur, kt + 2);
    ktile(F{}, T{}, T{}, (g + kt) & 1, nxt, 0);  // nk-2: stages the next tile's K tile 0
    if constexpr (EPI != EPI_QKV_NR) {
      ktile(F{}, T{}, T{}, (g + kt + 1) & 1, nxt, 1);  // nk-1: its K tile 1, reads its set 0
      ring_epilogue<8, EPI, I8, false>(acc, e, M, N, cur.m0 + wm * 128, cur.n0 + wn * 128, lane, smem);
    } else {
      // the norm + RoPE epilogue needs the 64 VGPRs of set 0: read it behind the epilogue (the
      // wait then also covers the epilogue's stores, issued after K tile 1's pieces)
      ktile(F{}, T{}, F{}, (g + kt + 1) & 1, nxt, 1);
      ring_epilogue<8, EPI, I8, false>(acc, e, M, N, cur.m0 + wm * 128, cur.n0 + wn * 128, lane, smem);
      xa0 ^= (uint32_t)kSlot;
      wa0 ^= (uint32_t)kSlot;
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      static_for<0, 16>([&](auto r_t) { rd(I0{}, r_t); });
    }
    if (!has_next) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // no LDS-DMA outlives the work-group
      break;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // nothing of the epilogue ahead of set 0's count
    g += nk;
    vb = vbn;
    cur = nxt;
  }
}

template <int EPI, bool I8>
int launch_gemm(const void* x, int64_t ldx, const void* w, int64_t ldw, int M, int N, int K,
                const EpiArgs& e, hipStream_t s) {
  const int eb = I8 ? 1 : 2;
  QIE_CHECK_ARG(x && w && e.out && e.bias);
  QIE_CHECK_ARG(M > 0 && N > 0 && K > 0);
  QIE_CHECK_ARG((K * eb) % kRowBytes == 0 && N % 4 == 0);
  QIE_CHECK_ARG(((ldx * eb) % 16) == 0 && ((ldw * eb) % 16) == 0);
  QIE_CHECK_ARG(((uintptr_t)x % 16) == 0 && ((uintptr_t)w % 16) == 0);
  const int64_t ldx_b = ldx * eb, ldw_b = ldw * eb;
  const int kb = K * eb;
  const int64_t big_tiles = (int64_t)((M + 255) / 256) * ((N + 255) / 256);
  const bool wide = N % 8 == 0 && ((uintptr_t)e.out % 16) == 0 && e.ldo % 8 == 0 &&
                    (EPI != EPI_GATE_RES || (((uintptr_t)e.gate % 16) == 0 && e.gate_bstride % 8 == 0)) &&
                    (EPI != EPI_QKV || e.head_dim % 8 == 0);
  if (wide && M >= 256 && N >= 256 && big_tiles >= 160 && kb >= (kRingD + 2) * k4RowBytes) {
    if constexpr (QIE_GEMM_W4 == 4 && EPI != EPI_QKV_NR) {
      if (g_cu_count == 0) {
        int dev = 0, cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cu <= 0)
          cu = 256;
        g_cu_count = cu;
      }
      const int grid = (int)std::min<int64_t>(big_tiles, g_cu_count);
      gemm_w4p_kernel<EPI, I8><<<grid, 256, 0, s>>>((const char*)x, ldx_b, (const char*)w, ldw_b, M, N, kb, e);
    } else if constexpr (QIE_GEMM_W4 >= 3)
      gemm_w4l_kernel<EPI, I8><<<(int)big_tiles, 256, 0, s>>>((const char*)x, ldx_b, (const char*)w, ldw_b, M, N,
                                                             kb, e);
    else if constexpr (QIE_GEMM_W4 == 2 && EPI != EPI_QKV_NR)
      gemm_w4s_kernel<EPI, I8><<<(int)big_tiles, 256, 0, s>>>((const char*)x, ldx_b, (const char*)w, ldw_b, M, N,
                                                             kb, e);
    else if constexpr (QIE_GEMM_W4 == 1 && EPI != EPI_QKV_NR)
      gemm_w4_kernel<EPI, I8><<<(int)big_tiles, 256, 0, s>>>((const char*)x, ldx_b, (const char*)w, ldw_b, M, N,
                                                            kb, e);
    else if constexpr (QIE_GEMM_PP)  // (kb % 128 == 0 and kb >= 320 hold, so nk >= 3)
      gemm_pp_kernel<EPI, I8><<<(int)big_tiles, 512, 0, s>>>((const char*)x, ldx_b, (const char*)w, ldw_b, M,
                                                            N, kb, e);
    else
      gemm_ring_kernel<kRingNT, EPI, I8><<<(int)big_tiles, 2 * (256 / (kRingNT * 16)) * 64, 0, s>>>(
          (const char*)x, ldx_b, (const char*)w, ldw_b, M, N, kb, e);
    return qie_last_error();
  }
  if (M >= 256 && N >= 256 && big_tiles >= 160) {
    const int nwg = (int)big_tiles;
    gemm_kernel<256, 256, 2, 4, EPI, I8><<<nwg, 512, 0, s>>>((const char*)x, ldx_b, (const char*)w,
                                                            ldw_b, M, N, kb, e);
  } else {
    const int nwg = ((M + 127) / 128) * ((N + 127) / 128);
    gemm_kernel<128, 128, 2, 2, EPI, I8><<<nwg, 256, 0, s>>>((const char*)x, ldx_b, (const char*)w,
                                                            ldw_b, M, N, kb, e);
  }
  return qie_last_error();
}

// Split-K reduce: adds the `splits` partial sums of 4 consecutive columns in range order (fp32
// for bf16, int32 for int8 -- the int8 total is then exactly the unsplit accumulator) and runs
// the same epilogue as the unsplit kernels.
template <int EPI, bool I8>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(EpiArgs e, int M, int N, int splits) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int n4 = N >> 2;
  if (q >= (int64_t)M * n4) return;
  const int m = (int)(q / n4), n = (int)(q - (int64_t)m * n4) * 4;
  const int64_t plane = (int64_t)M * N;
  float v[4];
  if constexpr (I8) {
    const i32x4_t* p = (const i32x4_t*)e.ws + q;
    i32x4_t t = p[0];
    for (int s = 1; s < splits; ++s) t += *(const i32x4_t*)((const int*)p + s * plane);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (float)t[r];
  } else {
    const f32x4_t* p = (const f32x4_t*)e.ws + q;
    f32x4_t t = p[0];
    for (int s = 1; s < splits; ++s) t += *(const f32x4_t*)((const float*)p + s * plane);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = t[r];
  }
  epilogue4<EPI, I8>(e, m, n, v);
}

template <bool I8>
int launch_splitk(const void* x, int64_t ldx, const void* w, int M, int N, int K, int splits,
                  int epi_kind, EpiArgs e, int64_t ws_bytes, hipStream_t s) {
  const int eb = I8 ? 1 : 2;
  QIE_CHECK_ARG(x && w && e.out && e.bias);
  QIE_CHECK_ARG(M > 0 && N > 0 && K > 0 && N % 4 == 0 && splits >= 1 && splits <= 64);
  QIE_CHECK_ARG((K * eb) % (splits * kRowBytes) == 0);
  QIE_CHECK_ARG(((ldx * eb) % 16) == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)w % 16) == 0);
  const int kb = K * eb / splits;
  if (splits == 1) {
    // one K range: the short-M tiles run with their real epilogue, no partials and no reduce
    // (the least CU-time per output, which is what a side-stream launch costs its neighbours)
    const bool wide = N % 8 == 0 && ((uintptr_t)e.out % 16) == 0 &&
                      (epi_kind == EPI_QKV ? e.head_dim % 8 == 0 : e.ldo % 8 == 0) &&
                      (epi_kind != EPI_GATE_RES || (((uintptr_t)e.gate % 16) == 0 && e.gate_bstride % 8 == 0));
    if (QIE_GEMM_PP && wide && N >= 256 && kb >= 3 * kRowBytes) {
      const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
      const char* xc = (const char*)x;
      const char* wc = (const char*)w;
      const int64_t lx = ldx * eb, lw = (int64_t)K * eb;
      switch (epi_kind) {
        case EPI_BIAS: gemm_pp_kernel<EPI_BIAS, I8><<<tiles, 512, 0, s>>>(xc, lx, wc, lw, M, N, kb, e); break;
        case EPI_GELU: gemm_pp_kernel<EPI_GELU, I8><<<tiles, 512, 0, s>>>(xc, lx, wc, lw, M, N, kb, e); break;
        case EPI_GATE_RES:
          gemm_pp_kernel<EPI_GATE_RES, I8><<<tiles, 512, 0, s>>>(xc, lx, wc, lw, M, N, kb, e);
          break;
        default: gemm_pp_kernel<EPI_QKV, I8><<<tiles, 512, 0, s>>>(xc, lx, wc, lw, M, N, kb, e); break;
      }
      return qie_last_error();
    }
  }
  QIE_CHECK_ARG(e.ws && ((uintptr_t)e.ws % 16) == 0 && ws_bytes >= (int64_t)splits * M * N * 4);
  if (QIE_GEMM_PP && QIE_SPLITK_PP && M >= 128 && N >= 256 && kb >= 3 * kRowBytes) {
    // 256x256 ping-pong tiles (the text stream: M = B * S_txt ~ 432 -> 2 row tiles)
    const dim3 grid(((M + 255) / 256) * ((N + 255) / 256), splits);
    gemm_pp_kernel<EPI_PARTIAL, I8><<<grid, 512, 0, s>>>((const char*)x, ldx * eb, (const char*)w,
                                                        (int64_t)K * eb, M, N, kb, e);
  } else {
    const dim3 grid(((M + 127) / 128) * ((N + 127) / 128), splits);
    gemm_kernel<128, 128, 2, 2, EPI_PARTIAL, I8><<<grid, 256, 0, s>>>((const char*)x, ldx * eb,
                                                                     (const char*)w, (int64_t)K * eb,
                                                                     M, N, kb, e);
  }
  const int64_t nq = (int64_t)M * (N / 4);
  const int nb = (int)((nq + 255) / 256);
  switch (epi_kind) {
    case EPI_BIAS: splitk_reduce_kernel<EPI_BIAS, I8><<<nb, 256, 0, s>>>(e, M, N, splits); break;
    case EPI_GELU: splitk_reduce_kernel<EPI_GELU, I8><<<nb, 256, 0, s>>>(e, M, N, splits); break;
    case EPI_GATE_RES: splitk_reduce_kernel<EPI_GATE_RES, I8><<<nb, 256, 0, s>>>(e, M, N, splits); break;
    default: splitk_reduce_kernel<EPI_QKV, I8><<<nb, 256, 0, s>>>(e, M, N, splits); break;
  }
  return qie_last_error();
}

// QKV projection + QK RMSNorm + RoPE of one stream's rows: ONE gemm_pp launch (EPI_QKV_NR) of
// 256x256 tiles whenever K spans >= 3 tiles (also the text stream's 2 x 36 tiles: on
// the side stream its CU-time, not its latency, is what it costs), otherwise the QKV GEMM followed
// by qie_qk_norm_rope_bf16 on the same rows (the same arithmetic in two launches).
// 1: the image QKV + norm + RoPE on the persistent gemm_w4p (RoPE rows through registers); 0: on
// gemm_w4l. Same bits and the same time alone (0.712 vs 0.710 ms), but 1.5 % slower end to end
// (277.2 vs 272.6 ms per step, same box): the persistent grid holds every CU, so the text stream's
// QKV waits for all of it and the attention then waits for the text QKV
#ifndef QIE_NR_W4P
#define QIE_NR_W4P 0
#endif
template <bool I8>
int launch_qkv_norm_rope(const void* x, int64_t ldx, const void* w, int M, int K, EpiArgs e,
                         const void* nq, const void* nk, const float* cos_tab, const float* sin_tab,
                         float eps, float q_scale, hipStream_t s) {
  QIE_CHECK_ARG(nq && nk && cos_tab && sin_tab && e.head_dim == 128);
  const int N = 3 * e.heads * e.head_dim;
  const int eb = I8 ? 1 : 2;
  const int64_t big_tiles = (int64_t)((M + 255) / 256) * ((N + 255) / 256);
  // no condition on M: a row's arithmetic must not depend on the batch size (batched CFG ==
  // sequential, stream batch == serial); rows past M are clamped / skipped by the kernel
  const bool fused = QIE_GEMM_PP && e.heads % 2 == 0 &&
                     (int64_t)K * eb >= 3 * kRowBytes && ((int64_t)K * eb) % kRowBytes == 0 &&
                     ((ldx * eb) % 16) == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)w % 16) == 0 &&
                     ((uintptr_t)e.out % 16) == 0 && ((uintptr_t)nq % 16) == 0 && ((uintptr_t)nk % 16) == 0 &&
                     ((uintptr_t)cos_tab % 16) == 0 && ((uintptr_t)sin_tab % 16) == 0;
  if (fused) {
    QIE_CHECK_ARG(x && w && e.out && e.bias);
    e.nq = (const bf16_t*)nq;
    e.nk = (const bf16_t*)nk;
    e.rcos = cos_tab;
    e.rsin = sin_tab;
    e.eps = eps;
    e.qscale = q_scale;
    // all kernels compute every row bit for bit alike (same K order, same epilogue sums)
    if (QIE_GEMM_W4 == 4 && QIE_NR_W4P && M >= 256 && big_tiles >= 160) {
      if (g_cu_count == 0) {
        int dev = 0, cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cu <= 0)
          cu = 256;
        g_cu_count = cu;
      }
      const int grid = (int)std::min<int64_t>(big_tiles, g_cu_count);
      gemm_w4p_kernel<EPI_QKV_NR, I8><<<grid, 256, 0, s>>>((const char*)x, ldx * eb, (const char*)w,
                                                           (int64_t)K * eb, M, N, K * eb, e);
    } else if (QIE_GEMM_W4 >= 3 && M >= 256 && big_tiles >= 160)
      gemm_w4l_kernel<EPI_QKV_NR, I8><<<(int)big_tiles, 256, 0, s>>>((const char*)x, ldx * eb, (const char*)w,
                                                                    (int64_t)K * eb, M, N, K * eb, e);
    else
      gemm_pp_kernel<EPI_QKV_NR, I8><<<(int)big_tiles, 512, 0, s>>>((const char*)x, ldx * eb, (const char*)w,
                                                                   (int64_t)K * eb, M, N, K * eb, e);
    return qie_last_error();
  }
  const int rc = launch_gemm<EPI_QKV, I8>(x, ldx, w, K, M, N, K, e, s);
  if (rc) return rc;
  return qie_qk_norm_rope_bf16(e.out, e.batch, e.heads, e.head_dim, e.s_pad, e.seq_offset, e.rows_per_batch,
                               nq, nk, cos_tab, sin_tab, eps, q_scale, s);
}

// ---------------------------------------------------------------------------------------------
// Implicit-GEMM 3x3 / 1x1 convolution over NHWC bf16 activations (the VAE decoder's
// QwenImageCausalConv3d on one frame and its Resample Conv2d): output pixel p
// (row of the GEMM) x output channel (column), K = (tap, input channel) in [ky][kx][C] order,
// zero padded to a multiple of 64. The X tile is gathered per lane straight from the input image
// (one 16-byte chunk = 8 channels of one tap of one pixel per LDS-DMA lane): the shifted pixel of
// the tap, through an optional nearest-2x upsample (source pixel = upsampled pixel >> 1), or the
// zero chunk when the tap falls into the padding. No im2col buffer exists; W is [Cout][Kpad].
// Body, LDS layout and epilogues are gemm_kernel<128, 128, 2, 2>'s.
struct ConvArgs {
  const bf16_t* in;
  int H_in, W_in, C;    // input image (NHWC), C % 8 == 0
  int H_out, W_out;     // output image
  int mode;             // 0: same size (pad ks/2); 1: nearest-2x upsample folded into the gather;
                        // 2: stride 2 after ZeroPad2d((0, 1, 0, 1)) (the encoder's Resample)
  int ks;               // 3 or 1
};
__device__ __attribute__((aligned(16))) unsigned g_conv_zero[4];
// Tile choice, measured (tools/conv_bench.py, same-process A/B on the VAE shapes): with the
// branch-free gather, 128-pixel tiles at 2 workgroups per CU beat 256-pixel tiles at 1 per CU by
// 3-11 %, and a 3-stage LDS ring (two K tiles in flight) loses 2-4 % (and 40 % where it halves
// the workgroups per CU). Both remain build options.
#ifndef QIE_CONV_BIG_MIN  // workgroup count of 256-pixel tiles from which they replace 128-pixel ones
#define QIE_CONV_BIG_MIN (1 << 30)
#endif
#ifndef QIE_CONV_STAGES  // 2: double-buffered K tiles, drain each step; 3: two tiles in flight
#define QIE_CONV_STAGES 2
#endif

template <int EPI, int BM, int WM, int BN, int MODE>
__global__ void __launch_bounds__(WM * 2 * 64)
    conv_kernel(ConvArgs c, const char* __restrict__ W, int64_t ldw_b, int M, int N, int K_bytes, EpiArgs e) {
  using Op = MfmaOp<false>;
  constexpr int WN = 2, NWAVE = WM * WN;
  constexpr int WPC = BN / 8;  // W pieces (8 rows x 128 B) per K tile, spread over the waves
  constexpr int TM = BM / WM, TN = BN / WN, MT = TM / 16, NTL = TN / 16;
  constexpr int A_BYTES = BM * kRowBytes, W_BYTES = BN * kRowBytes, STAGE = A_BYTES + W_BYTES;
  constexpr int PX = BM / 8 / NWAVE;  // X pieces per lane per K tile
  constexpr int NS = QIE_CONV_STAGES;  // LDS stages: tile kt + NS - 1 is in flight while kt computes
  __shared__ __attribute__((aligned(16))) char smem_raw[NS * STAGE];
  char QIE_LDS* smem = (char QIE_LDS*)smem_raw;

  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  const int wgid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int first_m = (wgid / per_group) * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (wgid % per_group) % gsz;
  const int tn = (wgid % per_group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  // wave index made provably uniform: the LDS-DMA destination (M0) must be, or hipcc waterfalls
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave / WN, wn = wave % WN;
  const char* wg = W + (int64_t)n0 * ldw_b;
  const int n_valid = N - n0;

  // per X piece: output pixel (y, x) of its row, and the (tap, channel) of its chunk in the K tile
  int py[PX], pxx[PX], tap[PX], ci[PX];
#pragma unroll
  for (int i = 0; i < PX; ++i) {
    const int r = (wave + i * NWAVE) * 8 + (lane >> 3);
    const int p = min(m0 + r, M - 1);
    py[i] = p / c.W_out;
    pxx[i] = p - py[i] * c.W_out;
    const int k = swz_chunk(r, lane & 7) * 8;  // K index of the chunk in tile 0
    tap[i] = k / c.C;
    ci[i] = k - tap[i] * c.C;
  }
  const int ntap = c.ks * c.ks, pad = c.ks >> 1;
  const int hlim = MODE == 2 ? c.H_in : c.H_out, wlim = MODE == 2 ? c.W_in : c.W_out;
  const char* zero = (const char*)g_conv_zero;
  // branch-free gather: the chunk's source pixel for its tap, or the zero chunk
  auto stage_x = [&](char QIE_LDS* lds) {
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      const int t = tap[i];
      const int dy = (t * 11) >> 5, dx = t - 3 * dy;  // tap / 3, tap % 3 for tap < 9 (0, 0 for 1x1)
      int yy, xx;
      if constexpr (MODE == 2) {  // stride 2 after ZeroPad2d((0, 1, 0, 1))
        yy = 2 * py[i] + dy;
        xx = 2 * pxx[i] + dx;
      } else {
        yy = py[i] + dy - pad;
        xx = pxx[i] + dx - pad;
      }
      const bool ok = t < ntap && yy >= 0 && xx >= 0 && yy < hlim && xx < wlim;
      if constexpr (MODE == 1) {  // nearest-2x: the upsampled pixel's source
        yy >>= 1;
        xx >>= 1;
      }
      // 32-bit element offset (the host checks H_in * W_in * C < 2^31)
      const char* src = ok ? (const char*)c.in + 2u * (uint32_t)((yy * c.W_in + xx) * c.C + ci[i]) : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (QIE_LDS void*)(lds + (wave + i * NWAVE) * 1024), 16, 0, 0);
      // advance to the next K tile: 64 channels on, wrapping into the following taps
      ci[i] += 64;
      if (c.C >= 64) {
        const int wr = ci[i] >= c.C;
        ci[i] -= wr * c.C;
        tap[i] += wr;
      } else {
        const int q = ci[i] / c.C;
        ci[i] -= q * c.C;
        tap[i] += q;
      }
    }
  };

  typename Op::acc acc[MT][NTL];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j) acc[i][j] = typename Op::acc{0, 0, 0, 0};

  const int nk = K_bytes / kRowBytes;
  // W rows: piece q (rows 8q..8q+7) by wave q % NWAVE; BN = 96 leaves some waves one piece short
  auto stage_w = [&](int64_t koff, char QIE_LDS* lds) {
#pragma unroll
    for (int i = 0; i < (WPC + NWAVE - 1) / NWAVE; ++i) {
      const int blk = wave + i * NWAVE;
      if (WPC % NWAVE == 0 || blk < WPC) {
        const int r = blk * 8 + (lane >> 3);
        const int cc = swz_chunk(r, lane & 7);
        const int gr = r < n_valid ? r : n_valid - 1;
        __builtin_amdgcn_global_load_lds((const void*)(wg + (int64_t)gr * ldw_b + koff + (cc << 4)),
                                         (QIE_LDS void*)(lds + blk * 1024), 16, 0, 0);
      }
    }
  };
  // loads one K tile puts in flight per wave (vmcnt counts them): PX gather pieces + this wave's W
  const int nw_mine = WPC / NWAVE + (wave < WPC % NWAVE ? 1 : 0);
  auto wait_newest_in_flight = [&](int n) {  // vmcnt(n): all but this wave's n newest loads landed
    switch (n) {
      case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
      case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
      case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
      case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
  };
  stage_x(smem);
  stage_w(0, smem + A_BYTES);
  if constexpr (NS == 3) {
    if (nk > 1) {
      stage_x(smem + STAGE);
      stage_w(kRowBytes, smem + STAGE + A_BYTES);
      wait_newest_in_flight(PX + nw_mine);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const int fr = lane & 15;
  const int sw = (fr >> 1) & 7;
  const int a_row = wm * TM + fr;
  const int w_row = wn * TN + fr;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt % NS;
    const bool more = kt + NS - 1 < nk;
    if (more) {
      char QIE_LDS* nb = smem + ((kt + NS - 1) % NS) * STAGE;
#ifndef QIE_CONV_ABL  // timing ablation bits (tools only): 1 no X gather, 2 no W staging, 4 no MFMA
#define QIE_CONV_ABL 0
#endif
      if (!(QIE_CONV_ABL & 1)) stage_x(nb);
      if (!(QIE_CONV_ABL & 2)) stage_w((int64_t)(kt + NS - 1) * kRowBytes, nb + A_BYTES);
    }
    const char QIE_LDS* at = smem + cur * STAGE;
    const char QIE_LDS* wt = at + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < ((QIE_CONV_ABL & 4) ? 0 : 2); ++kk) {
      const int cofs = ((kk * 4 + (lane >> 4)) ^ sw) << 4;
      typename Op::frag wf[NTL], af[MT];
#pragma unroll
      for (int j = 0; j < NTL; ++j) wf[j] = *(const typename Op::frag QIE_LDS*)(wt + (w_row + j * 16) * kRowBytes + cofs);
#pragma unroll
      for (int i = 0; i < MT; ++i) af[i] = *(const typename Op::frag QIE_LDS*)(at + (a_row + i * 16) * kRowBytes + cofs);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j) acc[i][j] = Op::mma(wf[j], af[i], acc[i][j]);
    }
    // tile kt+1 must have landed: NS = 3 leaves tile kt+2's loads (issued above) in flight
    if (NS == 3 && more) wait_newest_in_flight(PX + nw_mine);
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#ifndef QIE_CONV_EPI_PRELOAD  // 0: epilogue4 per accumulator tile (bias / residual loads between stores)
#define QIE_CONV_EPI_PRELOAD 1
#endif
  if constexpr (!QIE_CONV_EPI_PRELOAD || (EPI != EPI_BIAS && EPI != EPI_RES)) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int m = m0 + wm * TM + i * 16 + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < NTL; ++j) {
        const int n = n0 + wn * TN + j * 16 + (lane >> 4) * 4;
        if (n >= N) continue;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r];
        epilogue4<EPI, false>(e, m, n, v);
      }
    }
  } else {
    // every operand of the wave's stores loaded first -- the bias of its NTL column tiles and, for
    // the ResidualBlock sum, the residual it overwrites -- in one round trip: loaded between the
    // stores, each would wait behind the previous store (possible alias), MT * NTL round trips
    u32x2_t bw[NTL], xw[MT][NTL];
#pragma unroll
    for (int j = 0; j < NTL; ++j) bw[j] = *(const u32x2_t*)(e.bias + min(n0 + wn * TN + j * 16 + (lane >> 4) * 4, N - 4));
    if constexpr (EPI == EPI_RES) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j) {
          const int m = min(m0 + wm * TM + i * 16 + fr, M - 1);
          const int n = min(n0 + wn * TN + j * 16 + (lane >> 4) * 4, N - 4);
          xw[i][j] = *(const u32x2_t*)((const bf16_t*)e.out + (int64_t)m * e.ldo + n);
        }
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int m = m0 + wm * TM + i * 16 + fr;
#pragma unroll
      for (int j = 0; j < NTL; ++j) {
        const int n = n0 + wn * TN + j * 16 + (lane >> 4) * 4;
        float v[4] = {acc[i][j][0] + lo_f(bw[j].x), acc[i][j][1] + hi_f(bw[j].x), acc[i][j][2] + lo_f(bw[j].y),
                      acc[i][j][3] + hi_f(bw[j].y)};
        rbf2(v[0], v[1]);
        rbf2(v[2], v[3]);
        if constexpr (EPI == EPI_RES) {
          v[0] += lo_f(xw[i][j].x);
          v[1] += hi_f(xw[i][j].x);
          v[2] += lo_f(xw[i][j].y);
          v[3] += hi_f(xw[i][j].y);
        }
        if (m < M && n < N)
          *(u32x2_t*)((bf16_t*)e.out + (int64_t)m * e.ldo + n) = u32x2_t{pack2(v[0], v[1]), pack2(v[2], v[3])};
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Halo-tiled 3x3 convolution (pad 1; MODE 0 same size, MODE 1 with the nearest-2x upsample folded
// in) for the VAE's big 3x3 convolutions. conv_kernel above gathers every tap's
// pixels from L2 again (each input byte fetched 9 times) and runs 2-stage K tiles drained each step
// (timing ablations: its gather alone is 35 % of the time, its MFMA skeleton tops out at 785 TF/s).
// Here a workgroup owns TH x 32 output pixels x NT output channels:
//   * the input halo -- (TH + 2) x 34 pixels (MODE 1: (TH / 2 + 2) x 18 source pixels) x 32
//     channels -- is staged once per 32-channel chunk by LDS-DMA into one of two halo slots (the
//     next chunk's halo lands while the current one is consumed) and serves all 9 taps;
//   * K runs chunk-major: step s = (chunk c, tap t), s = 9c + t, K bytes (t * C + 32c) * 2 of the
//     [Cout][ky][kx][C] weight rows; the step's NT x 32 weight slice streams through a 6-slot LDS
//     ring, 4 steps ahead;
//   * 4 waves (WPX along pixel rows x 4 / WPX along output channels), each 4 output rows x 32
//     columns (8 pixel blocks of 16) x 96 channels: 48 MFMA 16x16x32 per step against 8 + 6
//     fragment reads; the step's barrier sits halfway through its MFMAs and the next step's
//     fragments are read behind it, so one wave per SIMD keeps the matrix core fed;
//   * LDS rows are 64 B (one pixel / one weight row of 32 channels), the 16-byte column XOR-ed
//     with 2 * bit 2 of the row index: conflict-free for ds_read_b128 at any pixel shift.
// The weight layout, zero padding and epilogues are conv_kernel's; the fp32 sums run chunk-major,
// so the rounding order differs from conv_kernel's (not bitwise equal; see tests/test_gpu_vae.py).
#ifndef QIE_CONV_HALO  // 0: every convolution on conv_kernel
#define QIE_CONV_HALO 1
#endif
#ifndef QIE_CONV_HALO_MIN  // workgroups from which a convolution takes the halo kernel
#define QIE_CONV_HALO_MIN 256
#endif
#ifndef QIE_HALO_PD  // weight prefetch distance (steps); the ring has PD + 2 slots
#define QIE_HALO_PD 4
#endif
#ifndef QIE_CONV_NORM_FUSE  // 1: qie_conv2d_rmsnorm_bf16 folds the norm into the halo epilogue
#define QIE_CONV_NORM_FUSE 1
#endif
#ifndef QIE_HALO_PERSIST  // 1: one workgroup per CU walking its tiles; 0: one workgroup per tile
#define QIE_HALO_PERSIST 1
#endif
#ifndef QIE_HALO_ABL  // timing ablations (tools only): 1 no weight DMA, 2 no halo DMA, 4 no MFMA, 8 no fragment reads
#define QIE_HALO_ABL 0
#endif
constexpr int kConvPD = QIE_HALO_PD, kConvRing = QIE_HALO_PD + 2;

template <int WPX, int MODE, int RPW>  // RPW: output rows per wave (4, or 2 for small images)
struct HaloGeo {
  static constexpr int WN = 4 / WPX;
  static constexpr int TH = RPW * WPX, NT = 96 * WN;               // output tile TH x 32 x NT
  static constexpr int NB = 2 * RPW;                               // 16-pixel blocks per wave
  static constexpr int NF = 6 + NB;                                // fragment reads per step
  static constexpr int HW = MODE == 1 ? 18 : 34;                   // halo columns
  static constexpr int HR = MODE == 1 ? TH / 2 + 2 : TH + 2;       // halo rows
  static constexpr int HPIX = HR * HW;
  static constexpr int NH = ((HPIX + 15) / 16 + 3) / 4;            // halo pieces (1 KiB) per wave
  static constexpr int HBYTES = NH * 4 * 1024;
  static constexpr int NW = (NT / 16 + 3) / 4;                     // weight pieces per wave
  static constexpr int WBYTES = NW * 4 * 1024;
  static constexpr int LDS = 2 * HBYTES + kConvRing * WBYTES;
  static constexpr int SRPW = MODE == 1 ? RPW / 2 : RPW;           // halo rows per wave
  static constexpr int ROWB = SRPW * HW * 64;                      // halo bytes between waves
};

// s_waitcnt vmcnt(n) + s_barrier: all but the wave's n newest LDS-DMA pieces landed
template <int n>
__device__ __forceinline__ void vm_wait_barrier() {
  static_assert(n >= 0 && n <= 63, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(n) : "memory");
}
template <int EPI, int WPX, int MODE, int RPW>
__global__ void __launch_bounds__(256, 1)
    conv_halo_kernel(const bf16_t* __restrict__ X, int H_in, int W_in, int C, int H, int Wd,
                     const char* __restrict__ Wt, int ldw_b, int N, EpiArgs e) {
  using G = HaloGeo<WPX, MODE, RPW>;
  constexpr int NH = G::NH, NW = G::NW, PD = kConvPD, R = kConvRing, NB = G::NB;
  __shared__ __attribute__((aligned(16))) char smem_raw[G::LDS];
  char QIE_LDS* smem = (char QIE_LDS*)smem_raw;

  // persistent: this workgroup's tiles are blockIdx.x + i * gridDim.x (n fastest, then x, then
  // y); the step stream -- weights PD steps ahead, the next chunk's halo -- runs on across its
  // tiles, so a tile's first steps load while the previous tile's last steps and stores run
  const int tiles_x = (Wd + 31) / 32, tiles_y = (H + G::TH - 1) / G::TH, tiles_n = N / G::NT;
  const int ntiles = tiles_x * tiles_y * tiles_n;
  const int my_tiles = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int NC = C / 32, GC = my_tiles * NC;  // 32-channel chunks over all this workgroup's tiles
  auto tile_of = [&](int ti, int& x0, int& y0, int& n0) __attribute__((always_inline)) {
    const int id = (int)blockIdx.x + min(ti, my_tiles - 1) * (int)gridDim.x;
    const int tn = id % tiles_n, txy = id / tiles_n;
    x0 = (txy % tiles_x) * 32;
    y0 = (txy / tiles_x) * G::TH;
    n0 = tn * G::NT;
  };
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wp = wave / G::WN, wn = wave % G::WN;
  const int fr = lane & 15, g = lane >> 4;

  // halo pieces of this wave: pixel p = P * 16 + lane / 4, 16-byte column lane % 4; a tile past
  // the workgroup's last loads zeros (out of the buffer's range)
  const i32x4_t xr = pp_rsrc((const char*)X, H_in * W_in * C * 2);
  uint32_t hoff[NH];
  auto set_hoff = [&](int ti) __attribute__((always_inline)) {
    int x0, y0, n0;
    tile_of(ti, x0, y0, n0);
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      const int p = (wave * NH + k) * 16 + (lane >> 2);
      const int lc = (lane & 3) ^ (((p >> 2) & 1) << 1);
      const int hrow = p / G::HW, hcol = p - hrow * G::HW;
      const int sy = (MODE == 1 ? (y0 >> 1) : y0) - 1 + hrow, sx = (MODE == 1 ? (x0 >> 1) : x0) - 1 + hcol;
      const bool ok = ti < my_tiles && p < G::HPIX && sy >= 0 && sx >= 0 && sy < H_in && sx < W_in;
      hoff[k] = ok ? (uint32_t)(((sy * W_in + sx) * C + lc * 8) * 2) : 0x80000000u;
    }
  };
  // weight pieces: tile row n = P * 16 + lane / 4 (the tile's first row and the step's K bytes
  // go in the scalar offset)
  const i32x4_t wr = pp_rsrc(Wt, N * ldw_b);
  uint32_t woff[NW];
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const int n = (wave + 4 * k) * 16 + (lane >> 2);
    const int lc = (lane & 3) ^ (((n >> 2) & 1) << 1);
    woff[k] = n < G::NT ? (uint32_t)(n * ldw_b + lc * 16) : 0x80000000u;
  }
  char QIE_LDS* const wring = smem + 2 * G::HBYTES;
  auto dma_halo = [&](int gc, int c) __attribute__((always_inline)) {  // global chunk gc = chunk c of its tile
    char QIE_LDS* slot = smem + (gc & 1) * G::HBYTES;
#pragma unroll
    for (int k = 0; k < NH; ++k) w4l_dma<0>(xr, slot + (wave * NH + k) * 1024, hoff[k], __builtin_amdgcn_readfirstlane(c * 64));
  };
  // the weight stream: (tap wt, chunk wc) of tile wti, K bytes (wt * C + 32 wc) * 2
  int wt = 0, wc = 0, wti = 0, wn0;
  {
    int x0, y0;
    tile_of(0, x0, y0, wn0);
  }
  auto w_advance = [&]() __attribute__((always_inline)) {
    if (++wt == 9) {
      wt = 0;
      if (++wc == NC) {
        wc = 0;
        int x0, y0;
        tile_of(++wti, x0, y0, wn0);
      }
    }
  };
  auto dma_w = [&](int s) __attribute__((always_inline)) {  // into the slot of global step s
    char QIE_LDS* slot = wring + (s % R) * G::WBYTES;
    const int soff = __builtin_amdgcn_readfirstlane(wn0 * ldw_b + (wt * C + wc * 32) * 2);
#pragma unroll
    for (int k = 0; k < NW; ++k) w4l_dma<0>(wr, slot + (wave + 4 * k) * 1024, woff[k], soff);
    w_advance();
  };

  // per-lane pixel-fragment offsets for halo row k (counted from the wave's first row) and tap
  // column dx: the lane's halo column q and its swizzled 16-byte column. Bit 2 of the pixel index
  // row * HW + column (HW = 32 + 2 or 16 + 2) is bit 2 of (2 * row) mod 8 + q, so k mod 4 (with
  // the wave's row base) and dx select it
  uint32_t aoff[4][3];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int q = MODE == 1 ? ((fr + dx - 1) >> 1) + 1 : fr + dx;   // halo column within the block
      const int hrow2 = (2 * (G::SRPW * wp + k)) & 7;                 // (2 * absolute halo row) mod 8
      const int col = g ^ ((((hrow2 + q) >> 2) & 1) << 1);
      aoff[k][dx] = (uint32_t)(q * 64 + col * 16);
    }
  const uint32_t hbase = (uint32_t)(uintptr_t)smem + wp * G::ROWB;
  const uint32_t wlane = (uint32_t)(fr * 64 + ((g ^ (((fr >> 2) & 1) << 1)) << 4)) + wn * 96 * 64;
  const uint32_t wbase = (uint32_t)(uintptr_t)wring + wlane;

  using acc_t = f32x4_t;
  acc_t acc[NB][6];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[i][j] = acc_t{0, 0, 0, 0};

  // fragments of global step s (tap T of global chunk gc): pixel block b = 2r + h (output row r
  // of the wave, half h). Fragment i of the step (i < 6: weights j = i; then pixel blocks
  // b = i - 6) is one asm ds_read_b128 with its row offset in the offset field; the reads are
  // awaited by the lgkmcnt(0) that opens the step which uses them.
  auto read_frag = [&](auto t_t, auto i_t, int gc, int s, bf16x8_t (&af)[NB], bf16x8_t (&wf)[6]) __attribute__((always_inline)) {
    constexpr int T = decltype(t_t)::value, dy = T / 3, dx = T % 3, i = decltype(i_t)::value;
    if constexpr (i < 6) {
      const uint32_t pw = wbase + (s % R) * G::WBYTES;
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(wf[i]) : "v"(pw), "i"(i * 16 * 64));
    } else {
      constexpr int b = i - 6, r = b >> 1, h = b & 1;
      constexpr int k = MODE == 1 ? ((r + dy - 1) >> 1) + 1 : r + dy;
      constexpr int imm = (k * G::HW + (MODE == 1 ? 8 : 16) * h) * 64;
      const uint32_t pa = hbase + (gc & 1) * G::HBYTES + aoff[k & 3][dx];
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(af[b]) : "v"(pa), "i"(imm));
    }
  };
  auto read_frags = [&](auto t_t, int gc, int s, bf16x8_t (&af)[NB], bf16x8_t (&wf)[6]) __attribute__((always_inline)) {
    static_for<0, G::NF>([&](auto i_t) __attribute__((always_inline)) { read_frag(t_t, i_t, gc, s, af, wf); });
  };
  // the step's fragments have landed; every fragment register is redefined behind the wait, so no
  // copy of one can be scheduled above it
  auto frags_landed = [&](bf16x8_t (&af)[NB], bf16x8_t (&wf)[6]) __attribute__((always_inline)) {
    if constexpr (NB == 8)
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(af[0]), "+v"(af[1]), "+v"(af[2]), "+v"(af[3]), "+v"(af[4]), "+v"(af[5]), "+v"(af[6]),
                     "+v"(af[7]), "+v"(wf[0]), "+v"(wf[1]), "+v"(wf[2]), "+v"(wf[3]), "+v"(wf[4]), "+v"(wf[5])
                   :
                   : "memory");
    else
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(af[0]), "+v"(af[1]), "+v"(af[2]), "+v"(af[3]), "+v"(wf[0]), "+v"(wf[1]), "+v"(wf[2]),
                     "+v"(wf[3]), "+v"(wf[4]), "+v"(wf[5])
                   :
                   : "memory");
  };

  // one step: fragments landed; MFMAs of blocks 0-3 with the step's LDS-DMA pieces (the weights
  // of step s + PD, at tap 1 the next chunk's halo) one after every second MFMA; wait + barrier
  // for step s + 1; MFMAs of blocks 4-7 with step s + 1's 14 fragment reads one after each of
  // the first 14. Branch-free: past the workgroup's last step the weight pieces, a zero halo and
  // the fragment reads of "step S" still run, into slots no remaining step reads.
  auto step = [&](auto t_t, int gc, int c, int ti, bf16x8_t (&af)[NB], bf16x8_t (&wf)[6], bf16x8_t (&an)[NB],
                  bf16x8_t (&wn_)[6]) __attribute__((always_inline)) {
    constexpr int MF = 3 * NB;  // MFMAs per half step
    constexpr int T = decltype(t_t)::value;
    constexpr bool HALO = T == 1 && !(QIE_HALO_ABL & 2);
    constexpr int NP = ((QIE_HALO_ABL & 1) ? 0 : NW) + (HALO ? NH : 0);
    const int s = 9 * gc + T;
    frags_landed(af, wf);
    if constexpr (HALO) {  // the next chunk's halo (the next tile's first)
      if (c + 1 == NC) set_hoff(ti + 1);
    }
    char QIE_LDS* const wslot = wring + ((s + PD) % R) * G::WBYTES;
    const int wsoff = __builtin_amdgcn_readfirstlane(wn0 * ldw_b + (wt * C + wc * 32) * 2);
    const int gn = gc + 1, cn = c + 1 == NC ? 0 : c + 1;
    char QIE_LDS* const hslot = smem + (gn & 1) * G::HBYTES;
    const int hsoff = __builtin_amdgcn_readfirstlane(cn * 64);
    static_assert(NP <= MF, "one LDS-DMA piece per MFMA at most");
    static_for<0, MF>([&](auto i_t) __attribute__((always_inline)) {
      constexpr int i = decltype(i_t)::value;
      if (!(QIE_HALO_ABL & 4)) Mma4<false>::acc(acc[i / 6][i % 6], wf[i % 6], af[i / 6]);
      // piece k after MFMA 2k + 1 (measured: early beats spread to the end, 5 % at 512^2), or
      // after MFMA (k + 1) * MF / NP - 1 where the pieces outnumber the odd MFMAs
      static_for<0, NP>([&](auto k_t) __attribute__((always_inline)) {
        constexpr int k = decltype(k_t)::value;
        constexpr int at = 2 * NP <= MF ? 2 * k + 1 : (k + 1) * MF / NP - 1;
        if constexpr (at == i) {
          if constexpr (!(QIE_HALO_ABL & 1) && k < NW) w4l_dma<0>(wr, wslot + (wave + 4 * k) * 1024, woff[k], wsoff);
          else {
            constexpr int kh = (QIE_HALO_ABL & 1) ? k : k - NW;
            w4l_dma<0>(xr, hslot + (wave * NH + kh) * 1024, hoff[kh], hsoff);
          }
        }
      });
    });
    if (!(QIE_HALO_ABL & 1)) w_advance();
    // step s + 1's weights landed (PD - 1 later weight steps may stay in flight, plus the next
    // halo while it is younger than the awaited weights)
    if constexpr (QIE_HALO_ABL & 3) vm_wait_barrier<0>();
    else if constexpr (T >= 1 && T <= PD) vm_wait_barrier<(PD - 1) * NW + NH>();
    else vm_wait_barrier<(PD - 1) * NW>();
    static_for<0, MF>([&](auto i_t) __attribute__((always_inline)) {
      constexpr int i = decltype(i_t)::value;
      if (!(QIE_HALO_ABL & 4)) Mma4<false>::acc(acc[NB / 2 + i / 6][i % 6], wf[i % 6], af[NB / 2 + i / 6]);
      if constexpr (i < G::NF && !(QIE_HALO_ABL & 8))
        read_frag(std::integral_constant<int, (T + 1) % 9>{}, i_t, T == 8 ? gc + 1 : gc, s + 1, an, wn_);
    });
    if constexpr (QIE_HALO_ABL & 8) {
#pragma unroll
      for (int b = 0; b < NB; ++b) an[b] = af[b];
#pragma unroll
      for (int j = 0; j < 6; ++j) wn_[j] = wf[j];
    }
  };

  // a finished tile: bias (and the ResidualBlock residual, in place) loaded before any store,
  // then the accumulators restart at zero
  auto epilogue = [&](int x0, int y0, int n0) __attribute__((always_inline)) {
    // the asm MFMAs' results are read by VALU: drain the matrix pipe first (hipcc does not pad
    // inline-asm MFMAs), then redefine the accumulators so no read is hoisted above the wait
    asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int b = 0; b < NB; ++b)
      asm volatile("" : "+a"(acc[b][0]), "+a"(acc[b][1]), "+a"(acc[b][2]), "+a"(acc[b][3]), "+a"(acc[b][4]),
                   "+a"(acc[b][5]));
    const int nb = n0 + wn * 96 + g * 4;
    u32x2_t bw[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) bw[j] = *(const u32x2_t*)(e.bias + nb + j * 16);
    int mrow[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int y = y0 + RPW * wp + (b >> 1), x = x0 + 16 * (b & 1) + fr;
      mrow[b] = (y < H && x < Wd) ? y * Wd + x : -1;
    }
    // the block's 6 packed 4-channel pieces, widened to 16-byte stores: one v_permlane16_swap per
    // dword between tiles j and j + 1 leaves each lane 8 consecutive channels of its pixel
    // (g = 0: channels 0-7 of the 32, 1: 16-23, 2: 8-15, 3: 24-31)
    const int dl = (g & 1) * 16 + (g >> 1) * 8;
    auto store_row = [&](int b, const u32x2_t (&pk)[6]) __attribute__((always_inline)) {
#pragma unroll
      for (int jp = 0; jp < 3; ++jp) {
        const auto sx = __builtin_amdgcn_permlane16_swap(pk[2 * jp].x, pk[2 * jp + 1].x, false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(pk[2 * jp].y, pk[2 * jp + 1].y, false, false);
        if (mrow[b] >= 0)
          *(u32x4_t*)((bf16_t*)e.out + (int64_t)mrow[b] * e.ldo + n0 + wn * 96 + jp * 32 + dl) =
              u32x4_t{sx[0], sy[0], sx[1], sy[1]};
      }
    };
    if constexpr (EPI == EPI_NORM) {
      static_assert(G::WN == 1, "the norm needs every channel of a pixel in one wave");
      // QwenImageRMS_norm of vae.hip's rms_norm_kernel on the rounded conv output: the pixel's 96
      // channels sit in its 4 lanes g (24 each), the sum of squares meets by two xor shuffles
      u32x2_t gw[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) gw[j] = *(const u32x2_t*)(e.ngamma + nb + j * 16);
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        float v[6][4];
        u32x2_t pk[6];
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          v[j][0] = acc[b][j][0] + lo_f(bw[j].x);
          v[j][1] = acc[b][j][1] + hi_f(bw[j].x);
          v[j][2] = acc[b][j][2] + lo_f(bw[j].y);
          v[j][3] = acc[b][j][3] + hi_f(bw[j].y);
          rbf2(v[j][0], v[j][1]);
          rbf2(v[j][2], v[j][3]);
#pragma unroll
          for (int r = 0; r < 4; ++r) ss = __builtin_fmaf(v[j][r], v[j][r], ss);
        }
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        const float d = fmaxf(rbf(sqrtf(ss)), 1e-12f);
        // v / d correctly rounded from one reciprocal: q = v * (1/d), then one residual step
        // q + (v - q d) / d (exact for these normal-range operands, 3 VALU instead of ~10 per value)
        const float rd = __builtin_amdgcn_rcpf(d);
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          const float gg[4] = {lo_f(gw[j].x), hi_f(gw[j].x), lo_f(gw[j].y), hi_f(gw[j].y)};
          float u[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float q0 = v[j][r] * rd;
            const float q = __builtin_fmaf(__builtin_fmaf(-q0, d, v[j][r]), rd, q0);
            u[r] = rbf(rbf(rbf(q) * e.nscale) * gg[r]);
            if (e.nsilu) u[r] = u[r] * __builtin_amdgcn_rcpf(1.0f + __expf(-u[r]));
          }
          pk[j] = u32x2_t{pack2(u[0], u[1]), pack2(u[2], u[3])};
          acc[b][j] = acc_t{0, 0, 0, 0};
        }
        store_row(b, pk);
      }
      return;
    }
    u32x2_t xw[NB][6];
    if constexpr (EPI == EPI_RES) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int j = 0; j < 6; ++j)
          xw[b][j] = *(const u32x2_t*)((const bf16_t*)e.out + (int64_t)max(mrow[b], 0) * e.ldo + nb + j * 16);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      u32x2_t pk[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        float v[4] = {acc[b][j][0] + lo_f(bw[j].x), acc[b][j][1] + hi_f(bw[j].x), acc[b][j][2] + lo_f(bw[j].y),
                      acc[b][j][3] + hi_f(bw[j].y)};
        rbf2(v[0], v[1]);
        rbf2(v[2], v[3]);
        if constexpr (EPI == EPI_RES) {
          v[0] += lo_f(xw[b][j].x);
          v[1] += hi_f(xw[b][j].x);
          v[2] += lo_f(xw[b][j].y);
          v[3] += hi_f(xw[b][j].y);
        }
        pk[j] = u32x2_t{pack2(v[0], v[1]), pack2(v[2], v[3])};
        acc[b][j] = acc_t{0, 0, 0, 0};
      }
      store_row(b, pk);
    }
  };

  // prologue: tile 0's first halo chunk, weight steps 0 .. PD - 1, then step 0's fragments
  set_hoff(0);
  dma_halo(0, 0);
#pragma unroll
  for (int s = 0; s < PD; ++s) dma_w(s);
  vm_wait_barrier<(PD - 1) * NW>();
  bf16x8_t a0[NB], w0[6], a1[NB], w1[6];
  read_frags(std::integral_constant<int, 0>{}, 0, 0, a0, w0);
  int cx0, cy0, cn0, ti = 0, c = 0;
  tile_of(0, cx0, cy0, cn0);
  auto chunk_end = [&]() __attribute__((always_inline)) {
    if (c + 1 == NC) {
      epilogue(cx0, cy0, cn0);
      tile_of(++ti, cx0, cy0, cn0);
      c = 0;
    } else {
      ++c;
    }
  };
  // two chunks per trip (9 taps alternate the fragment sets, so the parity flips every chunk)
  for (int gc = 0;; gc += 2) {
    static_for<0, 9>([&](auto t_t) __attribute__((always_inline)) {
      if constexpr (decltype(t_t)::value % 2 == 0) step(t_t, gc, c, ti, a0, w0, a1, w1);
      else step(t_t, gc, c, ti, a1, w1, a0, w0);
    });
    chunk_end();
    if (gc + 1 >= GC) break;
    static_for<0, 9>([&](auto t_t) __attribute__((always_inline)) {
      if constexpr (decltype(t_t)::value % 2 == 0) step(t_t, gc + 1, c, ti, a1, w1, a0, w0);
      else step(t_t, gc + 1, c, ti, a0, w0, a1, w1);
    });
    chunk_end();
    if (gc + 2 >= GC) break;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // the trailing pieces land before exit
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

}  // namespace

// ============================================================================ C ABI
extern "C" int qie_linear_bf16(const void* x, int64_t ldx, const void* w, const void* bias, void* y,
                               int64_t ldy, int M, int N, int K, int act, qie_stream_t stream) {
  QIE_CHECK_ARG(ldy % 4 == 0 && ((uintptr_t)y % 8) == 0);
  EpiArgs e = make_epi(y, ldy, bias);
  if (act == QIE_ACT_GELU_TANH)
    return launch_gemm<EPI_GELU, false>(x, ldx, w, K, M, N, K, e, (hipStream_t)stream);
  QIE_CHECK_ARG(act == QIE_ACT_NONE);
  return launch_gemm<EPI_BIAS, false>(x, ldx, w, K, M, N, K, e, (hipStream_t)stream);
}

extern "C" int qie_linear_gated_residual_bf16(const void* x, int64_t ldx, const void* w,
                                              const void* bias, const void* gate,
                                              int64_t gate_bstride, int rows_per_batch, void* resid,
                                              int64_t ldr, int M, int N, int K,
                                              qie_stream_t stream) {
  QIE_CHECK_ARG(gate && rows_per_batch > 0 && ldr % 4 == 0 && gate_bstride % 4 == 0);
  EpiArgs e = make_epi(resid, ldr, bias);
  e.gate = (const bf16_t*)gate;
  e.gate_bstride = gate_bstride;
  e.rows_per_batch = rows_per_batch;
  return launch_gemm<EPI_GATE_RES, false>(x, ldx, w, K, M, N, K, e, (hipStream_t)stream);
}

static int qkv_args(EpiArgs& e, int M, int rows_per_batch, int seq_offset, int batch, int heads,
                    int head_dim, int s_pad) {
  QIE_CHECK_ARG(rows_per_batch > 0 && batch > 0 && heads > 0 && head_dim % 4 == 0);
  QIE_CHECK_ARG(M == rows_per_batch * batch && seq_offset >= 0 &&
                seq_offset + rows_per_batch <= s_pad);
  e.rows_per_batch = rows_per_batch;
  e.seq_offset = seq_offset;
  e.batch = batch;
  e.heads = heads;
  e.head_dim = head_dim;
  e.s_pad = s_pad;
  return QIE_OK;
}

extern "C" int qie_linear_qkv_bf16(const void* x, int64_t ldx, const void* w, const void* bias,
                                   void* qkv, int M, int K, int rows_per_batch, int seq_offset,
                                   int batch, int heads, int head_dim, int s_pad,
                                   qie_stream_t stream) {
  EpiArgs e = make_epi(qkv, 0, bias);
  int rc = qkv_args(e, M, rows_per_batch, seq_offset, batch, heads, head_dim, s_pad);
  if (rc) return rc;
  return launch_gemm<EPI_QKV, false>(x, ldx, w, K, M, 3 * heads * head_dim, K, e,
                                     (hipStream_t)stream);
}

extern "C" int qie_linear_i8(const void* xq, int64_t ldx, const float* sx, const void* wq,
                             const float* sw, const void* bias, void* y, int64_t ldy, int M, int N,
                             int K, int act, qie_stream_t stream) {
  QIE_CHECK_ARG(sx && sw && ldy % 4 == 0);
  EpiArgs e = make_epi(y, ldy, bias);
  e.sx = sx;
  e.sw = sw;
  if (act == QIE_ACT_GELU_TANH)
    return launch_gemm<EPI_GELU, true>(xq, ldx, wq, K, M, N, K, e, (hipStream_t)stream);
  QIE_CHECK_ARG(act == QIE_ACT_NONE);
  return launch_gemm<EPI_BIAS, true>(xq, ldx, wq, K, M, N, K, e, (hipStream_t)stream);
}

extern "C" int qie_linear_gated_residual_i8(const void* xq, int64_t ldx, const float* sx,
                                            const void* wq, const float* sw, const void* bias,
                                            const void* gate, int64_t gate_bstride,
                                            int rows_per_batch, void* resid, int64_t ldr, int M,
                                            int N, int K, qie_stream_t stream) {
  QIE_CHECK_ARG(sx && sw && gate && rows_per_batch > 0 && ldr % 4 == 0 && gate_bstride % 4 == 0);
  EpiArgs e = make_epi(resid, ldr, bias);
  e.sx = sx;
  e.sw = sw;
  e.gate = (const bf16_t*)gate;
  e.gate_bstride = gate_bstride;
  e.rows_per_batch = rows_per_batch;
  return launch_gemm<EPI_GATE_RES, true>(xq, ldx, wq, K, M, N, K, e, (hipStream_t)stream);
}

extern "C" int qie_linear_qkv_i8(const void* xq, int64_t ldx, const float* sx, const void* wq,
                                 const float* sw, const void* bias, void* qkv, int M, int K,
                                 int rows_per_batch, int seq_offset, int batch, int heads,
                                 int head_dim, int s_pad, qie_stream_t stream) {
  QIE_CHECK_ARG(sx && sw);
  EpiArgs e = make_epi(qkv, 0, bias);
  e.sx = sx;
  e.sw = sw;
  int rc = qkv_args(e, M, rows_per_batch, seq_offset, batch, heads, head_dim, s_pad);
  if (rc) return rc;
  return launch_gemm<EPI_QKV, true>(xq, ldx, wq, K, M, 3 * heads * head_dim, K, e,
                                    (hipStream_t)stream);
}

extern "C" int qie_linear_qkv_norm_rope_bf16(const void* x, int64_t ldx, const void* w, const void* bias,
                                             void* qkv, int M, int K, int rows_per_batch, int seq_offset,
                                             int batch, int heads, int head_dim, int s_pad, const void* wq,
                                             const void* wk, const float* cos_tab, const float* sin_tab,
                                             float eps, float q_scale, qie_stream_t stream) {
  EpiArgs e = make_epi(qkv, 0, bias);
  int rc = qkv_args(e, M, rows_per_batch, seq_offset, batch, heads, head_dim, s_pad);
  if (rc) return rc;
  return launch_qkv_norm_rope<false>(x, ldx, w, M, K, e, wq, wk, cos_tab, sin_tab, eps, q_scale,
                                     (hipStream_t)stream);
}

extern "C" int qie_linear_qkv_norm_rope_i8(const void* xq, int64_t ldx, const float* sx, const void* wq,
                                           const float* sw, const void* bias, void* qkv, int M, int K,
                                           int rows_per_batch, int seq_offset, int batch, int heads,
                                           int head_dim, int s_pad, const void* nq, const void* nk,
                                           const float* cos_tab, const float* sin_tab, float eps,
                                           float q_scale, qie_stream_t stream) {
  QIE_CHECK_ARG(sx && sw);
  EpiArgs e = make_epi(qkv, 0, bias);
  e.sx = sx;
  e.sw = sw;
  int rc = qkv_args(e, M, rows_per_batch, seq_offset, batch, heads, head_dim, s_pad);
  if (rc) return rc;
  return launch_qkv_norm_rope<true>(xq, ldx, wq, M, K, e, nq, nk, cos_tab, sin_tab, eps, q_scale,
                                    (hipStream_t)stream);
}

// ---------------------------------------------------------------------------- split-K C ABI
static int splitk_epi(const qie_epilogue_t* p, const void* bias, int M, int N, void* ws, EpiArgs& e) {
  QIE_CHECK_ARG(p && p->out);
  e = make_epi(p->out, p->ldo, bias);
  e.ws = ws;
  switch (p->kind) {
    case QIE_EPI_BIAS:
    case QIE_EPI_GELU:
      QIE_CHECK_ARG(p->ldo >= N && p->ldo % 4 == 0 && ((uintptr_t)p->out % 8) == 0);
      return QIE_OK;
    case QIE_EPI_GATED_RESIDUAL:
      QIE_CHECK_ARG(p->gate && p->rows_per_batch > 0 && p->ldo >= N && p->ldo % 4 == 0 &&
                    p->gate_bstride % 4 == 0);
      e.gate = (const bf16_t*)p->gate;
      e.gate_bstride = p->gate_bstride;
      e.rows_per_batch = p->rows_per_batch;
      return QIE_OK;
    case QIE_EPI_QKV:
      QIE_CHECK_ARG(N == 3 * p->heads * p->head_dim);
      return qkv_args(e, M, p->rows_per_batch, p->seq_offset, p->batch, p->heads, p->head_dim, p->s_pad);
    default:
      return QIE_ERR_INVALID;
  }
}

extern "C" int qie_linear_splitk_bf16(const void* x, int64_t ldx, const void* w, const void* bias,
                                      const qie_epilogue_t* epi, int M, int N, int K, int splits,
                                      void* workspace, int64_t workspace_bytes, qie_stream_t stream) {
  EpiArgs e;
  int rc = splitk_epi(epi, bias, M, N, workspace, e);
  if (rc) return rc;
  return launch_splitk<false>(x, ldx, w, M, N, K, splits, epi->kind, e, workspace_bytes,
                              (hipStream_t)stream);
}

extern "C" int qie_linear_splitk_i8(const void* xq, int64_t ldx, const float* sx, const void* wq,
                                    const float* sw, const void* bias, const qie_epilogue_t* epi,
                                    int M, int N, int K, int splits, void* workspace,
                                    int64_t workspace_bytes, qie_stream_t stream) {
  QIE_CHECK_ARG(sx && sw);
  EpiArgs e;
  int rc = splitk_epi(epi, bias, M, N, workspace, e);
  if (rc) return rc;
  e.sx = sx;
  e.sw = sw;
  return launch_splitk<true>(xq, ldx, wq, M, N, K, splits, epi->kind, e, workspace_bytes,
                             (hipStream_t)stream);
}

// ---------------------------------------------------------------------------- VAE convolutions
static int conv2d_impl(const void* x, int H_in, int W_in, int C, int mode, int ksize, const void* w, int64_t ldw,
                       const void* bias, const void* resid, void* y, int N, const void* ngamma, int nsilu,
                       qie_stream_t stream);

extern "C" int qie_conv2d_bf16(const void* x, int H_in, int W_in, int C, int mode, int ksize, const void* w,
                               int64_t ldw, const void* bias, const void* resid, void* y, int N,
                               qie_stream_t stream) {
  return conv2d_impl(x, H_in, W_in, C, mode, ksize, w, ldw, bias, resid, y, N, nullptr, 0, stream);
}

// conv + QwenImageRMS_norm (+ SiLU) of its output (the ResidualBlock's conv1 + norm2): one launch
// where the halo kernel holds every output channel of a pixel in one wave (N = 96), otherwise the
// conv and qie_vae_rms_norm_bf16 in place
extern "C" int qie_conv2d_rmsnorm_bf16(const void* x, int H_in, int W_in, int C, int mode, int ksize, const void* w,
                                       int64_t ldw, const void* bias, const void* gamma, int silu, void* y, int N,
                                       qie_stream_t stream) {
  QIE_CHECK_ARG(gamma && ((uintptr_t)gamma % 16) == 0);
  const int rc = conv2d_impl(x, H_in, W_in, C, mode, ksize, w, ldw, bias, nullptr, y, N, gamma, silu, stream);
  if (rc != QIE_ERR_UNSUPPORTED) return rc;
  const int rc2 = conv2d_impl(x, H_in, W_in, C, mode, ksize, w, ldw, bias, nullptr, y, N, nullptr, 0, stream);
  if (rc2) return rc2;
  const int64_t P = (int64_t)(mode == 1 ? 2 * H_in : mode == 2 ? H_in / 2 : H_in) *
                    (mode == 1 ? 2 * W_in : mode == 2 ? W_in / 2 : W_in);
  return qie_vae_rms_norm_bf16(y, gamma, y, P, N, silu, stream);
}

static int conv2d_impl(const void* x, int H_in, int W_in, int C, int mode, int ksize, const void* w, int64_t ldw,
                       const void* bias, const void* resid, void* y, int N, const void* ngamma, int nsilu,
                       qie_stream_t stream) {
  QIE_CHECK_ARG(x && w && bias && y && H_in > 0 && W_in > 0 && C > 0 && C % 8 == 0);
  QIE_CHECK_ARG(mode >= 0 && mode <= 2 && (ksize == 1 || ksize == 3) && N > 0 && N % 4 == 0);
  QIE_CHECK_ARG(mode != 2 || (ksize == 3 && H_in % 2 == 0 && W_in % 2 == 0));
  const int kreal = ksize * ksize * C;
  const int kpad = (kreal + 63) / 64 * 64;
  QIE_CHECK_ARG(ldw >= kpad && ldw % 8 == 0 && ((uintptr_t)w % 16) == 0 && ((uintptr_t)x % 16) == 0);
  const int H_out = mode == 1 ? 2 * H_in : mode == 2 ? H_in / 2 : H_in;
  const int W_out = mode == 1 ? 2 * W_in : mode == 2 ? W_in / 2 : W_in;
  ConvArgs c{(const bf16_t*)x, H_in, W_in, C, H_out, W_out, mode, ksize};
  const int64_t M64 = (int64_t)c.H_out * c.W_out;
  QIE_CHECK_ARG(M64 < (1ll << 31) && (int64_t)H_in * W_in * C < (1ll << 31));
  const int M = (int)M64;
  const hipStream_t s = (hipStream_t)stream;
  QIE_CHECK_ARG(!resid || resid == y);  // y = bf16(resid + bf16(acc + bias)), in place
  EpiArgs e = make_epi(y, N, bias);
  e.ngamma = (const bf16_t*)ngamma;
  e.nscale = sqrtf((float)N);
  e.nsilu = nsilu;
  const char* wc = (const char*)w;
#if QIE_CONV_HALO
  // halo-tiled kernel: 3x3, same size or upsampled, 32-channel chunks, 96 / 192-channel tiles,
  // enough tiles to fill the chip (smaller grids stay on conv_kernel's 128-pixel tiles)
  if (ksize == 3 && mode != 2 && C % 32 == 0 && (N == 96 || N % 192 == 0) && (int64_t)N * ldw * 2 < (1ll << 31)) {
    const int wpx = N == 96 ? 4 : 2, nt = N == 96 ? 96 : 192;
    auto tiles = [&](int rpw) {
      return (int64_t)((c.W_out + 31) / 32) * ((c.H_out + rpw * wpx - 1) / (rpw * wpx)) * (N / nt);
    };
    // 4 output rows per wave; 2 where that leaves too few tiles for the chip (128^2 x 384)
    const int rpw = tiles(4) >= QIE_CONV_HALO_MIN ? 4 : 2;
    const int64_t nwg = tiles(rpw);
    if (nwg >= QIE_CONV_HALO_MIN) {
      const bf16_t* xb = (const bf16_t*)x;
      if (g_cu_count == 0) {
        int dev = 0, cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cu <= 0)
          cu = 256;
        g_cu_count = cu;
      }
      const int grid = QIE_HALO_PERSIST ? (int)std::min<int64_t>(nwg, g_cu_count) : (int)nwg;
      auto k = [&](auto epi_t, auto wpx_t, auto mode_t) {
        constexpr int EP = decltype(epi_t)::value, WX = decltype(wpx_t)::value, MD = decltype(mode_t)::value;
        if (rpw == 4)
          conv_halo_kernel<EP, WX, MD, 4><<<grid, 256, 0, s>>>(xb, H_in, W_in, C, c.H_out, c.W_out, wc, (int)(ldw * 2), N, e);
        else
          conv_halo_kernel<EP, WX, MD, 2><<<grid, 256, 0, s>>>(xb, H_in, W_in, C, c.H_out, c.W_out, wc, (int)(ldw * 2), N, e);
      };
      auto by_mode = [&](auto epi_t, auto wpx_t) {
        if (mode == 1) k(epi_t, wpx_t, std::integral_constant<int, 1>{});
        else k(epi_t, wpx_t, std::integral_constant<int, 0>{});
      };
      auto by_wpx = [&](auto epi_t) {
        if (wpx == 4) by_mode(epi_t, std::integral_constant<int, 4>{});
        else by_mode(epi_t, std::integral_constant<int, 2>{});
      };
      if (ngamma) {
        if (wpx != 4 || !QIE_CONV_NORM_FUSE) return QIE_ERR_UNSUPPORTED;
        by_mode(std::integral_constant<int, EPI_NORM>{}, std::integral_constant<int, 4>{});
      } else if (resid) {
        by_wpx(std::integral_constant<int, EPI_RES>{});
      } else {
        by_wpx(std::integral_constant<int, EPI_BIAS>{});
      }
      return qie_last_error();
    }
  }
#endif
  // 128-pixel tiles (4 waves, 2 workgroups per CU; 256-pixel / 8-wave tiles from QIE_CONV_BIG_MIN
  // workgroups); 96-wide output tiles when N is a multiple of 96 but not of 128 (96, 192)
  if (ngamma) return QIE_ERR_UNSUPPORTED;  // the caller runs the conv, then the norm
  const bool n96 = N % 128 != 0 && N % 96 == 0;
  const int bn = n96 ? 96 : 128;
  const int tn = (N + bn - 1) / bn;
  const int64_t big = (int64_t)((M + 255) / 256) * tn;
  const int64_t kb = kpad * 2, lw = ldw * 2;
  auto go = [&](auto bm_t, auto wm_t, auto bn_t) {
    constexpr int BM = decltype(bm_t)::value, WMv = decltype(wm_t)::value, BNv = decltype(bn_t)::value;
    const int nwg = ((M + BM - 1) / BM) * ((N + BNv - 1) / BNv);
    auto k = [&](auto mode_t) {
      constexpr int MD = decltype(mode_t)::value;
      if (resid) conv_kernel<EPI_RES, BM, WMv, BNv, MD><<<nwg, WMv * 128, 0, s>>>(c, wc, lw, M, N, (int)kb, e);
      else conv_kernel<EPI_BIAS, BM, WMv, BNv, MD><<<nwg, WMv * 128, 0, s>>>(c, wc, lw, M, N, (int)kb, e);
    };
    if (mode == 1) k(std::integral_constant<int, 1>{});
    else if (mode == 2) k(std::integral_constant<int, 2>{});
    else k(std::integral_constant<int, 0>{});
  };
  using I96 = std::integral_constant<int, 96>;
  using I128 = std::integral_constant<int, 128>;
  using I256 = std::integral_constant<int, 256>;
  using I2 = std::integral_constant<int, 2>;
  using I4 = std::integral_constant<int, 4>;
  if (big >= QIE_CONV_BIG_MIN) {
    if (n96) go(I256{}, I4{}, I96{});
    else go(I256{}, I4{}, I128{});
  } else {
    if (n96) go(I128{}, I2{}, I96{});
    else go(I128{}, I2{}, I128{});
  }
  return qie_last_error();
}

// Raw fp32 product y[M][N] = x[M][K] . w[N][K]^T (row strides ldx / ldw elements, no bias, no
// rounding): the scores of the VAE mid-block attention (one head over H*W tokens).
extern "C" int qie_matmul_f32out_bf16(const void* x, int64_t ldx, const void* w, int64_t ldw, float* y,
                                      int M, int N, int K, qie_stream_t stream) {
  QIE_CHECK_ARG(x && w && y && M > 0 && N > 0 && K > 0 && K % 64 == 0 && N % 4 == 0);
  QIE_CHECK_ARG(ldx % 8 == 0 && ldw % 8 == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)w % 16) == 0);
  QIE_CHECK_ARG(((uintptr_t)y % 16) == 0);
  EpiArgs e = make_epi(y, N, nullptr);
  e.ws = y;
  const hipStream_t s = (hipStream_t)stream;
  const int kb = K * 2;
  if (QIE_GEMM_PP && M >= 256 && N >= 256 && kb >= 3 * kRowBytes) {
    const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
    gemm_pp_kernel<EPI_PARTIAL, false><<<tiles, 512, 0, s>>>((const char*)x, ldx * 2, (const char*)w, ldw * 2, M,
                                                             N, kb, e);
  } else {
    const int nwg = ((M + 127) / 128) * ((N + 127) / 128);
    gemm_kernel<128, 128, 2, 2, EPI_PARTIAL, false><<<nwg, 256, 0, s>>>((const char*)x, ldx * 2, (const char*)w,
                                                                        ldw * 2, M, N, kb, e);
  }
  return qie_last_error();
}

// Head-batched product for the prompt encoder's attention: for z < batch,
//   y_z = x_z . w_{z / group}^T   (x_z = x + z bsx, w_g = w + g bsw, y_z = y + z bsy; elements)
// out_f32 = 1: raw fp32 [M][N] (ldy == N) -- the scores; out_f32 = 0: bf16(x.w^T + bias) with
// row stride ldy -- P.V into each head's column slice.
extern "C" int qie_matmul_batched_bf16(const void* x, int64_t ldx, int64_t bsx, const void* w, int64_t ldw,
                                       int64_t bsw, int group, const void* bias, void* y, int64_t ldy, int64_t bsy,
                                       int M, int N, int K, int batch, int out_f32, qie_stream_t stream) {
  QIE_CHECK_ARG(x && w && y && M > 0 && N > 0 && K > 0 && K % 64 == 0 && N % 4 == 0 && batch > 0 && group > 0);
  QIE_CHECK_ARG(batch <= 65535 && ldx % 8 == 0 && ldw % 8 == 0 && bsx % 8 == 0 && bsw % 8 == 0);
  QIE_CHECK_ARG(((uintptr_t)x % 16) == 0 && ((uintptr_t)w % 16) == 0);
  EpiArgs e = make_epi(y, ldy, bias);
  e.bsx_b = bsx * 2;
  e.bsw_b = bsw * 2;
  e.group = group;
  const dim3 grid(((M + 127) / 128) * ((N + 127) / 128), 1, batch);
  const hipStream_t s = (hipStream_t)stream;
  if (out_f32) {
    QIE_CHECK_ARG(ldy == N && ((uintptr_t)y % 16) == 0 && bsy % 4 == 0);
    e.ws = y;
    e.bso_b = bsy * 4;
    gemm_kernel<128, 128, 2, 2, EPI_PARTIAL, false><<<grid, 256, 0, s>>>((const char*)x, ldx * 2, (const char*)w,
                                                                         ldw * 2, M, N, K * 2, e);
  } else {
    QIE_CHECK_ARG(bias && ldy % 4 == 0 && ((uintptr_t)y % 8) == 0 && bsy % 4 == 0);
    e.bso_b = bsy * 2;
    gemm_kernel<128, 128, 2, 2, EPI_BIAS, false><<<grid, 256, 0, s>>>((const char*)x, ldx * 2, (const char*)w,
                                                                      ldw * 2, M, N, K * 2, e);
  }
  return qie_last_error();
}
