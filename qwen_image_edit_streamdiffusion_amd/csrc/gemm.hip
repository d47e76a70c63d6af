// MFMA GEMM family for the DiT linears: y = epilogue(x[M,K] . W[N,K]^T + bias).
//
// Replaces the cuBLAS(Lt) GEMMs that diffusers' nn.Linear layers run inside
// QwenImageTransformerBlock [U] -- the 68.7 %
// of DiT FLOPs that are linear.
//
// Design (gfx950, cdna_hip_programming.md §5):
//   * both operands are K-contiguous (activation rows, nn.Linear weight rows),
//     staged global -> LDS with 16-byte global_load_lds (LDS-DMA), one 128-byte
//     K-row per tile row (BK = 64 bf16 or 128 int8), double buffered;
//   * LDS image XOR-swizzled at 16-byte granularity, chunk' = chunk ^ ((row>>1)&7):
//     the 16-lane ds_read_b128 groups of the MFMA operand reads are conflict-free;
//     the swizzle is applied on the per-lane GLOBAL address (LDS-DMA writes are
//     lane-linear, rule 21);
//   * MFMA 16x16x32 bf16 (or 16x16x64 i8) with the WEIGHT tile as the A operand
//     and the activation tile as B, so each lane ends up owning 4 consecutive
//     output columns of one row -> 8-byte epilogue stores;
//   * XCD-aware bijective block remap + grouped tile order so the 32 CUs of one
//     XCD work on a compact block of tiles (L2 reuse).
#include "qie_common.h"

namespace {

constexpr int kRowBytes = 128;  // one LDS tile row = 64 bf16 or 128 int8 of K

enum Epi { EPI_BIAS = 0, EPI_GELU = 1, EPI_GATE_RES = 2, EPI_QKV = 3 };

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

template <int BM, int BN, int WM, int WN, int EPI, bool I8>
__global__ void __launch_bounds__(WM* WN * 64)
    gemm_kernel(const char* __restrict__ X, int64_t ldx_b, const char* __restrict__ W, int64_t ldw_b,
                int M, int N, int K_bytes, EpiArgs e) {
  using Op = MfmaOp<I8>;
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

  const char* xg = X + (int64_t)m0 * ldx_b;
  const char* wg = W + (int64_t)n0 * ldw_b;
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
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc_val<I8>(acc[i][j], r, 1.0f);
      epilogue4<EPI, I8>(e, m, n, v);
    }
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

EpiArgs make_epi(void* out, int64_t ldo, const void* bias) {
  EpiArgs e{};
  e.out = out;
  e.ldo = ldo;
  e.bias = (const bf16_t*)bias;
  e.rows_per_batch = 1;
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
