// MFMA GEMM family for the DiT linears: y = epilogue(x[M,K] . W[N,K]^T + bias).
//
// Replaces the cuBLAS(Lt) GEMMs that diffusers' nn.Linear layers run inside
// QwenImageTransformerBlock [U] -- the 68.7 %
// of DiT FLOPs that are linear.
//
// Kernels, all gfx950-only (cdna_hip_programming.md §5):
//   gemm_w4p_kernel (big shapes: M, N >= 256, >= 160 tiles, aligned output) -- persistent, one
//     work-group per CU walking 256x256 tiles; 4 waves of 128x128 (256 AGPR accumulators), 64-wide
//     K tiles of whole 128-byte lines double buffered by LDS-DMA, the K-tile pipeline running
//     across tile boundaries. gemm_w4l_kernel is the same tile as one work-group per tile (the
//     image QKV + RMSNorm + RoPE launch, whose epilogue stages its RoPE rows in the LDS).
//   gemm_pp_kernel (the text stream's M = B * S_txt rows, split-K partials, fp32 products) -- the
//     256x256 tile as 8 waves in two ping-pong groups on the same K tiles.
//   gemm_kernel (everything else: small N or K, unaligned outputs) -- BMxBN tile, 2-stage:
//     * both operands are K-contiguous (activation rows, nn.Linear weight rows),
//       staged global -> LDS with 16-byte global_load_lds (LDS-DMA), one 128-byte
//       K-row per tile row (BK = 64 bf16 or 128 int8), double buffered;
//     * LDS image XOR-swizzled at 16-byte granularity, chunk' = chunk ^ ((row>>1)&7):
//       conflict-free for the ds_read_b128 lane groups; the swizzle is applied on the
//       per-lane GLOBAL address (LDS-DMA writes are lane-linear, rule 21);
// Common: MFMA 16x16x32 bf16 (or 16x16x64 i8) with the WEIGHT tile as the A operand and the
// activation tile as B, so each lane owns 4 consecutive output columns of one row; XCD-aware
// bijective block remap + grouped tile order so the 32 CUs of one XCD share L2-resident tiles.
#include "gemm_common.h"

namespace {

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

// Epilogue of a wave's 128 x (16 NT) accumulator block at output (mrow0, ncol0) -- rows
// mrow0 + 16i + (lane & 15), four consecutive columns per lane and tile. Every lane takes part
// in the permlane16 swaps, after which a lane holds 8 consecutive columns of one row; rows/columns
// past M/N are clamped for the loads and skipped for the store (N % 8 == 0, host-checked).
// EPI_QKV / EPI_QKV_NR with head_dim == 128 (host-checked for NR): the wave's 64 columns lie in
// one head of one of q/k/v, so the scatter address is computed once per wave and row. EPI_QKV_NR
// also applies the per-head RMSNorm (fp32 sum of squares over the head's 128 columns: the wave's
// 64 + its partner wave's 64, exchanged through `smem`) and the RoPE rotation of q and k, with
// the rounding points of qie_qk_norm_rope_bf16; it needs every wave of the workgroup here.
// column pairs (of 4) whose residual loads go out together in the 128 x 128 block's gated-residual
// epilogue: 32 VGPRs of residual per pair (2 pairs at once measured equal)
constexpr int kGateJB = 1;
template <int NT, int EPI, bool I8>
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
                t = __builtin_fmaf(hi, hi, __builtin_fmaf(lo, lo, t));
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
          if constexpr (NT == 8) {
            // the work-group's 256 RoPE rows (cos | sin, 512 B of fp32 each) staged into the free
            // LDS slots in one round trip by LDS-DMA (32 KiB pieces per wave), chunks XOR-swizzled by
            // the row so the 16 rows of a ds_read_b128 lane group hit 16 different banks; then
            // pass 2 reads them from LDS -- instead of 8 row-group round trips to L2 per wave, each
            // held behind the previous group's stores (possible alias with the qkv buffer)
            const int m0w = mrow0 & ~255, wave = threadIdx.x >> 6;
            // table row of tile row r: (m0w + r) mod rows_per_batch, the division done once per tile
            // (at most one wrap inside a tile when a batch has at least 256 rows)
            const int mb = m0w % e.rows_per_batch, rmax = M - 1 - m0w;
#pragma unroll 1
            for (int p = 0; p < 32; ++p) {
              const int P = wave * 32 + p, r = 2 * P + (lane >> 5), q = lane & 31;
              const int t = mb + min(r, rmax);
              const int sl = e.rows_per_batch >= 256 ? (t >= e.rows_per_batch ? t - e.rows_per_batch : t)
                                                     : t % e.rows_per_batch;
              const float* src = (q < 16 ? e.rcos : e.rsin) + (int64_t)sl * 64 + (((q & 15) ^ (r & 15)) << 2);
              __builtin_amdgcn_global_load_lds((const void*)src, (QIE_LDS void*)(smem + P * 1024), 16, 0, 0);
            }
            u32x4_t wwv[4];
#pragma unroll
            for (int jp = 0; jp < 4; ++jp) wwv[jp] = *(const u32x4_t*)(nw + jp * 32 + dl);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            const int rl0 = (mrow0 & 255) + fr;  // the lane's row in the work-group tile, row group 0
            // row by row (its scatter address and 1/rms once), the row's four 32-column pairs
            // inside; the two bf16 roundings of the norm on both halves of a complex pair at once
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const int m = mrow0 + i * 16 + fr, rl = rl0 + i * 16;
              bf16_t* rp = row_ptr(min(m, M - 1));
              const float ssi = ss[i];
#pragma unroll
              for (int jp = 0; jp < 4; ++jp) {
                const int d0 = jp * 32 + dl;
                const uint32_t wv[4] = {wwv[jp].x, wwv[jp].y, wwv[jp].z, wwv[jp].w};
                const char QIE_LDS* rrow = smem + rl * 512 + (((d0 >> 3) ^ (rl & 15)) << 4);
                const f32x4_t cs = *(const f32x4_t QIE_LDS*)rrow;
                const f32x4_t sn = *(const f32x4_t QIE_LDS*)(rrow + 256);
                const u32x4_t v = cols8(i, jp);
                const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
                uint32_t o[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                  float x0 = lo_f(w4[k]) * ssi, x1 = hi_f(w4[k]) * ssi;
                  rbf2(x0, x1);
                  x0 *= lo_f(wv[k]);
                  x1 *= hi_f(wv[k]);
                  rbf2(x0, x1);
                  o[k] = pack2(__builtin_fmaf(x0, cs[k], -(x1 * sn[k])) * osc, __builtin_fmaf(x0, sn[k], x1 * cs[k]) * osc);
                }
                if (m < M) *(u32x4_t*)(rp + jp * 32) = u32x4_t{o[0], o[1], o[2], o[3]};
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
              const u32x4_t v = cols8(i, jp);
              const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
              uint32_t o[4];
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                float x0 = lo_f(w4[k]) * ss[i], x1 = hi_f(w4[k]) * ss[i];
                rbf2(x0, x1);
                x0 *= lo_f(wv[k]);
                x1 *= hi_f(wv[k]);
                rbf2(x0, x1);
                o[k] = pack2(__builtin_fmaf(x0, cs[k], -(x1 * sn[k])) * osc, __builtin_fmaf(x0, sn[k], x1 * cs[k]) * osc);
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
  if constexpr (EPI == EPI_GATE_RES && NT == 8) {
    // the 128 x 128 block of the 4-wave kernels, rows in one batch (wave-uniform): per column pair
    // the residual loads of all 8 row groups are issued together, ahead of that pair's stores --
    // 4 round trips per block; in store order every 16-byte chunk would be one (x is updated in
    // place, so hipcc keeps each load behind the stores before it). Same arithmetic as below.
    const int b0 = min(mrow0, M - 1) / e.rows_per_batch;
    if (b0 == min(mrow0 + 127, M - 1) / e.rows_per_batch) {
#pragma unroll
      for (int jq = 0; jq < 4; jq += kGateJB) {
        u32x4_t gv[kGateJB], xv[kGateJB][8];
#pragma unroll
        for (int jj = 0; jj < kGateJB; ++jj) {
          const int n = min(ncol0 + (jq + jj) * 32 + (g & 1) * 16 + (g >> 1) * 8, N - 8);
          gv[jj] = *(const u32x4_t*)(e.gate + (int64_t)b0 * e.gate_bstride + n);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int mc = min(mrow0 + i * 16 + fr, M - 1);
            xv[jj][i] = *(const u32x4_t*)((const bf16_t*)e.out + (int64_t)mc * e.ldo + n);
          }
        }
#pragma unroll
        for (int jj = 0; jj < kGateJB; ++jj) {
          const int jp = jq + jj;
          const int n = ncol0 + jp * 32 + (g & 1) * 16 + (g >> 1) * 8;
          const uint32_t gg[4] = {gv[jj].x, gv[jj].y, gv[jj].z, gv[jj].w};
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int m = mrow0 + i * 16 + fr;
            u32x2_t a = epi_pre_c<EPI, I8, NT>(cols, i, 2 * jp, acc[i][2 * jp]);
            u32x2_t b = epi_pre_c<EPI, I8, NT>(cols, i, 2 * jp + 1, acc[i][2 * jp + 1]);
            const auto sx = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
            const auto sy = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
            const uint32_t vv[4] = {sx[0], sy[0], sx[1], sy[1]};
            const uint32_t xx[4] = {xv[jj][i].x, xv[jj][i].y, xv[jj][i].z, xv[jj][i].w};
            uint32_t o[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
              o[k] = pack2(lo_f(xx[k]) + rbf(lo_f(gg[k]) * lo_f(vv[k])), hi_f(xx[k]) + rbf(hi_f(gg[k]) * hi_f(vv[k])));
            if (m < M && n < N) *(u32x4_t*)((bf16_t*)e.out + (int64_t)m * e.ldo + n) = u32x4_t{o[0], o[1], o[2], o[3]};
          }
        }
      }
      return;
    }
  }
  if constexpr (EPI != EPI_QKV_NR && EPI != EPI_PARTIAL) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mrow0 + i * 16 + fr;
#pragma unroll
      for (int jp = 0; jp < NT / 2; ++jp) {
        const int nb = ncol0 + jp * 32;
        u32x2_t a = epi_pre_c<EPI, I8, NT>(cols, i, 2 * jp, acc[i][2 * jp]);
        u32x2_t b = epi_pre_c<EPI, I8, NT>(cols, i, 2 * jp + 1, acc[i][2 * jp + 1]);
        const auto sx = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
        const int n = nb + (g & 1) * 16 + (g >> 1) * 8;
        if (m < M && n < N) epi_store8<EPI>(e, m, n, u32x4_t{sx[0], sy[0], sx[1], sy[1]});
      }
    }
  }
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
constexpr int kPPTile = 256 * kRowBytes;  // one operand of one K tile, 32 KiB
constexpr int kPPX = 2;                   // X slots (three, all 160 KiB of LDS, measured no faster); W has 2
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
    lds_dma(xr, xslot(kt) + (wave + i * NWAVE) * 1024, xo[i], kt * kRowBytes);
  };
  auto dmaW = [&](int kt, int i) {
    lds_dma(wr, wslot(kt) + (wave + i * NWAVE) * 1024, wo[i], kt * kRowBytes);
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
    static_assert(n == -1 || n == 0 || n == 4, "vmcnt");
    if constexpr (n == -1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (n == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  // section (MH, KS) of tile kt. DX: stage X(kt+1) pieces 2 KS, 2 KS + 1 (sections MH = 0);
  // DW: stage W(kt+2) pieces 2 KS, 2 KS + 1 (sections MH = 1); VM: vmcnt of section (1, 1)
  auto section = [&](auto mh_t, auto ks_t, auto init_t, auto dx_t, auto dw_t, auto vm_t, int kt) {
    constexpr int MH = decltype(mh_t)::value, KS = decltype(ks_t)::value;
    constexpr bool INIT = decltype(init_t)::value && KS == 0;
    constexpr bool DX = decltype(dx_t)::value, DW = decltype(dw_t)::value;
    if constexpr (MH == 0) {
#pragma unroll
      for (int j = 0; j < NT; ++j) wf[KS][j] = ldW(kt, j, KS);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = ldX(kt, 4 * MH + i, KS);
    if constexpr (DX) {
      dmaX(kt + kPPXA, 2 * KS);
      dmaX(kt + kPPXA, 2 * KS + 1);
    }
    if constexpr (DW) {
      dmaW(kt + 2, 2 * KS);
      dmaW(kt + 2, 2 * KS + 1);
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
  // tile kt: X(kt+1) if DX, W(kt+2) if DW; section (1,1) waits for tile kt+1
  auto tile = [&](auto init_t, auto dx_t, auto dw_t, auto vm_t, int kt) {
    section(I0{}, I0{}, init_t, dx_t, F{}, VNone{}, kt);
    section(I0{}, I1{}, init_t, dx_t, F{}, VNone{}, kt);
    section(I1{}, I0{}, init_t, F{}, dw_t, VNone{}, kt);
    section(I1{}, I1{}, init_t, F{}, dw_t, vm_t, kt);
  };

  // prologue: W(0), X(0), W(1); wait for tile 0; group 1 one barrier behind. Steady tile k stages
  // X(k + 1) and W(k + 2) and waits for everything but its own W pieces (vmcnt 4) -> tile k+1
  // has landed.
  using VS = std::integral_constant<int, 4>;
#pragma unroll
  for (int i = 0; i < PPO; ++i) dmaW(0, i);
#pragma unroll
  for (int i = 0; i < PPO; ++i) dmaX(0, i);
#pragma unroll
  for (int i = 0; i < PPO; ++i) dmaW(1, i);
  ld_end(VS{});
  if (wm == 1) asm volatile("s_barrier" ::: "memory");

  tile(T{}, T{}, T{}, VS{}, 0);
  int kt = 1;
  for (; kt < nk - 2; ++kt) tile(F{}, T{}, T{}, VS{}, kt);
  tile(F{}, T{}, F{}, V0{}, kt);                            // nk-2: stages X(nk-1), waits for it
  tile(F{}, F{}, F{}, VNone{}, kt + 1);                     // nk-1
  if (wm == 0) asm volatile("s_barrier" ::: "memory");  // every wave passes the same barrier count

  ring_epilogue<NT, EPI, I8>(acc, e, M, N, m0 + wm * 128, n0 + wn * NT * 16, lane, smem);
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
//     tile kt -- then the 16 pieces of tile kt+2 (X, then W) into tile kt's slot, spread evenly
//     over the MFMAs up to the next barrier;
//   phase B (k-step 1, set 1): the rest of those pieces; at MFMA 64 + QB2
//     `vmcnt(16); s_barrier` -- this wave's pieces of tile kt+1 (issued a whole tile earlier)
//     have landed, and after the barrier everyone's -- then set 0 of tile kt+1, one per MFMA.
// Two barriers per 128 MFMAs. The reads are inline asm with hand-counted lgkmcnt waits (hipcc
// counts neither them nor the DMA pieces, so it adds no waits of its own in the loop).
constexpr int kW4lQB1 = 24;  // MFMA of phase A after which the slot-free barrier sits
constexpr int kW4lQB2 = 48;  // MFMA of phase B after which the tile-landed barrier sits (then 16 reads)

// piece k (0..15) goes after MFMA g_k = QB1 + 1 + k * span / 16 of the tile's 128
__host__ __device__ constexpr int w4l_piece(int g) {
  constexpr int first = kW4lQB1 + 1, span = 64 + kW4lQB2 - 1 - first;
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
  static_assert(kW4lQB1 >= 16, "phase A placement");
  static_assert(kW4lQB2 + 16 <= 64, "phase B reads");
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
    lds_dma(xr, smem + (kt & 1) * kSlot + (wave + p * NWAVE) * 1024, xo[p], kt * kRowBytes);
  };
  auto dmaW = [&](int kt, int p) {
    lds_dma(wr, smem + (kt & 1) * kSlot + kPPTile + (wave + p * NWAVE) * 1024, wo[p], kt * kRowBytes);
  };

  // piece k of the schedule: X pieces 0..7, then W pieces 0..7
  auto dma_piece_k = [&](int kt, int k) {
    if (k < PPO) dmaX(kt, k);
    else dmaW(kt, k - PPO);
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
    __builtin_amdgcn_s_setprio(decltype(p_t)::value);
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
      if constexpr (q == kW4lQB1) {
        prio(I0{});
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        prio(I3{});
      }
      if constexpr (DMA) {
        constexpr int k = w4l_piece(q);
        if constexpr (k >= 0) dma_piece_k(kt + 2, k);
      }
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
      if constexpr (DMA) {
        constexpr int k = w4l_piece(64 + q);
        if constexpr (k >= 0) dma_piece_k(kt + 2, k);
      }
      if constexpr (NEXT && q == kW4lQB2) {
        prio(I0{});
        if constexpr (DMA) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        prio(I3{});
      }
      if constexpr (NEXT && q >= kW4lQB2 && q < kW4lQB2 + 16) rd(I0{}, std::integral_constant<int, q - kW4lQB2>{});
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
// past the buffer descriptor's range and read as zeros (never stored). The QKV + norm + RoPE
// epilogue stays on gemm_w4l: it stages its RoPE rows in the LDS, which here holds the next tile
// (and a persistent grid holding every CU makes the text stream's QKV, and so the attention, wait).

template <int EPI, bool I8>
__global__ void __launch_bounds__(256, 1)
    gemm_w4p_kernel(const char* __restrict__ X, int64_t ldx_b, const char* __restrict__ W, int64_t ldw_b,
                    int M, int N, int K_bytes, EpiArgs e) {
  static_assert(EPI != EPI_PARTIAL && EPI != EPI_QKV_NR, "w4p epilogues");
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
    const int GROUP = tiles_n <= 16 ? 4 : 8;
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
      lds_dma(tr.xr, smem + sl * kSlot + (wave + k * NWAVE) * 1024, xo[k], dkt * kRowBytes);
    else
      lds_dma(tr.wr, smem + sl * kSlot + kPPTile + (wave + (k - PPO) * NWAVE) * 1024, wo[k - PPO],
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
    __builtin_amdgcn_s_setprio(decltype(p_t)::value);
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
      if constexpr (q == kW4lQB1) {
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
      if constexpr (NEXT && q == kW4lQB2) {
        prio(I0{});
        if constexpr (DMA) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        prio(I3{});
      }
      if constexpr (NEXT && q >= kW4lQB2 && q < kW4lQB2 + 16) rd(I0{}, std::integral_constant<int, q - kW4lQB2>{});
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
    ktile(F{}, T{}, T{}, (g + kt + 1) & 1, nxt, 1);  // nk-1: its K tile 1, reads its set 0
    ring_epilogue<8, EPI, I8>(acc, e, M, N, cur.m0 + wm * 128, cur.n0 + wn * 128, lane, smem);
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
  if constexpr (EPI != EPI_QKV_NR) {
    if (wide && M >= 256 && N >= 256 && big_tiles >= 160 && kb >= 3 * kRowBytes) {  // nk >= 3
      const int grid = (int)std::min<int64_t>(big_tiles, cu_count());
      gemm_w4p_kernel<EPI, I8><<<grid, 256, 0, s>>>((const char*)x, ldx_b, (const char*)w, ldw_b, M, N, kb, e);
      return qie_last_error();
    }
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
    if (wide && N >= 256 && kb >= 3 * kRowBytes) {
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
  if (M >= 128 && N >= 256 && kb >= 3 * kRowBytes) {
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

// QKV projection + QK RMSNorm + RoPE of one stream's rows: ONE launch (EPI_QKV_NR; gemm_w4l for the
// image stream's shapes, gemm_pp otherwise) of 256x256 tiles whenever K spans >= 3 tiles (also the
// text stream's 2 x 36 tiles: on
// the side stream its CU-time, not its latency, is what it costs), otherwise the QKV GEMM followed
// by qie_qk_norm_rope_bf16 on the same rows (the same arithmetic in two launches).
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
  const bool fused = e.heads % 2 == 0 &&
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
    if (M >= 256 && big_tiles >= 160)
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
  if (M >= 256 && N >= 256 && kb >= 3 * kRowBytes) {
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

