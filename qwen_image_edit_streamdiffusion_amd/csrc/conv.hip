// Implicit-GEMM convolutions of the VAE (AutoencoderKLQwenImage on one frame):
// conv_kernel (per-tap gather, any shape) and conv_halo_kernel (halo-tiled 3x3, the big shapes),
// on the tile / epilogue pieces of gemm_common.h.
#include "gemm_common.h"

namespace {

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
// the workgroups per CU).

template <int EPI, int BM, int WM, int BN, int MODE>
__global__ void __launch_bounds__(WM * 2 * 64)
    conv_kernel(ConvArgs c, const char* __restrict__ W, int64_t ldw_b, int M, int N, int K_bytes, EpiArgs e) {
  using Op = MfmaOp<false>;
  constexpr int WN = 2, NWAVE = WM * WN;
  constexpr int WPC = BN / 8;  // W pieces (8 rows x 128 B) per K tile, spread over the waves
  constexpr int TM = BM / WM, TN = BN / WN, MT = TM / 16, NTL = TN / 16;
  constexpr int A_BYTES = BM * kRowBytes, W_BYTES = BN * kRowBytes, STAGE = A_BYTES + W_BYTES;
  constexpr int PX = BM / 8 / NWAVE;  // X pieces per lane per K tile
  constexpr int NS = 2;  // LDS stages: tile kt + NS - 1 is in flight while kt computes
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
  stage_x(smem);
  stage_w(0, smem + A_BYTES);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
      stage_x(nb);
      stage_w((int64_t)(kt + NS - 1) * kRowBytes, nb + A_BYTES);
    }
    const char QIE_LDS* at = smem + cur * STAGE;
    const char QIE_LDS* wt = at + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
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
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile kt+1 has landed
    __syncthreads();
  }
  if constexpr (EPI != EPI_BIAS && EPI != EPI_RES) {
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
constexpr int kConvHaloMin = 256;  // workgroups from which a convolution takes the halo kernel
constexpr int kConvPD = 4, kConvRing = kConvPD + 2;  // weight prefetch distance (steps), ring slots

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
    for (int k = 0; k < NH; ++k) lds_dma(xr, slot + (wave * NH + k) * 1024, hoff[k], __builtin_amdgcn_readfirstlane(c * 64));
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
    for (int k = 0; k < NW; ++k) lds_dma(wr, slot + (wave + 4 * k) * 1024, woff[k], soff);
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
    constexpr bool HALO = T == 1;
    constexpr int NP = NW + (HALO ? NH : 0);
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
      Mma4<false>::acc(acc[i / 6][i % 6], wf[i % 6], af[i / 6]);
      // piece k after MFMA 2k + 1 (measured: early beats spread to the end, 5 % at 512^2), or
      // after MFMA (k + 1) * MF / NP - 1 where the pieces outnumber the odd MFMAs
      static_for<0, NP>([&](auto k_t) __attribute__((always_inline)) {
        constexpr int k = decltype(k_t)::value;
        constexpr int at = 2 * NP <= MF ? 2 * k + 1 : (k + 1) * MF / NP - 1;
        if constexpr (at == i) {
          if constexpr (k < NW) lds_dma(wr, wslot + (wave + 4 * k) * 1024, woff[k], wsoff);
          else lds_dma(xr, hslot + (wave * NH + (k - NW)) * 1024, hoff[k - NW], hsoff);
        }
      });
    });
    w_advance();
    // step s + 1's weights landed (PD - 1 later weight steps may stay in flight, plus the next
    // halo while it is younger than the awaited weights)
    if constexpr (T >= 1 && T <= PD) vm_wait_barrier<(PD - 1) * NW + NH>();
    else vm_wait_barrier<(PD - 1) * NW>();
    static_for<0, MF>([&](auto i_t) __attribute__((always_inline)) {
      constexpr int i = decltype(i_t)::value;
      Mma4<false>::acc(acc[NB / 2 + i / 6][i % 6], wf[i % 6], af[NB / 2 + i / 6]);
      if constexpr (i < G::NF)
        read_frag(std::integral_constant<int, (T + 1) % 9>{}, i_t, T == 8 ? gc + 1 : gc, s + 1, an, wn_);
    });
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
        // v / d from one reciprocal: q = v * (1/d), then one residual step q + (v - q d) / d
        // (3 VALU instead of ~10 per value). Close to, not guaranteed equal to, the correctly
        // rounded quotient rms_norm_kernel computes, and the sum of squares runs in another order:
        // the fused result is within one bf16 ulp of the two-launch path, not bitwise equal to it
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

}  // namespace

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
  // halo-tiled kernel: 3x3, same size or upsampled, 32-channel chunks, 96 / 192-channel tiles,
  // enough tiles to fill the chip (smaller grids stay on conv_kernel's 128-pixel tiles)
  if (ksize == 3 && mode != 2 && C % 32 == 0 && (N == 96 || N % 192 == 0) && (int64_t)N * ldw * 2 < (1ll << 31)) {
    const int wpx = N == 96 ? 4 : 2, nt = N == 96 ? 96 : 192;
    auto tiles = [&](int rpw) {
      return (int64_t)((c.W_out + 31) / 32) * ((c.H_out + rpw * wpx - 1) / (rpw * wpx)) * (N / nt);
    };
    // 4 output rows per wave; 2 where that leaves too few tiles for the chip (128^2 x 384)
    const int rpw = tiles(4) >= kConvHaloMin ? 4 : 2;
    const int64_t nwg = tiles(rpw);
    if (nwg >= kConvHaloMin) {
      const bf16_t* xb = (const bf16_t*)x;
      const int grid = (int)std::min<int64_t>(nwg, cu_count());  // persistent: one workgroup per CU
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
        if (wpx != 4) return QIE_ERR_UNSUPPORTED;
        by_mode(std::integral_constant<int, EPI_NORM>{}, std::integral_constant<int, 4>{});
      } else if (resid) {
        by_wpx(std::integral_constant<int, EPI_RES>{});
      } else {
        by_wpx(std::integral_constant<int, EPI_BIAS>{});
      }
      return qie_last_error();
    }
  }
  // 128-pixel tiles (4 waves, 2 workgroups per CU); 96-wide output tiles when N is a multiple of
  // 96 but not of 128 (96, 192)
  if (ngamma) return QIE_ERR_UNSUPPORTED;  // the caller runs the conv, then the norm
  const bool n96 = N % 128 != 0 && N % 96 == 0;
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
  using I2 = std::integral_constant<int, 2>;
  if (n96) go(I128{}, I2{}, I96{});
  else go(I128{}, I2{}, I128{});
  return qie_last_error();
}

