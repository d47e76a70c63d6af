// Joint non-causal flash attention forward, head_dim 128, bf16 in/out.
//
// Replaces the SDPA call of diffusers' QwenDoubleStreamAttnProcessor2_0 [U]:
// softmax(Q K^T / sqrt(128)) V over the joint
// [image; text] sequence (8408 tokens at 1024^2), 31 % of DiT FLOPs.
//
// Layout: qkv = [3][B][H][s_pad][128] bf16 (written by the fused QKV GEMM
// epilogue).  The joint sequence is ordered [image tokens; text tokens; pad], so
// the valid keys of batch row b are the prefix [0, kv_len[b]) -- key order does
// not change softmax, RoPE was applied per token beforehand.
//
// Structure (gfx950): one workgroup = 8 waves = 256 query rows of one (b, h), 32 rows per
// wave, 64-key tiles:
//   S^T = K . Q^T      (mfma 32x32x16 bf16, K rows by ds_read_b128 from an XOR-swizzled LDS
//                       image, Q^T held in registers)
//   -> each lane owns one query row: online softmax (running max / sum, exp2, lazy rescale T13)
//      is lane-local except for one max exchange with the partner half-wave
//   O^T += V^T . P^T   (the S^T accumulator registers ARE the P^T operand,
//                       cdna_hip_programming.md §3 "accumulator as operand"; V^T fragments by
//                       ds_read_b64_tr_b16 with the matching permuted key order)
// scheduled as a two-group ping-pong (attn_pp_kernel below). Workgroups of one (b, h) share an
// XCD so its K/V stream from L2; the last query block of every (b, h) can be split over the
// key range into fp32 partials + a combine kernel (qie_attention_fwd_split_bf16).
#include <type_traits>

#include "qie_common.h"

namespace {

constexpr int kDh = 128;
constexpr int kQB = 256;   // query rows per workgroup
constexpr int kKB = 64;    // keys per tile
constexpr int kTileBytes = kKB * kDh * 2;  // 16 KiB
constexpr float kRescaleThr = 8.0f;        // lazy-rescale threshold, log2 units

struct AttnArgs {
  const bf16_t* qkv;
  bf16_t* out_img;
  bf16_t* out_txt;
  int B, H, s_pad, s_img, txt_rows, qblocks;
  float c;  // scale * log2(e)
  int split;  // key ranges of the last query block (0: none)
  float* ws;  // split partials: O [B*H][split][256][128] fp32, then (m, l) [B*H][split][256][2]
  QieBatchI kv_len;
};

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// =============================================================================================
// attn_pp_kernel. Waves 0-3 (group 0) and 4-7 (group 1) put one
// wave of each group on every SIMD. Group 1 runs one phase behind group 0, so while one wave
// of a SIMD is in its MFMA phase the other is in its VALU phase:
//   M-phase t : S(t) = K(t) Q^T (16 MFMA) then O += V(t-1)^T P(t-1)^T (16 MFMA), operands
//               streamed from LDS five MFMAs ahead, at raised issue priority;
//   V-phase t : masking, online softmax of S(t) -> P(t) (bf16), lazy O rescale, and the
//               LDS-DMA of K(t+2) / V(t+1).
// The MFMAs are asm volatile (their order and the LDS reads between them stay as written) and
// empty register fences on S / O / P pin every softmax instruction inside its V-phase (hipcc
// would otherwise hoist it between MFMAs, where the unpadded MFMA -> VALU hazard bites). K and
// V live in 4-slot LDS rings filled by buffer_load...lds: V-phase t issues K(t+3) / V(t+2) and
// ends with vmcnt(pieces just issued), so every tile has landed two phases before its first
// read and the M-phase ends with a bare barrier; one barrier per phase.
constexpr int kRing = 4;  // a power of two: slots are indexed t & (kRing - 1), tile indices are never negative
#ifndef QIE_ATTN_MPRIO  // issue priority of a wave in its MFMA phase
#define QIE_ATTN_MPRIO 2
#endif
#ifndef QIE_ATTN_VPRIO  // ... and in its softmax phase
#define QIE_ATTN_VPRIO 0
#endif

// Raw buffer descriptor (base, stride 0, num_records, dword3 0x00020000) in SGPRs.
__device__ __forceinline__ i32x4_t attn_rsrc(const bf16_t* base, int bytes) {
  const uint64_t p = (uint64_t)base;
  return i32x4_t{__builtin_amdgcn_readfirstlane((int)(uint32_t)p),
                 __builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32)),
                 __builtin_amdgcn_readfirstlane(bytes), 0x00020000};
}
// One 1-KiB LDS-DMA piece (buffer_load_dwordx4 ... lds) as inline asm: hipcc does not track it,
// so it inserts no conservative vmcnt(0) before LDS reads it cannot prove disjoint from the
// DMA target (the loop's own counted waits cover it). M0 is declared clobbered.
__device__ __forceinline__ void attn_dma(const i32x4_t& r, const char QIE_LDS* dst, uint32_t voff, int soff) {
  const int lds = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)dst);
  asm volatile(
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %1, %3 offen lds"
      :
      : "v"(voff), "s"(r), "s"(lds), "s"(soff)
      : "memory", "m0");
}
__device__ __forceinline__ void mma32(f32x16_t& c, const bf16x8_t& a, const bf16x8_t& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mma32_z(f32x16_t& c, const bf16x8_t& a, const bf16x8_t& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(a), "v"(b));
}
// first MFMA of a chain with a separate C operand (D = A.B + C0)
__device__ __forceinline__ void mma32_c(f32x16_t& c, const bf16x8_t& a, const bf16x8_t& b, const f32x16_t& c0) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %3" : "=&v"(c) : "v"(a), "v"(b), "v"(c0));
}
template <typename T>
__device__ __forceinline__ void rfence(T& x) {
  asm volatile("" : "+v"(x));
}

struct PPState {
  f32x16_t s[2];
  f32x16_t negm;  // PRE: splat(-m_run), the C operand of each tile's first QK^T MFMA
  f32x16_t o[4];
  bf16x8_t pf[4];
  bf16x8_t qf[8];
  float m_run, l_run;
};

// PRE: Q was written pre-multiplied by scale * log2(e) (the QKV epilogue folds it in before its
// single bf16 rounding), so S^T holds log2-unit logits. Each tile's QK^T chain then starts from
// C = -m_run and its accumulator is already the exponent: the softmax drops one v_fma_f32 per
// score (32 per lane and tile, ~1/5 of the phase's VALU issue). The lazy rescale subtracts the
// max growth from S in its (rare) branch; the first tile of a range always takes it.
template <bool PRE>
__global__ void __launch_bounds__(512) attn_pp_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * kRing * kTileBytes];  // K ring, V ring
  char QIE_LDS* smem = (char QIE_LDS*)smem_raw;

  // blocks [0, nfull): whole query blocks (XCD-grouped per (b, h)); then, if split, the last
  // query block of every (b, h) as `split` key ranges -- dispatched last, filling the final round
  const int qbf = a.split ? a.qblocks - 1 : a.qblocks;
  const int nfull = qbf * a.H * a.B;
  int qb, bh, chunk = -1;
  if ((int)blockIdx.x < nfull) {
    const int wgid = xcd_remap(blockIdx.x, nfull);
    qb = wgid % qbf;
    bh = wgid / qbf;
  } else {
    const int j = blockIdx.x - nfull;
    bh = j / a.split;
    chunk = j - bh * a.split;
    qb = a.qblocks - 1;
  }
  const int h = bh % a.H, b = bh / a.H;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;
  const int hf = lane >> 5;
  const int ql = lane & 31;
  const int64_t plane = (int64_t)a.s_pad * kDh;
  const bf16_t* Qp = a.qkv + ((int64_t)(0 * a.B + b) * a.H + h) * plane;
  const bf16_t* Kp = a.qkv + ((int64_t)(1 * a.B + b) * a.H + h) * plane;
  const bf16_t* Vp = a.qkv + ((int64_t)(2 * a.B + b) * a.H + h) * plane;
  const int kv_len = a.kv_len.v[b];
  const int ntot = (kv_len + kKB - 1) / kKB;
  // key tiles [t0, ntiles) of this work-group
  const int t0 = chunk < 0 ? 0 : chunk * ntot / a.split;
  const int ntiles = chunk < 0 ? ntot : (chunk + 1) * ntot / a.split;

  PPState st;
  const int q_row = qb * kQB + wave * 32 + ql;
  {
    const bf16_t* qr = Qp + (int64_t)q_row * kDh + 8 * hf;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) st.qf[ks] = *(const bf16x8_t*)(qr + 16 * ks);
  }

  // ---- LDS-DMA: wave w fills rows 4(w + 8p) .. +3 of a tile (p = 0, 1) for K and for V; the
  // per-lane source chunk carries the XOR swizzle (LDS-DMA writes are lane-linear)
  const auto kr = attn_rsrc(Kp, a.s_pad * kDh * 2);
  const auto vr = attn_rsrc(Vp, a.s_pad * kDh * 2);
  uint32_t ko[2], vo[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int row = (wave + 8 * p) * 4 + (lane >> 4), c = lane & 15;
    ko[p] = row * 256 + ((c ^ (row & 15)) << 4);
    vo[p] = row * 256 + ((c ^ ((row & 3) << 2)) << 4);
  }
  auto dmaK = [&](int t) {
    char QIE_LDS* base = smem + (t & (kRing - 1)) * kTileBytes;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      attn_dma(kr, base + (wave + 8 * p) * 1024, ko[p], t * kTileBytes);
    }
  };
  auto dmaV = [&](int t) {
    char QIE_LDS* base = smem + (kRing + (t & (kRing - 1))) * kTileBytes;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      attn_dma(vr, base + (wave + 8 * p) * 1024, vo[p], t * kTileBytes);
    }
  };

  // per-lane LDS read offsets (K: chunk ^ (row & 15); V: transposed 4x16 reads, chunk ^ ((row & 3) << 2))
  const int ksw = lane & 15;
  const int tri = lane & 15;
  const int tr_row = tri >> 2;
  const int tr_sw = tr_row << 2;
  const int tr_g1 = (lane >> 4) & 1;
  const int tr_cb = 8 * (tri & 1);

  // A operand of MFMA i of an M-phase: i < 16 -> K fragment (cb = i>>3, ks = i&7) of tile tk;
  // i >= 16 -> V^T fragment (ks = (i-16)>>2, db = (i-16)&3) of tile tv
  auto opA = [&](int i, int tk, int tv) -> bf16x8_t {
    if (i < 16) {
      const int cb = i >> 3, ks = i & 7;
      const char QIE_LDS* krow = smem + (tk & (kRing - 1)) * kTileBytes + (cb * 32 + ql) * 256;
      return *(const bf16x8_t QIE_LDS*)(krow + (((2 * ks + hf) ^ ksw) << 4));
    }
    const int j = i - 16, ks = j >> 2, db = j & 3;
    const char QIE_LDS* vb = smem + (kRing + (tv & (kRing - 1))) * kTileBytes;
    const int r0 = 16 * ks + 4 * hf + tr_row;
    const int chunk = (4 * db + 2 * tr_g1 + ((tri & 3) >> 1)) ^ tr_sw;
    const char QIE_LDS* p0 = vb + r0 * 256 + (chunk << 4) + tr_cb;
    const s16x4_t va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4_t QIE_LDS*)p0);
    const s16x4_t vb2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4_t QIE_LDS*)(p0 + 8 * 256));
    return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(va, vb2, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto mfma_i = [&](int i, const bf16x8_t& A) {
    if (i < 16) {
      const int cb = i >> 3, ks = i & 7;
      if (ks == 0) {
        if constexpr (PRE) mma32_c(st.s[cb], A, st.qf[0], st.negm);
        else mma32_z(st.s[cb], A, st.qf[0]);
      }
      else mma32(st.s[cb], A, st.qf[ks]);
    } else {
      const int j = i - 16;
      mma32(st.o[j & 3], A, st.pf[j >> 2]);
    }
  };
  // M-phase over MFMAs [i0, i1): operands prefetched PF MFMAs ahead
  constexpr int PF = 5;  // operand prefetch distance in MFMAs (3: -0.7 %, 7: -0.3 %)
  bf16x8_t A[8];
  auto mphase = [&](auto i0_t, auto i1_t, int tk, int tv) {
    constexpr int i0 = decltype(i0_t)::value, i1 = decltype(i1_t)::value;
    // the MFMA wave outranks its SIMD partner (in its softmax phase) for issue: otherwise the
    // older wave group wins arbitration and starves the younger group's MFMA phase
    __builtin_amdgcn_s_setprio(QIE_ATTN_MPRIO);
#pragma unroll
    for (int i = i0; i < i0 + PF && i < i1; ++i) A[i & 7] = opA(i, tk, tv);
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      if (i + PF < i1) A[(i + PF) & 7] = opA(i + PF, tk, tv);
      mfma_i(i, A[i & 7]);
    }
    __builtin_amdgcn_s_setprio(QIE_ATTN_VPRIO);
  };
  // V-phase: softmax of S(t) into P(t), DMA of later tiles; ends with the phase barrier
  auto vphase = [&](int t) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) rfence(st.s[cb]);
#pragma unroll
    for (int db = 0; db < 4; ++db) rfence(st.o[db]);
    int pieces = 0;
    if (t + 3 < ntiles) { dmaK(t + 3); pieces += 2; }
    if (t + 2 < ntiles) { dmaV(t + 2); pieces += 2; }
    const int kv0 = t * kKB;
    if (kv0 + kKB > kv_len) {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kv = kv0 + cb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf;
          if (kv >= kv_len) st.s[cb][r] = -INFINITY;
        }
    }
    const float c = a.c;
    auto row_max = [&]() -> float {
      float m0 = fmaxf(st.s[0][0], st.s[0][1]), m1 = fmaxf(st.s[0][2], st.s[0][3]);
#pragma unroll
      for (int r = 4; r < 16; r += 2) { m0 = fmaxf(m0, st.s[0][r]); m1 = fmaxf(m1, st.s[0][r + 1]); }
#pragma unroll
      for (int r = 0; r < 16; r += 2) { m0 = fmaxf(m0, st.s[1][r]); m1 = fmaxf(m1, st.s[1][r + 1]); }
      const float mh = fmaxf(m0, m1);
      // max with the partner half-wave (lane l <-> l ^ 32) without an LDS round trip
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mh), __float_as_uint(mh), false, false);
      return fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    };
    float ps0 = 0.f, ps1 = 0.f;
    auto exp_tile = [&]() {  // P = exp2(S), row sums (two interleaved chains), bf16 P^T fragments
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const float p0 = __builtin_amdgcn_exp2f(st.s[cb][r]);
          const float p1 = __builtin_amdgcn_exp2f(st.s[cb][r + 1]);
          ps0 += p0;
          ps1 += p1;
          st.pf[cb * 2 + (r >> 3)][r & 7] = (__bf16)p0;
          st.pf[cb * 2 + (r >> 3)][(r & 7) + 1] = (__bf16)p1;
        }
    };
    if constexpr (PRE) {
      // S already holds s*c - m_run (log2 units); tile t0 always rescales (it sets m_run)
      const float mx = row_max();
      if (__any(t == t0 || mx > kRescaleThr)) {
        const float d = t == t0 ? mx : fmaxf(mx, 0.f);  // growth of the running max
        const float alpha = __builtin_amdgcn_exp2f(-d);
        st.m_run += d;
        st.l_run *= alpha;
#pragma unroll
        for (int db = 0; db < 4; ++db) st.o[db] *= alpha;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) st.s[cb] -= d;
#pragma unroll
        for (int r = 0; r < 16; ++r) st.negm[r] = -st.m_run;
      }
      exp_tile();
    } else {
    const float mx = row_max();
    if (__any((mx - st.m_run) * c > kRescaleThr)) {
      const float m_new = fmaxf(st.m_run, mx);
      const float alpha = __builtin_amdgcn_exp2f((st.m_run - m_new) * c);
      st.m_run = m_new;
      st.l_run *= alpha;
#pragma unroll
      for (int db = 0; db < 4; ++db) st.o[db] *= alpha;
    }
    const float mc = st.m_run * c;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const float p0 = __builtin_amdgcn_exp2f(__builtin_fmaf(st.s[cb][r], c, -mc));
        const float p1 = __builtin_amdgcn_exp2f(__builtin_fmaf(st.s[cb][r + 1], c, -mc));
        ps0 += p0;
        ps1 += p1;
        st.pf[cb * 2 + (r >> 3)][r & 7] = (__bf16)p0;
        st.pf[cb * 2 + (r >> 3)][(r & 7) + 1] = (__bf16)p1;
      }
    }
    st.l_run += ps0 + ps1;
#pragma unroll
    for (int k = 0; k < 4; ++k) rfence(st.pf[k]);
    rfence(st.l_run);  // keep the row-sum adds in this phase (hipcc sinks them into the M-phase)
    rfence(st.m_run);
    if constexpr (PRE) rfence(st.negm);
#pragma unroll
    for (int db = 0; db < 4; ++db) rfence(st.o[db]);
    if (pieces == 4) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    else if (pieces == 2) asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  };
  using I0 = std::integral_constant<int, 0>;
  using I16 = std::integral_constant<int, 16>;
  using I32 = std::integral_constant<int, 32>;

  const int q_loc = wave * 32 + ql;  // row within the query block
  if (t0 >= ntiles) {                // empty key range (fewer tiles than ranges): neutral partial
    float* po = a.ws + (((int64_t)bh * a.split + chunk) * kQB + q_loc) * kDh;
    float* pml = a.ws + (int64_t)a.B * a.H * a.split * kQB * kDh;
#pragma unroll
    for (int k = 0; k < 16; ++k) *(f32x4_t*)(po + 8 * k + 4 * hf) = f32x4_t{0, 0, 0, 0};
    if (hf == 0) *(f32x2_t*)(pml + (((int64_t)bh * a.split + chunk) * kQB + q_loc) * 2) = f32x2_t{-INFINITY, 0.f};
    return;
  }
  // ---- prologue: K(t0..t0+2), V(t0), V(t0+1) resident; group 1 waits one phase
  dmaK(t0);
  if (t0 + 1 < ntiles) dmaK(t0 + 1);
  dmaV(t0);
  if (t0 + 2 < ntiles) dmaK(t0 + 2);
  if (t0 + 1 < ntiles) dmaV(t0 + 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the asm DMA pieces
  __builtin_amdgcn_s_waitcnt(0);                     // Q fragments (hipcc-tracked)
  asm volatile("s_barrier" ::: "memory");
  if (grp == 1) asm volatile("s_barrier" ::: "memory");
#pragma unroll
  for (int db = 0; db < 4; ++db) st.o[db] = f32x16_t{};
  st.m_run = PRE ? 0.f : -INFINITY;  // PRE: finite (it is the MFMA's C); tile t0 sets it
  st.l_run = 0.f;
  if constexpr (PRE) st.negm = f32x16_t{};

  // no vmcnt at the M-end: the V-end wait covers every tile two phases before its first read
  auto mend = [&]() { asm volatile("s_barrier" ::: "memory"); };
  mphase(I0{}, I16{}, t0, t0);  // S(t0)
  mend();
  vphase(t0);
  for (int t = t0 + 1; t < ntiles; ++t) {
    mphase(I0{}, I32{}, t, t - 1);  // S(t), O += V(t-1) P(t-1)
    mend();
    vphase(t);
  }
  mphase(I16{}, I32{}, t0, ntiles - 1);  // O += V(T-1) P(T-1)
  if (grp == 0) asm volatile("s_barrier" ::: "memory");
  // MFMA D -> VALU read hazard before the epilogue reads O (asm MFMAs are not padded by hipcc)
  asm volatile("s_nop 15\n\ts_nop 7" : "+v"(st.o[0]), "+v"(st.o[1]), "+v"(st.o[2]), "+v"(st.o[3]));
  const float l_tot = st.l_run + __shfl_xor(st.l_run, 32, 64);
  if (chunk >= 0) {  // fp32 partial: unnormalised O (d = 32db + 8g + 4hf + 0..3), row max, row sum
    float* po = a.ws + (((int64_t)bh * a.split + chunk) * kQB + q_loc) * kDh;
    float* pml = a.ws + (int64_t)a.B * a.H * a.split * kQB * kDh;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *(f32x4_t*)(po + 32 * db + 8 * g + 4 * hf) =
            f32x4_t{st.o[db][4 * g], st.o[db][4 * g + 1], st.o[db][4 * g + 2], st.o[db][4 * g + 3]};
    if (hf == 0) *(f32x2_t*)(pml + (((int64_t)bh * a.split + chunk) * kQB + q_loc) * 2) = f32x2_t{st.m_run, l_tot};
    return;
  }
  const float inv = 1.0f / l_tot;
  const int s = q_row;
  bf16_t* dst = nullptr;
  if (s < a.s_img) {
    dst = a.out_img + ((int64_t)b * a.s_img + s) * (a.H * kDh) + h * kDh;
  } else if (s < a.s_img + a.txt_rows) {
    dst = a.out_txt + ((int64_t)b * a.txt_rows + (s - a.s_img)) * (a.H * kDh) + h * kDh;
  }
  if (dst) {
    // lane (ql, hf) holds d = 32db + 8g + 4hf + 0..3; one permlane32 swap per dword of the group
    // pair (g, g+1) gives each lane 8 consecutive d (16-byte stores, T21)
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g = 0; g < 4; g += 2) {
        u32x2_t w0 = {pack2(st.o[db][4 * g] * inv, st.o[db][4 * g + 1] * inv),
                      pack2(st.o[db][4 * g + 2] * inv, st.o[db][4 * g + 3] * inv)};
        u32x2_t w1 = {pack2(st.o[db][4 * g + 4] * inv, st.o[db][4 * g + 5] * inv),
                      pack2(st.o[db][4 * g + 6] * inv, st.o[db][4 * g + 7] * inv)};
        const auto sx = __builtin_amdgcn_permlane32_swap(w0.x, w1.x, false, false);
        const auto sy = __builtin_amdgcn_permlane32_swap(w0.y, w1.y, false, false);
        *(u32x4_t*)(dst + 32 * db + 8 * g + 8 * hf) = u32x4_t{sx[0], sy[0], sx[1], sy[1]};
      }
  }
}

// Merges the `split` partials of the last query block: O = sum_c w_c O_c / sum_c w_c l_c with
// w_c = exp2((m_c - max_c m_c) * c). One wave per (b, h, row), two d values per lane.
__global__ void __launch_bounds__(256) attn_combine_kernel(AttnArgs a) {
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wid >= a.B * a.H * kQB) return;
  const int bh = wid / kQB, r = wid - bh * kQB;
  const int h = bh % a.H, b = bh / a.H;
  const int s = (a.qblocks - 1) * kQB + r;
  bf16_t* dst = nullptr;
  if (s < a.s_img) dst = a.out_img + ((int64_t)b * a.s_img + s) * (a.H * kDh) + h * kDh;
  else if (s < a.s_img + a.txt_rows)
    dst = a.out_txt + ((int64_t)b * a.txt_rows + (s - a.s_img)) * (a.H * kDh) + h * kDh;
  if (!dst) return;
  const float* pml = a.ws + (int64_t)a.B * a.H * a.split * kQB * kDh;
  float mx = -INFINITY;
  for (int c = 0; c < a.split; ++c) mx = fmaxf(mx, pml[(((int64_t)bh * a.split + c) * kQB + r) * 2]);
  float l = 0.f, o0 = 0.f, o1 = 0.f;
  for (int c = 0; c < a.split; ++c) {
    const int64_t pi = ((int64_t)bh * a.split + c) * kQB + r;
    const float mc = pml[pi * 2], lc = pml[pi * 2 + 1];
    const float w = mc == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((mc - mx) * a.c);
    const f32x2_t ov = *(const f32x2_t*)(a.ws + pi * kDh + 2 * lane);
    l = __builtin_fmaf(w, lc, l);
    o0 = __builtin_fmaf(w, ov[0], o0);
    o1 = __builtin_fmaf(w, ov[1], o1);
  }
  const float inv = 1.0f / l;
  *(uint32_t*)(dst + 2 * lane) = pack2(o0 * inv, o1 * inv);
}

}  // namespace

namespace {
int attn_args(AttnArgs& a, const void* qkv, int batch, int heads, int s_pad, const int* kv_len_host,
              void* out_img, void* out_txt, int s_img, int txt_rows, float scale) {
  QIE_CHECK_ARG(qkv && kv_len_host && out_img && (out_txt || txt_rows == 0));
  QIE_CHECK_ARG(batch > 0 && batch <= QIE_MAX_BATCH && heads > 0);
  QIE_CHECK_ARG(s_pad > 0 && s_pad % kQB == 0 && s_img >= 0 && txt_rows >= 0);
  QIE_CHECK_ARG(s_img + txt_rows <= s_pad && s_img + txt_rows > 0);
  a = AttnArgs{};
  a.qkv = (const bf16_t*)qkv;
  a.out_img = (bf16_t*)out_img;
  a.out_txt = (bf16_t*)out_txt;
  a.B = batch;
  a.H = heads;
  a.s_pad = s_pad;
  a.s_img = s_img;
  a.txt_rows = txt_rows;
  a.qblocks = (s_img + txt_rows + kQB - 1) / kQB;
  a.c = scale * 1.4426950408889634f;
  for (int i = 0; i < batch; ++i) {
    QIE_CHECK_ARG(kv_len_host[i] > 0 && kv_len_host[i] <= s_pad);
    a.kv_len.v[i] = kv_len_host[i];
  }
  return QIE_OK;
}

int64_t split_bytes(int batch, int heads, int qblocks) {
  return qblocks > 1 ? (int64_t)batch * heads * QIE_ATTN_SPLIT * kQB * (kDh + 2) * 4 : 0;
}
}  // namespace

namespace {
// whole query blocks (+ the split tail and its combine when `ws` is given)
int launch_attn(AttnArgs& a, bool pre, void* workspace, int64_t workspace_bytes, hipStream_t s) {
  const int64_t need = workspace ? split_bytes(a.B, a.H, a.qblocks) : 0;
  if (pre) a.c = 1.0f;  // logits already in log2 units (combine weights too)
  if (need == 0) {      // no workspace, or a single query block: nothing to split
    if (pre) attn_pp_kernel<true><<<a.qblocks * a.H * a.B, 512, 0, s>>>(a);
    else attn_pp_kernel<false><<<a.qblocks * a.H * a.B, 512, 0, s>>>(a);
    return qie_last_error();
  }
  QIE_CHECK_ARG(workspace_bytes >= need && ((uintptr_t)workspace % 16) == 0);
  a.split = QIE_ATTN_SPLIT;
  a.ws = (float*)workspace;
  const int grid = ((a.qblocks - 1) + a.split) * a.H * a.B;
  if (pre) attn_pp_kernel<true><<<grid, 512, 0, s>>>(a);
  else attn_pp_kernel<false><<<grid, 512, 0, s>>>(a);
  attn_combine_kernel<<<(a.B * a.H * kQB + 3) / 4, 256, 0, s>>>(a);
  return qie_last_error();
}
}  // namespace

extern "C" int qie_attention_fwd_bf16(const void* qkv, int batch, int heads, int s_pad,
                                      const int* kv_len_host, void* out_img, void* out_txt,
                                      int s_img, int txt_rows, float scale, qie_stream_t stream) {
  AttnArgs a;
  const int rc = attn_args(a, qkv, batch, heads, s_pad, kv_len_host, out_img, out_txt, s_img, txt_rows, scale);
  if (rc) return rc;
  return launch_attn(a, false, nullptr, 0, (hipStream_t)stream);
}

extern "C" int qie_attention_workspace_bytes(int batch, int heads, int s_pad, int s_img, int txt_rows,
                                             int64_t* bytes) {
  QIE_CHECK_ARG(bytes && batch > 0 && heads > 0 && s_pad > 0 && s_img >= 0 && txt_rows >= 0);
  *bytes = split_bytes(batch, heads, (s_img + txt_rows + kQB - 1) / kQB);
  return QIE_OK;
}

extern "C" int qie_attention_fwd_split_bf16(const void* qkv, int batch, int heads, int s_pad,
                                            const int* kv_len_host, void* out_img, void* out_txt,
                                            int s_img, int txt_rows, float scale, void* workspace,
                                            int64_t workspace_bytes, qie_stream_t stream) {
  AttnArgs a;
  const int rc = attn_args(a, qkv, batch, heads, s_pad, kv_len_host, out_img, out_txt, s_img, txt_rows, scale);
  if (rc) return rc;
  QIE_CHECK_ARG(workspace || split_bytes(batch, heads, a.qblocks) == 0);
  return launch_attn(a, false, workspace, workspace_bytes, (hipStream_t)stream);
}

extern "C" int qie_attention_fwd_log2q_bf16(const void* qkv, int batch, int heads, int s_pad,
                                            const int* kv_len_host, void* out_img, void* out_txt,
                                            int s_img, int txt_rows, void* workspace,
                                            int64_t workspace_bytes, qie_stream_t stream) {
  AttnArgs a;
  const int rc = attn_args(a, qkv, batch, heads, s_pad, kv_len_host, out_img, out_txt, s_img, txt_rows, 1.0f);
  if (rc) return rc;
  return launch_attn(a, true, workspace, workspace_bytes, (hipStream_t)stream);
}
