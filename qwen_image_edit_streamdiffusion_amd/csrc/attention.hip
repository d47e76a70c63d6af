// Joint non-causal flash attention forward, head_dim 128, bf16 in/out.
//
// Replaces the SDPA call of diffusers' QwenDoubleStreamAttnProcessor2_0 [U]
// (SURVEY.md §2D K8, §8 a12): softmax(Q K^T / sqrt(128)) V over the joint
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
// V live in 3-slot LDS rings filled by buffer_load...lds two tiles ahead. Waits: vmcnt(0) at
// the end of an M-phase (this wave's pieces from its previous V-phase), vmcnt(pieces) at the
// end of a V-phase; one barrier per phase.
#ifndef QIE_ATTN_EARLY  // bit 0: 4-slot rings, DMA one tile further ahead, no vmcnt at the M-end;
#define QIE_ATTN_EARLY 1  // bit 1: the next M-phase's first reads before the V-end barrier;
#endif                    // bit 2: keep the M-end vmcnt(0)
constexpr int kRing = (QIE_ATTN_EARLY & 1) ? 4 : 3;
#ifndef QIE_ATTN_MPRIO  // issue priority of a wave in its MFMA phase
#define QIE_ATTN_MPRIO 2
#endif
#ifndef QIE_ATTN_VPRIO  // ... and in its softmax phase
#define QIE_ATTN_VPRIO 0
#endif
#ifndef QIE_ATTN_STATIC  // >= 0: waves 4-7 at this priority for the whole loop, no per-phase flips
#define QIE_ATTN_STATIC -1
#endif
#ifndef QIE_ATTN_ONES  // 1: row sums by 4 MFMAs against a ones operand in the MFMA phase (log2q path)
#define QIE_ATTN_ONES 0
#endif
#ifndef QIE_ATTN_PKSUM  // 1: the log2-q softmax's row sums as packed f32x2 adds
#define QIE_ATTN_PKSUM 0  // measured 8 % slower (1.413 -> 1.530 ms): packed FP32 beside the partner wave's MFMAs
#endif
#ifndef QIE_ATTN_ABL  // diagnostic ablations (wrong results): 1 no K/V DMA in the loop, 2 no exp2
#define QIE_ATTN_ABL 0
#endif

#ifdef QIE_ATTN_STAMP
// diagnostic build only (tools/attn_stamp.hip): per-group sums of phase cycles
__device__ unsigned long long g_stamp[2][6];
#define STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define STAMP_ADD(i, d) acc_st[i] += (d)
#else
#define STAMP(v)
#define STAMP_ADD(i, d)
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
// DMA target (the loop's own counted waits cover it). M0 is set and restored inside the
// statement; s_nop 4 covers a just-readfirstlane'd SGPR operand (cdna_hip_programming §5.7).
__device__ __forceinline__ void attn_dma(const i32x4_t& r, const char QIE_LDS* dst, uint32_t voff, int soff) {
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
#ifndef QIE_ATTN_LEAN  // 1: DMA pieces without the hand-saved M0 / leading s_nop (M0 declared clobbered)
#define QIE_ATTN_LEAN 1
#endif
__device__ __forceinline__ void attn_dma_lean(const i32x4_t& r, const char QIE_LDS* dst, uint32_t voff, int soff) {
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
  f32x16_t lsum;  // PRE && QIE_ATTN_ONES: every element = the lane's query row sum
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
  bf16x8_t ones;
#pragma unroll
  for (int k = 0; k < 8; ++k) ones[k] = (__bf16)1.0f;
#ifdef QIE_ATTN_STAMP
  unsigned long long acc_st[6] = {0, 0, 0, 0, 0, 0};
#endif
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
    char QIE_LDS* base = smem + (t % kRing) * kTileBytes;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      if constexpr (QIE_ATTN_LEAN) attn_dma_lean(kr, base + (wave + 8 * p) * 1024, ko[p], t * kTileBytes);
      else attn_dma(kr, base + (wave + 8 * p) * 1024, ko[p], t * kTileBytes);
    }
  };
  auto dmaV = [&](int t) {
    char QIE_LDS* base = smem + (kRing + t % kRing) * kTileBytes;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      if constexpr (QIE_ATTN_LEAN) attn_dma_lean(vr, base + (wave + 8 * p) * 1024, vo[p], t * kTileBytes);
      else attn_dma(vr, base + (wave + 8 * p) * 1024, vo[p], t * kTileBytes);
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
      const char QIE_LDS* krow = smem + (tk % kRing) * kTileBytes + (cb * 32 + ql) * 256;
      return *(const bf16x8_t QIE_LDS*)(krow + (((2 * ks + hf) ^ ksw) << 4));
    }
    const int j = i - 16, ks = j >> 2, db = j & 3;
    const char QIE_LDS* vb = smem + (kRing + tv % kRing) * kTileBytes;
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
  // EARLY: the first PF operands of an M-phase are read at the end of the preceding V-phase,
  // before its barrier (their tiles landed two V-phases ago, see vphase), so the MFMAs start
  // right behind the barrier instead of behind one LDS round trip
  auto mpre = [&](int i0, int i1, int tk, int tv) {
#pragma unroll
    for (int i = 0; i < 32; ++i)
      if (i >= i0 && i < i0 + PF && i < i1) A[i & 7] = opA(i, tk, tv);
  };
  auto mphase = [&](auto i0_t, auto i1_t, int tk, int tv, bool pre_read) {
    constexpr int i0 = decltype(i0_t)::value, i1 = decltype(i1_t)::value;
    // the MFMA wave outranks its SIMD partner (in its softmax phase) for issue: otherwise the
    // older wave group wins arbitration and starves the younger group's MFMA phase
    if (QIE_ATTN_STATIC < 0) __builtin_amdgcn_s_setprio(QIE_ATTN_MPRIO);
    if (!pre_read) {
#pragma unroll
      for (int i = i0; i < i0 + PF && i < i1; ++i) A[i & 7] = opA(i, tk, tv);
    }
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      if (i + PF < i1) A[(i + PF) & 7] = opA(i + PF, tk, tv);
      mfma_i(i, A[i & 7]);
      if constexpr (PRE && QIE_ATTN_ONES && i1 == 32) {  // row sums of P(t-1), beside the PV MFMAs
        if (i >= 16 && ((i - 16) & 3) == 3) mma32(st.lsum, ones, st.pf[(i - 16) >> 2]);
      }
    }
    if (QIE_ATTN_STATIC < 0) __builtin_amdgcn_s_setprio(QIE_ATTN_VPRIO);
  };
  // V-phase: softmax of S(t) into P(t), DMA of later tiles; ends with the phase barrier
  auto vphase = [&](int t) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) rfence(st.s[cb]);
#pragma unroll
    for (int db = 0; db < 4; ++db) rfence(st.o[db]);
    int pieces = 0;
    if (!(QIE_ATTN_ABL & 1)) {
      constexpr int ahead = (QIE_ATTN_EARLY & 1) ? 1 : 0;  // EARLY: K(t+3), V(t+2)
      if (t + 2 + ahead < ntiles) { dmaK(t + 2 + ahead); pieces += 2; }
      if (t + 1 + ahead < ntiles) { dmaV(t + 1 + ahead); pieces += 2; }
    }
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
    auto exp_tile = [&]() {  // P = exp2(S), row sums, bf16 P^T fragments
      // the two interleaved row-sum chains as one f32x2 (v_pk_add_f32: 16 adds per tile, not 32;
      // same per-chain order, so the same bits)
      f32x2_t ps = {0.f, 0.f};
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const float p0 = __builtin_amdgcn_exp2f(st.s[cb][r]);
          const float p1 = __builtin_amdgcn_exp2f(st.s[cb][r + 1]);
          if (!(PRE && QIE_ATTN_ONES)) {
            if constexpr (QIE_ATTN_PKSUM) {
              ps += f32x2_t{p0, p1};
            } else {
              ps0 += p0;
              ps1 += p1;
            }
          }
          st.pf[cb * 2 + (r >> 3)][r & 7] = (__bf16)p0;
          st.pf[cb * 2 + (r >> 3)][(r & 7) + 1] = (__bf16)p1;
        }
      if constexpr (QIE_ATTN_PKSUM) {
        ps0 = ps.x;
        ps1 = ps.y;
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
        if constexpr (QIE_ATTN_ONES) st.lsum *= alpha;
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
#if QIE_ATTN_ABL & 2
        const float p0 = __builtin_fmaf(st.s[cb][r], c, -mc);
        const float p1 = __builtin_fmaf(st.s[cb][r + 1], c, -mc);
#else
        const float p0 = __builtin_amdgcn_exp2f(__builtin_fmaf(st.s[cb][r], c, -mc));
        const float p1 = __builtin_amdgcn_exp2f(__builtin_fmaf(st.s[cb][r + 1], c, -mc));
#endif
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
    if constexpr (PRE && QIE_ATTN_ONES) rfence(st.lsum);
#pragma unroll
    for (int db = 0; db < 4; ++db) rfence(st.o[db]);
    // EARLY: the next M-phase reads K(t+1) and V(t) (whole M-phase) or V(t) (the tail); their
    // pieces were issued in V-phase t-2 and every wave's V-phase t-1 ended with vmcnt(pieces of
    // t-1), i.e. with them landed, before the barrier that precedes this V-phase
    if (QIE_ATTN_EARLY & 2) {
      if (t + 1 < ntiles) mpre(0, 32, t + 1, t);
      else mpre(16, 32, t0, t);
    }
    if (pieces == 4) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    else if (pieces == 2) asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  };
  using I0 = std::integral_constant<int, 0>;
  using I16 = std::integral_constant<int, 16>;
  using I32 = std::integral_constant<int, 32>;
  using IMEND = I32;

  const int q_loc = wave * 32 + ql;  // row within the query block
  if (t0 >= ntiles) {                // empty key range (fewer tiles than ranges): neutral partial
    float* po = a.ws + (((int64_t)bh * a.split + chunk) * kQB + q_loc) * kDh;
    float* pml = a.ws + (int64_t)a.B * a.H * a.split * kQB * kDh;
#pragma unroll
    for (int k = 0; k < 16; ++k) *(f32x4_t*)(po + 8 * k + 4 * hf) = f32x4_t{0, 0, 0, 0};
    if (hf == 0) *(f32x2_t*)(pml + (((int64_t)bh * a.split + chunk) * kQB + q_loc) * 2) = f32x2_t{-INFINITY, 0.f};
    return;
  }
  // ---- prologue: K(t0), K(t0+1), V(t0) resident (EARLY: + K(t0+2), V(t0+1)); group 1 waits
  // one phase
  dmaK(t0);
  if (t0 + 1 < ntiles) dmaK(t0 + 1);
  dmaV(t0);
  if (QIE_ATTN_EARLY & 1) {
    if (t0 + 2 < ntiles) dmaK(t0 + 2);
    if (t0 + 1 < ntiles) dmaV(t0 + 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the asm DMA pieces
  __builtin_amdgcn_s_waitcnt(0);                     // Q fragments (hipcc-tracked)
  asm volatile("s_barrier" ::: "memory");
  if (grp == 1) asm volatile("s_barrier" ::: "memory");
  // static form (MI355X_MICROARCH.md "Two waves per SIMD" item 4): one priority per wave group
  // for the whole loop instead of per-phase flips
  if (QIE_ATTN_STATIC >= 0 && grp == 1) __builtin_amdgcn_s_setprio(QIE_ATTN_STATIC);
#pragma unroll
  for (int db = 0; db < 4; ++db) st.o[db] = f32x16_t{};
  st.m_run = PRE ? 0.f : -INFINITY;  // PRE: finite (it is the MFMA's C); tile t0 sets it
  st.l_run = 0.f;
  if constexpr (PRE) st.negm = f32x16_t{};
  if constexpr (PRE && QIE_ATTN_ONES) st.lsum = f32x16_t{};

  // EARLY: no vmcnt at the M-end (the V-end wait covers every tile two phases before its use)
  auto mend = [&](int) {
    if ((QIE_ATTN_EARLY & 5) == 1) asm volatile("s_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  };
  mphase(I0{}, I16{}, t0, t0, false);  // S(t0)
  mend(t0);
  vphase(t0);
  for (int t = t0 + 1; t < ntiles; ++t) {
    STAMP(t0);
    mphase(I0{}, IMEND{}, t, t - 1, QIE_ATTN_EARLY & 2);  // S(t), O += V(t-1) P(t-1)
    STAMP(t1);
    mend(t);
    STAMP(t2);
    vphase(t);
    STAMP(t3);
    STAMP_ADD(0, t1 - t0);  // M-phase body
    STAMP_ADD(1, t2 - t1);  // M-end wait + barrier
    STAMP_ADD(2, t3 - t2);  // V-phase body incl. its end barrier
    STAMP_ADD(3, 1);
  }
#ifdef QIE_ATTN_STAMP
  if (lane == 0)
    for (int i = 0; i < 4; ++i) atomicAdd(&g_stamp[grp][i], acc_st[i]);
#endif
  mphase(I16{}, IMEND{}, t0, ntiles - 1, QIE_ATTN_EARLY & 2);  // O += V(T-1) P(T-1)
  if (grp == 0) asm volatile("s_barrier" ::: "memory");
  // MFMA D -> VALU read hazard before the epilogue reads O (asm MFMAs are not padded by hipcc)
  asm volatile("s_nop 15\n\ts_nop 7" : "+v"(st.o[0]), "+v"(st.o[1]), "+v"(st.o[2]), "+v"(st.o[3]));
  float l_tot;
  if constexpr (PRE && QIE_ATTN_ONES) {
    asm volatile("s_nop 7" : "+v"(st.lsum));
    l_tot = st.lsum[0];  // the MFMA summed all 64 keys of every tile into each row of the column
  } else {
    l_tot = st.l_run + __shfl_xor(st.l_run, 32, 64);
  }
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

// =============================================================================================
// attn16_kernel: the log2-q (PRE) attention on v_mfma_f32_16x16x32_bf16. Same work-group shape,
// K / V rings, LDS-DMA, two-group ping-pong and barriers as attn_pp_kernel; only the MFMA shape
// changes. MI355X_MICROARCH.md "DVFS give-back" (7): on random data the chip holds a higher
// clock under 16x16x32 loops than under 32x32x16 ones (~1.12-1.15x FLOP/s at equal cycles per
// FLOP), and this kernel is MFMA-paced.
// Per wave: 32 query rows = two 16-row column blocks qb; per 64-key tile four 16-key blocks kb.
// Lane (g = lane >> 4, c = lane & 15):
//   S^T[kb][qb] (16 keys x 16 queries, f32x4): query qb*16 + c, keys kb*16 + 4g + r (r = 0..3)
//     = sum_ks K[kb*16 + c][32ks + 8g ..] (A, ds_read_b128) x Q^T (B, registers qf[qb][ks])
//   -> the lane's 16 scores of a query are reduced over the 4 lane groups by two swaps
//   P^T B operand of key step ks2 (32 keys): elements 0..3 = kb 2ks2, 4..7 = kb 2ks2 + 1, so the
//   k index 8g + j maps to key 32ks2 + 4g + j (j < 4) / 32ks2 + 16 + 4g + (j - 4)
//   O^T[db][qb] (f32x4): d = 16db + 4g + r of query qb*16 + c
//     += V^T (A: two ds_read_b64_tr_b16 of 4 keys x 16 d each, keys as the P^T permutation) x P^T
// V ring swizzle: chunk ^ ((row & 3) << 2) ^ (((row >> 2) & 1) << 1), so both 16-lane groups of a
// transposed read's 32-lane half (rows 4 apart) hit distinct banks.
#ifndef QIE_ATTN16
#define QIE_ATTN16 0  // 1: log2-q launches on attn16_kernel (measured 1.5-3 % slower, off)
#endif
#ifndef QIE_ATTN16_PF
#define QIE_ATTN16_PF 4  // operand prefetch distance in fragments (2 MFMAs each)
#endif

__device__ __forceinline__ void mma16(f32x4_t& c, const bf16x8_t& a, const bf16x8_t& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mma16_c(f32x4_t& c, const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c0) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %3" : "=&v"(c) : "v"(a), "v"(b), "v"(c0));
}
__device__ __forceinline__ float max_over_groups(float m) {  // max over lanes c, c+16, c+32, c+48
  const auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  m = fmaxf(__uint_as_float(s16[0]), __uint_as_float(s16[1]));
  const auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return fmaxf(__uint_as_float(s32[0]), __uint_as_float(s32[1]));
}

struct P16State {
  f32x4_t s[4][2];  // [kb][qb]
  f32x4_t o[8][2];  // [db][qb]
  f32x4_t negm[2];  // splat(-m_run[qb]): C operand of each tile's first QK^T MFMA
  bf16x8_t pf[2][2];  // [ks2][qb]
  bf16x8_t qf[2][4];  // [qb][ks]
  float m_run[2], l_run[2];
};

__global__ void __launch_bounds__(512) attn16_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * kRing * kTileBytes];  // K ring, V ring
  char QIE_LDS* smem = (char QIE_LDS*)smem_raw;

  const int qbf = a.split ? a.qblocks - 1 : a.qblocks;
  const int nfull = qbf * a.H * a.B;
  int qblk, bh, chunk = -1;
  if ((int)blockIdx.x < nfull) {
    const int wgid = xcd_remap(blockIdx.x, nfull);
    qblk = wgid % qbf;
    bh = wgid / qbf;
  } else {
    const int j = blockIdx.x - nfull;
    bh = j / a.split;
    chunk = j - bh * a.split;
    qblk = a.qblocks - 1;
  }
  const int h = bh % a.H, b = bh / a.H;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;
  const int g = lane >> 4;
  const int c = lane & 15;
  const int64_t plane = (int64_t)a.s_pad * kDh;
  const bf16_t* Qp = a.qkv + ((int64_t)(0 * a.B + b) * a.H + h) * plane;
  const bf16_t* Kp = a.qkv + ((int64_t)(1 * a.B + b) * a.H + h) * plane;
  const bf16_t* Vp = a.qkv + ((int64_t)(2 * a.B + b) * a.H + h) * plane;
  const int kv_len = a.kv_len.v[b];
  const int ntot = (kv_len + kKB - 1) / kKB;
  const int t0 = chunk < 0 ? 0 : chunk * ntot / a.split;
  const int ntiles = chunk < 0 ? ntot : (chunk + 1) * ntot / a.split;

  P16State st;
  const int q_wave = qblk * kQB + wave * 32;  // first query row of this wave
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const bf16_t* qr = Qp + (int64_t)(q_wave + qb * 16 + c) * kDh + 8 * g;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) st.qf[qb][ks] = *(const bf16x8_t*)(qr + 32 * ks);
  }

  // ---- LDS-DMA: wave w fills rows 4(w + 8p) .. +3 of a tile (p = 0, 1) for K and for V
  const auto kr = attn_rsrc(Kp, a.s_pad * kDh * 2);
  const auto vr = attn_rsrc(Vp, a.s_pad * kDh * 2);
  uint32_t ko[2], vo[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int row = (wave + 8 * p) * 4 + (lane >> 4), cc = lane & 15;
    ko[p] = row * 256 + ((cc ^ (row & 15)) << 4);
    vo[p] = row * 256 + ((cc ^ ((row & 3) << 2) ^ (((row >> 2) & 1) << 1)) << 4);
  }
  auto dmaK = [&](int t) {
    char QIE_LDS* base = smem + (t % kRing) * kTileBytes;
#pragma unroll
    for (int p = 0; p < 2; ++p) attn_dma_lean(kr, base + (wave + 8 * p) * 1024, ko[p], t * kTileBytes);
  };
  auto dmaV = [&](int t) {
    char QIE_LDS* base = smem + (kRing + t % kRing) * kTileBytes;
#pragma unroll
    for (int p = 0; p < 2; ++p) attn_dma_lean(vr, base + (wave + 8 * p) * 1024, vo[p], t * kTileBytes);
  };

  // per-lane LDS offsets: K row c of a 16-key block; V transposed-read lane (q, p) = (c >> 2, c & 3)
  const int k_lane = c * 256;
  const int tq = c >> 2, tp = c & 3;
  const int v_sw = (tq << 1) ^ (g & 1);  // the V swizzle of rows 4g + tq, in units of 2 chunks
  const int v_lane = (4 * g + tq) * 256 + ((tp >> 1) << 4) + 8 * (tp & 1);

  // fragment f of an M-phase: f < 16 -> K (kb = f >> 2, ks = f & 3) of tile tk;
  // f >= 16 -> V^T (ks2 = (f-16) >> 3, db = (f-16) & 7) of tile tv
  auto opA = [&](int f, int tk, int tv) -> bf16x8_t {
    if (f < 16) {
      const int kb = f >> 2, ks = f & 3;
      const char QIE_LDS* p = smem + (tk % kRing) * kTileBytes + kb * 16 * 256 + k_lane;
      return *(const bf16x8_t QIE_LDS*)(p + (((4 * ks + g) ^ c) << 4));
    }
    const int j = f - 16, ks2 = j >> 3, db = j & 7;
    const char QIE_LDS* p = smem + (kRing + tv % kRing) * kTileBytes + ks2 * 32 * 256 + v_lane +
                            ((db ^ v_sw) << 5);
    const s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4_t QIE_LDS*)p);
    const s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4_t QIE_LDS*)(p + 16 * 256));
    return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto mfma_f = [&](int f, const bf16x8_t& A) {
    if (f < 16) {
      const int kb = f >> 2, ks = f & 3;
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        if (ks == 0) mma16_c(st.s[kb][qb], A, st.qf[qb][0], st.negm[qb]);
        else mma16(st.s[kb][qb], A, st.qf[qb][ks]);
      }
    } else {
      const int j = f - 16, ks2 = j >> 3, db = j & 7;
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) mma16(st.o[db][qb], A, st.pf[ks2][qb]);
    }
  };
  auto mphase = [&](auto f0_t, auto f1_t, int tk, int tv) {
    constexpr int f0 = decltype(f0_t)::value, f1 = decltype(f1_t)::value;
    constexpr int PF = QIE_ATTN16_PF;
    bf16x8_t A[8];
    __builtin_amdgcn_s_setprio(QIE_ATTN_MPRIO);
#pragma unroll
    for (int f = f0; f < f0 + PF && f < f1; ++f) A[f & 7] = opA(f, tk, tv);
#pragma unroll
    for (int f = f0; f < f1; ++f) {
      if (f + PF < f1) A[(f + PF) & 7] = opA(f + PF, tk, tv);
      mfma_f(f, A[f & 7]);
    }
    __builtin_amdgcn_s_setprio(QIE_ATTN_VPRIO);
  };
  auto vphase = [&](int t) {
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) rfence(st.s[kb][qb]);
#pragma unroll
    for (int db = 0; db < 8; ++db)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) rfence(st.o[db][qb]);
    int pieces = 0;
    if (t + 2 < ntiles) { dmaK(t + 2); pieces += 2; }
    if (t + 1 < ntiles) { dmaV(t + 1); pieces += 2; }
    const int kv0 = t * kKB;
    if (kv0 + kKB > kv_len) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kv = kv0 + kb * 16 + 4 * g + r;
          if (kv >= kv_len) {
            st.s[kb][0][r] = -INFINITY;
            st.s[kb][1][r] = -INFINITY;
          }
        }
    }
    float mx[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      float m0 = fmaxf(st.s[0][qb][0], st.s[0][qb][1]), m1 = fmaxf(st.s[0][qb][2], st.s[0][qb][3]);
#pragma unroll
      for (int kb = 1; kb < 4; ++kb) {
        m0 = fmaxf(m0, fmaxf(st.s[kb][qb][0], st.s[kb][qb][1]));
        m1 = fmaxf(m1, fmaxf(st.s[kb][qb][2], st.s[kb][qb][3]));
      }
      mx[qb] = max_over_groups(fmaxf(m0, m1));
    }
    // S holds s*c - m_run (log2 units); tile t0 always rescales (it sets m_run)
    if (__any(t == t0 || mx[0] > kRescaleThr || mx[1] > kRescaleThr)) {
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const float d = t == t0 ? mx[qb] : fmaxf(mx[qb], 0.f);
        const float alpha = __builtin_amdgcn_exp2f(-d);
        st.m_run[qb] += d;
        st.l_run[qb] *= alpha;
#pragma unroll
        for (int db = 0; db < 8; ++db) st.o[db][qb] *= alpha;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) st.s[kb][qb] -= d;
        const float nm = -st.m_run[qb];
        st.negm[qb] = f32x4_t{nm, nm, nm, nm};
      }
    }
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      float ps0 = 0.f, ps1 = 0.f;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const float p0 = __builtin_amdgcn_exp2f(st.s[kb][qb][0]);
        const float p1 = __builtin_amdgcn_exp2f(st.s[kb][qb][1]);
        const float p2 = __builtin_amdgcn_exp2f(st.s[kb][qb][2]);
        const float p3 = __builtin_amdgcn_exp2f(st.s[kb][qb][3]);
        ps0 += p0 + p2;
        ps1 += p1 + p3;
        const int e = (kb & 1) * 4;
        st.pf[kb >> 1][qb][e] = (__bf16)p0;
        st.pf[kb >> 1][qb][e + 1] = (__bf16)p1;
        st.pf[kb >> 1][qb][e + 2] = (__bf16)p2;
        st.pf[kb >> 1][qb][e + 3] = (__bf16)p3;
      }
      st.l_run[qb] += ps0 + ps1;
    }
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) rfence(st.pf[k][qb]);
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      rfence(st.l_run[qb]);
      rfence(st.m_run[qb]);
      rfence(st.negm[qb]);
    }
#pragma unroll
    for (int db = 0; db < 8; ++db)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) rfence(st.o[db][qb]);
    if (pieces == 4) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    else if (pieces == 2) asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  };
  using F0 = std::integral_constant<int, 0>;
  using F16 = std::integral_constant<int, 16>;
  using F32 = std::integral_constant<int, 32>;

  float* po_base = nullptr;
  float* pml = nullptr;
  if (chunk >= 0) {
    po_base = a.ws + ((int64_t)bh * a.split + chunk) * kQB * kDh;
    pml = a.ws + (int64_t)a.B * a.H * a.split * kQB * kDh + ((int64_t)bh * a.split + chunk) * kQB * 2;
  }
  if (t0 >= ntiles) {  // empty key range (fewer tiles than ranges): neutral partial
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int q_loc = wave * 32 + qb * 16 + c;
#pragma unroll
      for (int db = 0; db < 8; ++db)
        *(f32x4_t*)(po_base + (int64_t)q_loc * kDh + 16 * db + 4 * g) = f32x4_t{0, 0, 0, 0};
      if (g == 0) *(f32x2_t*)(pml + q_loc * 2) = f32x2_t{-INFINITY, 0.f};
    }
    return;
  }
  // ---- prologue: K(t0), K(t0+1), V(t0) resident; group 1 waits one phase
  dmaK(t0);
  if (t0 + 1 < ntiles) dmaK(t0 + 1);
  dmaV(t0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0);
  asm volatile("s_barrier" ::: "memory");
  if (grp == 1) asm volatile("s_barrier" ::: "memory");
#pragma unroll
  for (int db = 0; db < 8; ++db)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) st.o[db][qb] = f32x4_t{};
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    st.m_run[qb] = 0.f;  // finite (it is the MFMA's C); tile t0 sets it
    st.l_run[qb] = 0.f;
    st.negm[qb] = f32x4_t{};
  }

  auto mend = [&]() { asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory"); };
  mphase(F0{}, F16{}, t0, t0);  // S(t0)
  mend();
  vphase(t0);
  for (int t = t0 + 1; t < ntiles; ++t) {
    mphase(F0{}, F32{}, t, t - 1);  // S(t), O += V(t-1) P(t-1)
    mend();
    vphase(t);
  }
  mphase(F16{}, F32{}, t0, ntiles - 1);  // O += V(T-1) P(T-1)
  if (grp == 0) asm volatile("s_barrier" ::: "memory");
  // MFMA D -> VALU read hazard before the epilogue reads O (asm MFMAs are not padded by hipcc)
#pragma unroll
  for (int db = 0; db < 8; db += 2)
    asm volatile("s_nop 7" : "+v"(st.o[db][0]), "+v"(st.o[db][1]), "+v"(st.o[db + 1][0]), "+v"(st.o[db + 1][1]));
  asm volatile("s_nop 15" ::: "memory");
  float l_tot[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    float l = st.l_run[qb];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    l_tot[qb] = l;
  }
  if (chunk >= 0) {  // fp32 partial: unnormalised O, row max, row sum
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int q_loc = wave * 32 + qb * 16 + c;
#pragma unroll
      for (int db = 0; db < 8; ++db)
        *(f32x4_t*)(po_base + (int64_t)q_loc * kDh + 16 * db + 4 * g) = st.o[db][qb];
      if (g == 0) *(f32x2_t*)(pml + q_loc * 2) = f32x2_t{st.m_run[qb], l_tot[qb]};
    }
    return;
  }
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int s = q_wave + qb * 16 + c;
    bf16_t* dst = nullptr;
    if (s < a.s_img) {
      dst = a.out_img + ((int64_t)b * a.s_img + s) * (a.H * kDh) + h * kDh;
    } else if (s < a.s_img + a.txt_rows) {
      dst = a.out_txt + ((int64_t)b * a.txt_rows + (s - a.s_img)) * (a.H * kDh) + h * kDh;
    }
    const float inv = 1.0f / l_tot[qb];
    // lane (g, c) holds d = 16db + 4g + 0..3; one permlane16 swap per dword of the pair (db, db+1)
    // gives an even-g lane d = 16db + 4g .. +7 and an odd-g lane d = 16(db+1) + 4(g-1) .. +7
#pragma unroll
    for (int db = 0; db < 8; db += 2) {
      const f32x4_t& x0 = st.o[db][qb];
      const f32x4_t& x1 = st.o[db + 1][qb];
      const unsigned w0x = pack2(x0[0] * inv, x0[1] * inv), w0y = pack2(x0[2] * inv, x0[3] * inv);
      const unsigned w1x = pack2(x1[0] * inv, x1[1] * inv), w1y = pack2(x1[2] * inv, x1[3] * inv);
      const auto sx = __builtin_amdgcn_permlane16_swap(w0x, w1x, false, false);
      const auto sy = __builtin_amdgcn_permlane16_swap(w0y, w1y, false, false);
      const int d0 = (g & 1) ? 16 * (db + 1) + 4 * (g - 1) : 16 * db + 4 * g;
      if (dst) *(u32x4_t*)(dst + d0) = u32x4_t{sx[0], sy[0], sx[1], sy[1]};
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
    l += w * lc;
    o0 += w * ov[0];
    o1 += w * ov[1];
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
    if (pre && QIE_ATTN16) attn16_kernel<<<a.qblocks * a.H * a.B, 512, 0, s>>>(a);
    else if (pre) attn_pp_kernel<true><<<a.qblocks * a.H * a.B, 512, 0, s>>>(a);
    else attn_pp_kernel<false><<<a.qblocks * a.H * a.B, 512, 0, s>>>(a);
    return qie_last_error();
  }
  QIE_CHECK_ARG(workspace_bytes >= need && ((uintptr_t)workspace % 16) == 0);
  a.split = QIE_ATTN_SPLIT;
  a.ws = (float*)workspace;
  const int grid = ((a.qblocks - 1) + a.split) * a.H * a.B;
  if (pre && QIE_ATTN16) attn16_kernel<<<grid, 512, 0, s>>>(a);
  else if (pre) attn_pp_kernel<true><<<grid, 512, 0, s>>>(a);
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
