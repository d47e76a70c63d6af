// Flash attention for the VAE mid-block (QwenImageAttentionBlock [U]): ONE head
// of C = 384 channels over the P = h*w latent pixels (16384 at 1024^2), softmax(q k^T / sqrt(C)) v.
// Replaces the materialised form (fp32 scores [P][P] = 1 GiB at 1024^2, a row softmax to bf16,
// then P.V): the scores never leave the registers.
//
// Layout: q, k are the first two C-column blocks of the to_qkv output rows [P][3C] (bf16); v comes
// transposed, vt [C][ldvt] (bf16, keys contiguous, zero past P). A workgroup owns 128 query rows
// (4 waves x 32) and one of `nsplit` key ranges; its fp32 partial (unnormalised O, running max m
// and sum l) goes to a workspace that vae_attn_combine_kernel folds into the bf16 output.
//
// Per 32-key step and wave (MFMA 16x16x32 bf16, swapped products so each lane owns one query
// column): S^T[32 keys][32 q] = K . Q^T (48 MFMAs, Q^T fragments held in registers for the whole
// launch), online softmax in log2 units (the row max only re-based when it grows by more than 8,
// so the O rescale is rare), O^T[384][32 q] += V^T . P^T (48 MFMAs, P^T straight from the S^T
// accumulators: the lane's keys {4g..4g+3, 16+4g..16+4g+3} are the k order of both operands).
// K and V^T tiles (24 KiB each) land by LDS-DMA in a 3-stage ring two steps ahead.
// LDS images: K rows of 768 B with the 16-byte chunk XOR-ed by (key & 15); V^T rows of 64 B with
// the 16-byte chunk XOR-ed by ((d >> 2) & 3): conflict-free for the b128 / b64 fragment reads.
#include <algorithm>

#include "qie_common.h"

namespace {

constexpr int kC = 384;                  // head width (channels)
constexpr int kKB = 32;                  // keys per step
constexpr int kKT = kKB * kC * 2;        // K tile bytes: [32 keys][384]
constexpr int kVT = kC * kKB * 2;        // V^T tile bytes: [384][32 keys]
constexpr int kStage = kKT + kVT;        // 48 KiB
constexpr int kStages = 3;
#ifndef QIE_VA_QB  // query blocks of 16 per wave: 1 (8 waves, 2 per SIMD) or 2 (4 waves, 1 per SIMD)
#define QIE_VA_QB 1
#endif
constexpr int kQB = QIE_VA_QB, kNW = 8 / kQB;  // waves per workgroup (128 query rows)
constexpr int kPieces = kStage / 1024 / kNW;  // 1-KiB LDS-DMA pieces per wave and step

__device__ __forceinline__ i32x4_t va_rsrc(const void* base, uint32_t bytes) {
  const uint64_t p = (uint64_t)base;
  return i32x4_t{__builtin_amdgcn_readfirstlane((int)(uint32_t)p),
                 __builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32)),
                 __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000};
}
// one 1-KiB buffer_load_dwordx4 ... lds piece (offsets past the descriptor's range read zeros);
// inline asm, so hipcc adds no vmcnt of its own before the LDS reads
__device__ __forceinline__ void va_dma(const i32x4_t& r, const char QIE_LDS* dst, uint32_t voff) {
  const int lds = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)dst);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :
               : "v"(voff), "s"(r), "s"(lds)
               : "memory", "m0");
}
// O^T accumulators stay in AGPRs: asm MFMAs (hipcc would otherwise rotate 192 accumulators through
// VGPR copies next to the 96 VGPRs of Q^T fragments)
#if QIE_VA_QB == 1  // 2 waves per SIMD: 256 registers per lane, the accumulators in VGPRs
#define QIE_VA_ACC "+v"
#else
#define QIE_VA_ACC "+a"
#endif
__device__ __forceinline__ void va_mma(f32x4_t& c, const bf16x8_t& a, const bf16x8_t& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : QIE_VA_ACC(c) : "v"(a), "v"(b));
}
template <int n>
__device__ __forceinline__ void va_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(n) : "memory");
}

__global__ void __launch_bounds__(kNW * 64, 1)
    vae_attn_kernel(const bf16_t* __restrict__ qkv, int P, int ldqkv, const bf16_t* __restrict__ vt, int ldvt,
                    int kspan, float* __restrict__ opart, float* __restrict__ mlpart, float cscale) {
  __shared__ __attribute__((aligned(16))) char smem_raw[kStages * kStage];
  char QIE_LDS* smem = (char QIE_LDS*)smem_raw;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int fr = lane & 15, g = lane >> 4;
  const int split = blockIdx.y;
  const int kbeg = split * kspan, kend = min(P, kbeg + kspan);
  const int nsteps = kend > kbeg ? (kend - kbeg + kKB - 1) / kKB : 0;
  const int q0 = blockIdx.x * 128 + wave * 16 * kQB;

  // Q^T fragments (B operand: lane = query column fr, channels 8g..8g+7 of each 32-channel chunk)
  bf16x8_t qf[kQB][12];
#pragma unroll
  for (int qb = 0; qb < kQB; ++qb) {
    const bf16_t* qr = qkv + (int64_t)min(q0 + qb * 16 + fr, P - 1) * ldqkv + 8 * g;
#pragma unroll
    for (int dc = 0; dc < 12; ++dc) qf[qb][dc] = *(const bf16x8_t*)(qr + dc * 32);
  }

  // LDS-DMA pieces of a step: K pieces 0..5 and V^T pieces 6..11 of this wave
  const i32x4_t kr = va_rsrc(qkv, (uint32_t)P * ldqkv * 2);
  const i32x4_t vr = va_rsrc(vt, (uint32_t)kC * ldvt * 2);
  constexpr int NPK = kPieces / 2;  // K (and V^T) pieces per wave and step
  uint32_t koff[NPK], voff[NPK];
#pragma unroll
  for (int i = 0; i < NPK; ++i) {
    const int pc = wave + kNW * i;
    const int L = pc * 64 + lane, row = L / 48, cp = L - row * 48;
    const int c = (cp & ~15) | ((cp ^ row) & 15);  // chunk XOR (key & 15) inside its 16-chunk group
    koff[i] = (uint32_t)(row * ldqkv * 2 + (kC + c * 8) * 2);
    const int d = pc * 16 + (lane >> 2), vc = (lane & 3) ^ ((d >> 2) & 3);
    voff[i] = (uint32_t)(d * ldvt * 2 + vc * 16);
  }
  auto dma_step = [&](int s) {
    char QIE_LDS* st = smem + (s % kStages) * kStage;
    const int key0 = kbeg + s * kKB;
    const uint32_t kadd = (uint32_t)key0 * ldqkv * 2, vadd = (uint32_t)key0 * 2;
#pragma unroll
    for (int i = 0; i < NPK; ++i) va_dma(kr, st + (wave + kNW * i) * 1024, koff[i] + kadd);
#pragma unroll
    for (int i = 0; i < NPK; ++i) va_dma(vr, st + kKT + (wave + kNW * i) * 1024, voff[i] + vadd);
  };

  f32x4_t o[24][kQB];
#pragma unroll
  for (int db = 0; db < 24; ++db)
#pragma unroll
    for (int qb = 0; qb < kQB; ++qb) o[db][qb] = f32x4_t{0, 0, 0, 0};
  float m[kQB], l[kQB];
#pragma unroll
  for (int qb = 0; qb < kQB; ++qb) m[qb] = -INFINITY, l[qb] = 0.f;

  auto redefine_o = [&]() {
#pragma unroll
    for (int db = 0; db < 24; db += 4)
#pragma unroll
      for (int qb = 0; qb < kQB; ++qb)
        asm volatile("" : QIE_VA_ACC(o[db][qb]), QIE_VA_ACC(o[db + 1][qb]), QIE_VA_ACC(o[db + 2][qb]), QIE_VA_ACC(o[db + 3][qb]));
  };
  if (nsteps > 0) dma_step(0);
  if (nsteps > 1) dma_step(1);
  if (nsteps > 1) va_wait_barrier<kPieces>();
  else va_wait_barrier<0>();
  for (int s = 0; s < nsteps; ++s) {
    const bool pre = s + 2 < nsteps;
    if (pre) dma_step(s + 2);
    // the accumulators redefined behind the previous step's PV MFMAs (and, the first time, their
    // zeroing): the re-base below reads them only after this step's 48 QK^T MFMAs, far past the
    // MFMA -> VALU hazard window, and no read can be hoisted above this point
    redefine_o();
    const char QIE_LDS* kt = smem + (s % kStages) * kStage;
    const char QIE_LDS* vtt = kt + kKT;
    // S^T = K . Q^T
    f32x4_t sc[2][kQB];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int qb = 0; qb < kQB; ++qb) sc[kb][qb] = f32x4_t{0, 0, 0, 0};
    // K fragments one 32-channel chunk ahead of their MFMAs; sched_barriers keep hipcc from
    // hoisting all 24 reads (96 VGPRs) to the top
    auto kfrag = [&](int dc, int kb) {
      const int c = dc * 4 + g;
      return *(const bf16x8_t QIE_LDS*)(kt + (kb * 16 + fr) * (kC * 2) + (((c & ~15) | ((c ^ fr) & 15)) << 4));
    };
    bf16x8_t kf[2][2];
    kf[0][0] = kfrag(0, 0);
    kf[0][1] = kfrag(0, 1);
#pragma unroll
    for (int dc = 0; dc < 12; ++dc) {
      if (dc + 1 < 12) {
        kf[(dc + 1) & 1][0] = kfrag(dc + 1, 0);
        kf[(dc + 1) & 1][1] = kfrag(dc + 1, 1);
      }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int qb = 0; qb < kQB; ++qb)
          sc[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[dc & 1][kb], qf[qb][dc], sc[kb][qb], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // online softmax (log2 units); keys past kend masked
    const int key0 = kbeg + s * kKB;
    float t[2][kQB][4];
    bool grow = false;
    float mnew[kQB];
#pragma unroll
    for (int qb = 0; qb < kQB; ++qb) {
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = key0 + kb * 16 + 4 * g + r;
          const float v = key < kend ? sc[kb][qb][r] * cscale : -INFINITY;
          t[kb][qb][r] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      mnew[qb] = fmaxf(m[qb], mx);
      grow |= mnew[qb] > m[qb] + 8.0f;
    }
    if (__builtin_amdgcn_ballot_w64(grow)) {  // re-base: rare after the first steps
#pragma unroll
      for (int qb = 0; qb < kQB; ++qb) {
        const float a = m[qb] == -INFINITY ? 0.f : exp2f(m[qb] - mnew[qb]);
        const bool up = mnew[qb] > m[qb] + 8.0f;
        const float alpha = up ? a : 1.0f;
        if (up) m[qb] = mnew[qb];
        l[qb] *= alpha;
#pragma unroll
        for (int db = 0; db < 24; ++db) o[db][qb] *= alpha;
      }
    }
    bf16x8_t pf[kQB];
#pragma unroll
    for (int qb = 0; qb < kQB; ++qb) {
      float p[8];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) p[kb * 4 + r] = m[qb] == -INFINITY ? 0.f : exp2f(t[kb][qb][r] - m[qb]);
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) sum += p[k];
      l[qb] += sum;
      const uint32_t w4[4] = {pack2(p[0], p[1]), pack2(p[2], p[3]), pack2(p[4], p[5]), pack2(p[6], p[7])};
      pf[qb] = __builtin_bit_cast(bf16x8_t, u32x4_t{w4[0], w4[1], w4[2], w4[3]});
    }
    // O^T += V^T . P^T, V^T fragments two channel blocks ahead
    auto vfrag = [&](int db) {
      const char QIE_LDS* vrow = vtt + (db * 16 + fr) * (kKB * 2);
      const int sw = (fr >> 2) & 3;
      const u32x2_t lo = *(const u32x2_t QIE_LDS*)(vrow + (((g >> 1) ^ sw) << 4) + ((g & 1) << 3));
      const u32x2_t hi = *(const u32x2_t QIE_LDS*)(vrow + (((2 + (g >> 1)) ^ sw) << 4) + ((g & 1) << 3));
      return __builtin_bit_cast(bf16x8_t, u32x4_t{lo.x, lo.y, hi.x, hi.y});
    };
    bf16x8_t vf[3];
    vf[0] = vfrag(0);
    vf[1] = vfrag(1);
#pragma unroll
    for (int db = 0; db < 24; ++db) {
      if (db + 2 < 24) vf[(db + 2) % 3] = vfrag(db + 2);
#pragma unroll
      for (int qb = 0; qb < kQB; ++qb) va_mma(o[db][qb], vf[db % 3], pf[qb]);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (pre) va_wait_barrier<kPieces>();
    else va_wait_barrier<0>();
  }

  // partials: O^T lane = query fr, channels db*16 + 4g .. +3; (m, l) by the g == 0 lanes. The last
  // asm MFMAs' results are read by VALU / stores: 23 wait states, then every accumulator redefined
  asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");
  redefine_o();
#pragma unroll
  for (int qb = 0; qb < kQB; ++qb) {
    float lt = l[qb];
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    const int q = q0 + qb * 16 + fr;
    if (q < P) {
      float* orow = opart + ((int64_t)split * P + q) * kC + 4 * g;
#pragma unroll
      for (int db = 0; db < 24; ++db) *(f32x4_t*)(orow + db * 16) = o[db][qb];
      if (g == 0) *(float2*)(mlpart + ((int64_t)split * P + q) * 2) = float2{m[qb], lt};
    }
  }
}

// out[q][d] = bf16(sum_s O_s[q][d] 2^(m_s - m) / sum_s l_s 2^(m_s - m)), m = max_s m_s; 4 channels
// per thread
__global__ void __launch_bounds__(256)
    vae_attn_combine_kernel(const float* __restrict__ opart, const float* __restrict__ mlpart, int P, int nsplit,
                            bf16_t* __restrict__ out, int ldo) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)P * (kC / 4)) return;
  const int q = (int)(i / (kC / 4)), d = (int)(i - (int64_t)q * (kC / 4)) * 4;
  float mx = -INFINITY;
  for (int s = 0; s < nsplit; ++s) mx = fmaxf(mx, mlpart[((int64_t)s * P + q) * 2]);
  float den = 0.f, acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < nsplit; ++s) {
    const float ms = mlpart[((int64_t)s * P + q) * 2], ls = mlpart[((int64_t)s * P + q) * 2 + 1];
    if (ms == -INFINITY) continue;
    const float w = exp2f(ms - mx);
    den = __builtin_fmaf(ls, w, den);
    const f32x4_t v = *(const f32x4_t*)(opart + ((int64_t)s * P + q) * kC + d);
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = __builtin_fmaf(v[k], w, acc[k]);
  }
  const float inv = den > 0.f ? 1.0f / den : 0.f;
  *(u32x2_t*)(out + (int64_t)q * ldo + d) = u32x2_t{pack2(acc[0] * inv, acc[1] * inv), pack2(acc[2] * inv, acc[3] * inv)};
}

// key-range splits: enough workgroups for the CUs (two at 16384 pixels), at most 4
int va_splits(int P, int& kspan) {
  const int qblocks = (P + 127) / 128, ksteps = (P + kKB - 1) / kKB;
  int n = qblocks >= 256 ? 1 : (256 + qblocks - 1) / qblocks;
  n = std::max(1, std::min(std::min(n, 4), ksteps));
  kspan = (ksteps + n - 1) / n * kKB;
  return (P + kspan - 1) / kspan;
}

}  // namespace

static int64_t va_workspace(int P) {
  int kspan;
  const int n = va_splits(P, kspan);
  return (int64_t)n * P * (kC + 2) * 4;
}

extern "C" int qie_vae_attention_workspace(int P, int C, int64_t* bytes) {
  QIE_CHECK_ARG(bytes && P > 0 && C == kC);
  *bytes = va_workspace(P);
  return QIE_OK;
}

extern "C" int qie_vae_attention_bf16(const void* qkv, int64_t ldqkv, const void* vt, int64_t ldvt, int P, int C,
                                      void* out, int64_t ldo, void* workspace, int64_t workspace_bytes,
                                      qie_stream_t stream) {
  QIE_CHECK_ARG(qkv && vt && out && workspace && P > 0 && C == kC);
  QIE_CHECK_ARG(ldqkv >= 3 * C && ldqkv % 8 == 0 && ldvt >= (P + kKB - 1) / kKB * kKB && ldvt % 8 == 0 && ldo % 4 == 0);
  QIE_CHECK_ARG(((uintptr_t)qkv % 16) == 0 && ((uintptr_t)vt % 16) == 0 && ((uintptr_t)out % 8) == 0 &&
                ((uintptr_t)workspace % 16) == 0);
  QIE_CHECK_ARG((int64_t)P * ldqkv * 2 < (1ll << 31) && (int64_t)C * ldvt * 2 < (1ll << 31));
  QIE_CHECK_ARG(workspace_bytes >= va_workspace(P));
  int kspan;
  const int nsplit = va_splits(P, kspan);
  float* opart = (float*)workspace;
  float* ml = opart + (int64_t)nsplit * P * kC;
  const hipStream_t s = (hipStream_t)stream;
  const float cscale = 1.4426950408889634f / sqrtf((float)C);
  vae_attn_kernel<<<dim3((P + 127) / 128, nsplit), kNW * 64, 0, s>>>((const bf16_t*)qkv, P, (int)ldqkv, (const bf16_t*)vt,
                                                                (int)ldvt, kspan, opart, ml, cscale);
  const int64_t n = (int64_t)P * (kC / 4);
  vae_attn_combine_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(opart, ml, P, nsplit, (bf16_t*)out, (int)ldo);
  return qie_last_error();
}
