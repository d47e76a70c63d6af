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
// Structure (gfx950): one workgroup = 8 waves = 256 query rows of one (b, h);
// each wave owns 32 query rows.  Per 64-key tile:
//   S^T = K . Q^T      (mfma 32x32x16 bf16, K rows by ds_read_b128 from an
//                       XOR-swizzled LDS image, Q^T held in registers)
//   -> each lane owns one query row: online softmax (running max / sum, exp2)
//      is lane-local except for one max exchange with the partner half-wave
//   O^T += V^T . P^T   (the S^T accumulator registers ARE the P^T operand,
//                       cdna_hip_programming.md §3 "accumulator as operand";
//                       V^T fragments by ds_read_b64_tr_b16 with the matching
//                       permuted key order)
// K/V tiles are double buffered in LDS and register-staged: the next tile's
// global loads are issued before the MFMAs and written after them (T14).
// Workgroups of one (b, h) are placed on one XCD so its K/V stream from L2.
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
  QieBatchI kv_len;
};

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

__global__ void __launch_bounds__(512) attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char smem_raw[4 * kTileBytes];  // K0 V0 K1 V1
  char QIE_LDS* smem = (char QIE_LDS*)smem_raw;

  const int nwg = a.qblocks * a.H * a.B;
  const int wgid = xcd_remap(blockIdx.x, nwg);
  const int qb = wgid % a.qblocks;
  const int bh = wgid / a.qblocks;
  const int h = bh % a.H, b = bh / a.H;

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int hf = lane >> 5;   // half-wave
  const int ql = lane & 31;   // query row within the wave / d column
  const int64_t plane = (int64_t)a.s_pad * kDh;
  const bf16_t* Qp = a.qkv + ((int64_t)(0 * a.B + b) * a.H + h) * plane;
  const bf16_t* Kp = a.qkv + ((int64_t)(1 * a.B + b) * a.H + h) * plane;
  const bf16_t* Vp = a.qkv + ((int64_t)(2 * a.B + b) * a.H + h) * plane;
  const int kv_len = a.kv_len.v[b];
  const int ntiles = (kv_len + kKB - 1) / kKB;

  // ---- Q^T fragments (B operand): lane (q, hf) element j = Q[q][16ks + 8hf + j]
  const int q_row = qb * kQB + wave * 32 + ql;
  bf16x8_t qf[8];
  {
    const bf16_t* qr = Qp + (int64_t)q_row * kDh + 8 * hf;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = *(const bf16x8_t*)(qr + 16 * ks);
  }

  // ---- staging: each thread moves 2 K chunks + 2 V chunks (16 B) per tile
  u32x4_t stK[2], stV[2];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + 512 * i;
      const int row = id >> 4, ch = id & 15;
      const int64_t off = (int64_t)(t * kKB + row) * kDh + ch * 8;
      stK[i] = *(const u32x4_t*)(Kp + off);
      stV[i] = *(const u32x4_t*)(Vp + off);
    }
  };
  auto lwrite = [&](int buf) {
    char QIE_LDS* kb = smem + buf * 2 * kTileBytes;
    char QIE_LDS* vb = kb + kTileBytes;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + 512 * i;
      const int row = id >> 4, ch = id & 15;
      *(u32x4_t QIE_LDS*)(kb + row * 256 + ((ch ^ (row & 15)) << 4)) = stK[i];
      *(u32x4_t QIE_LDS*)(vb + row * 256 + ((ch ^ ((row & 3) << 2)) << 4)) = stV[i];
    }
  };

  gload(0);
  lwrite(0);
  __syncthreads();
  // Drain every outstanding load (Q fragments included) with a waitcnt the
  // compiler's scoreboard sees: otherwise it keeps Q "pending" into the loop and
  // waits on the in-order vmcnt there -- i.e. on the NEXT tile's prefetch,
  // exposing the full global-load latency every tile.
  __builtin_amdgcn_s_waitcnt(0);

  f32x16_t o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = f32x16_t{};
  float m_run = -INFINITY, l_run = 0.f;
  const float c = a.c;

  // per-lane LDS offsets
  const int ksw = lane & 15;                        // K swizzle term (row & 15)
  const int tri = lane & 15;                        // lane within 16-lane group
  const int tr_row = (tri >> 2);                    // row within 4-row block
  const int tr_sw = tr_row << 2;                    // V swizzle term ((row & 3) << 2)
  const int tr_g1 = (lane >> 4) & 1;
  const int tr_cb = 8 * (tri & 1);                  // byte within 16-B chunk

  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) gload(t + 1);
    const char QIE_LDS* kb = smem + cur * 2 * kTileBytes;
    const char QIE_LDS* vb = kb + kTileBytes;

    // ---- S^T = K Q^T : two 32-key blocks
    f32x16_t s[2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      s[cb] = f32x16_t{};
      const char QIE_LDS* krow = kb + (cb * 32 + ql) * 256;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const bf16x8_t kf = *(const bf16x8_t QIE_LDS*)(krow + (((2 * ks + hf) ^ ksw) << 4));
        s[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s[cb], 0, 0, 0);
      }
    }
    // ---- mask keys >= kv_len (only the last tile can contain them)
    const int kv0 = t * kKB;
    if (kv0 + kKB > kv_len) {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kv = kv0 + cb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf;
          if (kv >= kv_len) s[cb][r] = -INFINITY;
        }
    }
    // ---- online softmax (lane-local row; partner half holds the other 32 keys)
    float mx = s[0][0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s[0][r]);
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[1][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    // lazy rescale (cdna_hip_programming.md T13): keep the running max unless a
    // row of this wave grows by more than kRescaleThr (log2 units); P is then
    // bounded by 2^kRescaleThr.  The decision covers this tile before any of its
    // P is formed, and the previous tile's P.V is complete.
    if (__any((mx - m_run) * c > kRescaleThr)) {
      const float m_new = fmaxf(m_run, mx);
      const float alpha = __builtin_amdgcn_exp2f((m_run - m_new) * c);
      m_run = m_new;
      l_run *= alpha;
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db] *= alpha;
    }
    const float mc = m_run * c;
    float psum = 0.f;
    bf16x8_t pf[4];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[cb][r], c, -mc));
        psum += p;
        pf[cb * 2 + (r >> 3)][r & 7] = (__bf16)p;
      }
    l_run += psum;

    // ---- O^T += V^T P^T
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int r0 = 16 * ks + 4 * hf + tr_row;   // rows r0 and r0 + 8
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int chunk = (4 * db + 2 * tr_g1 + ((tri & 3) >> 1)) ^ tr_sw;
        const char QIE_LDS* p0 = vb + r0 * 256 + (chunk << 4) + tr_cb;
        const s16x4_t va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4_t QIE_LDS*)p0);
        const s16x4_t vb2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4_t QIE_LDS*)(p0 + 8 * 256));
        typedef __attribute__((ext_vector_type(8))) short s16x8_t;
        const s16x8_t vv = __builtin_shufflevector(va, vb2, 0, 1, 2, 3, 4, 5, 6, 7);
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, vv), pf[ks],
                                                        o[db], 0, 0, 0);
      }
    }
    if (t + 1 < ntiles) lwrite(cur ^ 1);
    __syncthreads();
  }

  // ---- normalise and store: lane (q, hf) holds d = 32db + 8g + 4hf + (0..3)
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = 1.0f / l_tot;
  const int s = q_row;
  bf16_t* dst = nullptr;
  if (s < a.s_img) {
    dst = a.out_img + ((int64_t)b * a.s_img + s) * (a.H * kDh) + h * kDh;
  } else if (s < a.s_img + a.txt_rows) {
    dst = a.out_txt + ((int64_t)b * a.txt_rows + (s - a.s_img)) * (a.H * kDh) + h * kDh;
  }
  if (dst) {
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * db + 8 * g + 4 * hf;
        const u32x2_t w = {pack2(o[db][4 * g] * inv, o[db][4 * g + 1] * inv),
                           pack2(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv)};
        *(u32x2_t*)(dst + d) = w;
      }
  }
}

}  // namespace

extern "C" int qie_attention_fwd_bf16(const void* qkv, int batch, int heads, int s_pad,
                                      const int* kv_len_host, void* out_img, void* out_txt,
                                      int s_img, int txt_rows, float scale, qie_stream_t stream) {
  QIE_CHECK_ARG(qkv && kv_len_host && out_img && (out_txt || txt_rows == 0));
  QIE_CHECK_ARG(batch > 0 && batch <= QIE_MAX_BATCH && heads > 0);
  QIE_CHECK_ARG(s_pad > 0 && s_pad % kQB == 0 && s_img >= 0 && txt_rows >= 0);
  QIE_CHECK_ARG(s_img + txt_rows <= s_pad);
  AttnArgs a{};
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
  const int nwg = a.qblocks * heads * batch;
  attn_fwd_kernel<<<nwg, 512, 0, (hipStream_t)stream>>>(a);
  return qie_last_error();
}
