/*
 * qie.h -- C ABI of libqie.so, the MI355X (gfx950) hot-path kernels of the
 * Qwen-Image-Edit-2509 denoise loop (DiT forward + batched CFG + stream batch).
 *
 * The reference (shi3z/Qwen-Image-Edit-StreamDiffusion) has no native code: its
 * hot path is the un-vendored diffusers QwenImageEditPlusPipeline /
 * QwenImageTransformer2DModel [U], called at server.py:137-153,
 * qwen_realtime.py:247-255 and benchmark_lightning.py:41-49, and swapped as a
 * module at benchmark_compile.py:102-106 (`pipeline.transformer = ...`).  Each
 * entry point below names the upstream operation it replaces inside that call.
 *
 * Conventions:
 *   - bf16 tensors are raw 16-bit words; every pointer is device memory owned by
 *     the caller (PyTorch caching allocator).  The library never allocates,
 *     frees or synchronises, and keeps no mutable global state.
 *   - `stream` is a hipStream_t (the caller's current stream), passed as void*.
 *   - per-batch scalars (`*_host` arrays, <= QIE_MAX_BATCH entries) are read on
 *     the host at launch time and passed to the kernel by value.
 *   - return 0 on success, QIE_ERR_* (< 0) on a rejected argument, or a
 *     positive hipError_t when the launch itself failed.
 *   - re-entrant; one caller thread per process (server.py:39 single worker).
 */
#ifndef QIE_H_
#define QIE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QIE_ABI_VERSION 2
#define QIE_MAX_BATCH 16

#define QIE_OK 0
#define QIE_ERR_INVALID (-1)     /* bad shape / stride / alignment / null pointer */
#define QIE_ERR_UNSUPPORTED (-2) /* valid but not implemented for these sizes */

#define QIE_ACT_NONE 0
#define QIE_ACT_GELU_TANH 1

typedef void* qie_stream_t; /* hipStream_t */

int qie_abi_version(void);
const char* qie_strerror(int code);

/* ------------------------------------------------------------------ linears
 * All linears compute y = x[M,K] . W[N,K]^T + bias[N] with bf16 operands, fp32
 * MFMA accumulation and one rounding of (acc + bias) to bf16 (nn.Linear in
 * bf16).  K % 64 == 0, N % 4 == 0, 16-byte aligned rows.
 */

/* nn.Linear (+ FeedForward GELU(approximate="tanh")) [U]:
 * attn.to_q/k/v, add_*_proj, img_mlp.net.0.proj (act=GELU), img_in, txt_in,
 * proj_out.  y = act(bf16(acc + bias)) -> bf16. */
int qie_linear_bf16(const void* x, int64_t ldx, const void* w, const void* bias, void* y,
                    int64_t ldy, int M, int N, int K, int act, qie_stream_t stream);

/* attn.to_out[0] / to_add_out / *_mlp.net.2 followed by the block's
 * gated residual `hidden = hidden + gate * out` [U] (QwenImageTransformerBlock):
 * resid[m,n] = bf16(resid + bf16(gate[b(m),n] * bf16(acc + bias))),
 * b(m) = m / rows_per_batch, gate row stride gate_bstride (elements). */
int qie_linear_gated_residual_bf16(const void* x, int64_t ldx, const void* w, const void* bias,
                                   const void* gate, int64_t gate_bstride, int rows_per_batch,
                                   void* resid, int64_t ldr, int M, int N, int K,
                                   qie_stream_t stream);

/* Fused: to_q|to_k|to_v (or add_q|k|v_proj) as ONE GEMM over the packed
 * weight [3*H*Dh, K]; the epilogue scatters bf16(acc + bias) into the
 * head-major joint buffer qkv[3][batch][heads][s_pad][head_dim] at sequence
 * position seq_offset + (m % rows_per_batch) of batch m / rows_per_batch
 * (replaces the projections + unflatten + torch.cat of
 * QwenDoubleStreamAttnProcessor2_0 [U]). */
int qie_linear_qkv_bf16(const void* x, int64_t ldx, const void* w, const void* bias, void* qkv,
                        int M, int K, int rows_per_batch, int seq_offset, int batch, int heads,
                        int head_dim, int s_pad, qie_stream_t stream);

/* skinny linear for M <= 16 rows (img_mod/txt_mod Linear(3072->18432)
 * on SiLU(temb), timestep_embedder linears, norm_out.linear) [U]:
 * weight-bandwidth bound, y = bf16(acc + bias). */
int qie_gemv_bf16(const void* x, int64_t ldx, const void* w, const void* bias, void* y,
                  int64_t ldy, int M, int N, int K, qie_stream_t stream);

/* ------------------------------------------------------------------ norms */

/* nn.LayerNorm(elementwise_affine=False, eps) + _modulate [U]:
 * y = bf16(bf16(bf16(LN(x)) * bf16(1 + scale[b])) + shift[b]), fp32 statistics.
 * shift/scale rows are mod_bstride elements apart per batch. */
int qie_layernorm_modulate_bf16(const void* x, int64_t ldx, const void* shift, const void* scale,
                                int64_t mod_bstride, int rows_per_batch, void* y, int64_t ldy,
                                int rows, int D, float eps, qie_stream_t stream);

/* RMSNorm(D, eps, elementwise_affine=True) [U] (txt_norm):
 * y = bf16(bf16(x * rsqrt(mean(x^2) + eps)) * w). */
int qie_rmsnorm_bf16(const void* x, const void* w, void* y, int rows, int D, float eps,
                     qie_stream_t stream);

/* attn.norm_q/norm_k (or norm_added_q/k) RMSNorm(head_dim) followed by
 * apply_rotary_emb_qwen(use_real=False) [U], in place on sequence rows
 * [seg_start, seg_start + seg_len) of the Q and K planes of the joint buffer.
 * cos_tab/sin_tab: fp32 [seg_len][head_dim/2] rows for that segment.
 * q_scale multiplies the rotated q rows before their single bf16 rounding (1.0: the plain op;
 * scale * log2(e) feeds qie_attention_fwd_log2q_bf16); k rows are unscaled. */
int qie_qk_norm_rope_bf16(void* qkv, int batch, int heads, int head_dim, int s_pad, int seg_start,
                          int seg_len, const void* wq, const void* wk, const float* cos_tab,
                          const float* sin_tab, float eps, float q_scale, qie_stream_t stream);

/* Fused: the q|k|v projection of one stream (as qie_linear_qkv_bf16) followed by
 * attn.norm_q/norm_k (norm_added_q/k) RMSNorm(head_dim) and apply_rotary_emb_qwen [U] on its q
 * and k rows, with the rounding points of qie_qk_norm_rope_bf16. head_dim == 128; cos_tab /
 * sin_tab: fp32 [rows_per_batch][64] for this stream's segment. Big shapes run as ONE GEMM
 * whose epilogue normalises and rotates each head (the two halves of a head meet through LDS);
 * other shapes run the GEMM and then qie_qk_norm_rope_bf16. q_scale as there. */
int qie_linear_qkv_norm_rope_bf16(const void* x, int64_t ldx, const void* w, const void* bias, void* qkv,
                                  int M, int K, int rows_per_batch, int seq_offset, int batch, int heads,
                                  int head_dim, int s_pad, const void* wq, const void* wk,
                                  const float* cos_tab, const float* sin_tab, float eps,
                                  float q_scale, qie_stream_t stream);

/* ------------------------------------------------------------------ attention */

/* joint non-causal SDPA of QwenDoubleStreamAttnProcessor2_0 [U] over the
 * head-major joint buffer (head_dim 128).  Keys j >= kv_len_host[b] are masked
 * (batched CFG text padding).  Query row s of batch b is written to
 * out_img[(b*s_img + s)*heads*128 + h*128 + d] for s < s_img and to
 * out_txt[(b*txt_rows + s - s_img)*...] for s_img <= s < s_img + txt_rows.
 * s_pad % 256 == 0.  scale = 1/sqrt(head_dim) in the reference. */
int qie_attention_fwd_bf16(const void* qkv, int batch, int heads, int s_pad,
                           const int* kv_len_host, void* out_img, void* out_txt, int s_img,
                           int txt_rows, float scale, qie_stream_t stream);

/* Same attention with the LAST 256-row query block of every (batch, head) computed as
 * QIE_ATTN_SPLIT key ranges. Each range writes its fp32 partial (unnormalised O, row max, row
 * sum) to `workspace`, then a combine kernel merges them. These blocks are dispatched after the
 * others so they fill the grid's final, otherwise mostly idle, round. At 1024^2 there are
 * 32 * 24 * B full blocks: a multiple of the 256 CUs. The split depends only on the block
 * index, so every row's arithmetic is independent of the batch size.
 * qie_attention_workspace_bytes returns the bytes needed in *bytes (0: no split for this
 * shape); a workspace smaller than that returns QIE_ERR_INVALID. */
#define QIE_ATTN_SPLIT 5
int qie_attention_workspace_bytes(int batch, int heads, int s_pad, int s_img, int txt_rows,
                                  int64_t* bytes);
int qie_attention_fwd_split_bf16(const void* qkv, int batch, int heads, int s_pad,
                                 const int* kv_len_host, void* out_img, void* out_txt, int s_img,
                                 int txt_rows, float scale, void* workspace,
                                 int64_t workspace_bytes, qie_stream_t stream);

/* The same SDPA for a q plane that already holds q * scale * log2(e) -- the producers fold that
 * factor in before their single bf16 rounding (q_scale of qie_qk_norm_rope_bf16 /
 * qie_linear_qkv_norm_rope_*). The logits then come out of the MFMA in log2 units, offset by
 * the running max (the first MFMA's C operand), and the softmax skips one multiply-add per
 * score. workspace may be NULL (no split); otherwise as qie_attention_fwd_split_bf16. */
int qie_attention_fwd_log2q_bf16(const void* qkv, int batch, int heads, int s_pad,
                                 const int* kv_len_host, void* out_img, void* out_txt, int s_img,
                                 int txt_rows, void* workspace, int64_t workspace_bytes,
                                 qie_stream_t stream);

/* ------------------------------------------------------------------ small ops */

/* Timesteps(dim, flip_sin_to_cos=True, downscale_freq_shift=0,
 * scale=1000) [U]: t bf16 [batch] -> bf16 [batch, dim] = [cos | sin]. */
int qie_timestep_embed_bf16(const void* t, void* out, int batch, int dim, qie_stream_t stream);

/* nn.SiLU on a bf16 vector (temb -> SiLU(temb) feeding every *_mod Linear). */
int qie_silu_bf16(const void* x, void* y, int64_t n, qie_stream_t stream);

/* true-CFG combine + per-token norm rescale of the Edit-Plus pipeline
 * [U]: comb = u + s*(c-u); out = comb*(|c|/|comb|), all bf16
 * tensor ops, norms over the last dim C (fp32 accumulate).  Each of the `batch`
 * slices is [rows][C] contiguous; slices are *_bstride elements apart. */
int qie_cfg_combine_bf16(const void* cond, int64_t cond_bstride, const void* uncond,
                         int64_t uncond_bstride, void* out, int64_t out_bstride, int batch, int rows,
                         int C, float scale, qie_stream_t stream);

/* FlowMatchEulerDiscreteScheduler.step [U] with per-batch-row dt
 * (stream batch: each row at its own sigma): out = bf16(x + bf16(dt[b] * v)).
 * Tensors are [batch][n] with independent batch strides (elements). */
int qie_euler_step_bf16(const void* x, int64_t x_bstride, const void* v, int64_t v_bstride,
                        void* out, int64_t out_bstride, int batch, int64_t n,
                        const float* dt_host, qie_stream_t stream);

/* strided batch copy of bf16 rows (latents / cond latents into the model input) */
int qie_copy_bf16(const void* src, int64_t src_bstride, void* dst, int64_t dst_bstride, int batch,
                  int64_t n, qie_stream_t stream);

/* _pack_latents / _unpack_latents [U]: [B,C,H,W] <-> [B,(H/2)(W/2),4C]. */
int qie_pack_latents_bf16(const void* x, void* y, int batch, int C, int H, int W,
                          qie_stream_t stream);
int qie_unpack_latents_bf16(const void* x, void* y, int batch, int C, int H, int W,
                            qie_stream_t stream);

/* ------------------------------------------------------------------ int8
 * Int8Linear (README.md:136-141, absent from the snapshot; bnb LLM.int8 at
 * benchmark_int8.py:72-76 is the reference's int8 semantics): W8A8 with
 * per-output-channel weight scales and per-token dynamic activation scales,
 * i8 MFMA with int32 accumulation, fp32 dequant epilogue (oracle/int8_ref.py). */

/* per-row symmetric quantisation: q = clamp(rint(x*127/amax)), scale = amax/127 */
int qie_quantize_rows_i8(const void* x, int64_t ldx, void* q, int64_t ldq, float* scale, int rows,
                         int D, qie_stream_t stream);

/* Fused LayerNorm + quantisation prologue: LayerNorm+modulate as above, emitted as
 * int8 rows + fp32 per-row scales (the bf16 value is quantised). */
int qie_layernorm_modulate_i8(const void* x, int64_t ldx, const void* shift, const void* scale,
                              int64_t mod_bstride, int rows_per_batch, void* q, int64_t ldq,
                              float* qscale, int rows, int D, float eps, qie_stream_t stream);

/* int8 linears: y = epilogue(bf16(fma(float(acc), sx[m]*sw[n], bias[n]))),
 * K % 128 == 0; same epilogues as the bf16 family. */
int qie_linear_i8(const void* xq, int64_t ldx, const float* sx, const void* wq, const float* sw,
                  const void* bias, void* y, int64_t ldy, int M, int N, int K, int act,
                  qie_stream_t stream);
int qie_linear_gated_residual_i8(const void* xq, int64_t ldx, const float* sx, const void* wq,
                                 const float* sw, const void* bias, const void* gate,
                                 int64_t gate_bstride, int rows_per_batch, void* resid,
                                 int64_t ldr, int M, int N, int K, qie_stream_t stream);
int qie_linear_qkv_i8(const void* xq, int64_t ldx, const float* sx, const void* wq,
                      const float* sw, const void* bias, void* qkv, int M, int K,
                      int rows_per_batch, int seq_offset, int batch, int heads, int head_dim,
                      int s_pad, qie_stream_t stream);

/* qie_linear_qkv_norm_rope_bf16 on the int8 linear (dequant epilogue as qie_linear_qkv_i8),
 * q_scale as there. */
int qie_linear_qkv_norm_rope_i8(const void* xq, int64_t ldx, const float* sx, const void* wq,
                                const float* sw, const void* bias, void* qkv, int M, int K,
                                int rows_per_batch, int seq_offset, int batch, int heads, int head_dim,
                                int s_pad, const void* nq, const void* nk, const float* cos_tab,
                                const float* sin_tab, float eps, float q_scale, qie_stream_t stream);

/* ---- split-K linears for short-M shapes (the text stream, M = B * S_txt) ---------------------
 * Replaces the same diffusers linears as the entry points above (text-stream add_q/k/v_proj,
 * to_add_out, txt_mlp: transformer_qwenimage.py [U]) for shapes whose
 * output tiles cannot fill the chip (M = 432 gives 96 tiles for N = 3072). K is cut into
 * `splits` equal ranges (K must be a multiple of splits * 64 bf16 / splits * 128 int8). Each
 * range writes its partial sums to `workspace`, and a second kernel adds them in range order
 * and applies the epilogue described by `epi`.
 *   - workspace: caller-owned, >= splits * M * N * 4 bytes. Partials are fp32 for bf16 and
 *     int32 for int8, so the int8 result is bitwise the unsplit one.
 *   - The per-row arithmetic depends only on (K, splits), never on M, so rows stay batch
 *     independent (batched CFG == sequential).
 *   - splits == 1: one launch of 256x256 tiles with the epilogue applied directly (no partials,
 *     no reduce; workspace may be NULL) -- the least CU-time per output, for launches that run
 *     beside the image stream on a second HIP stream. */
#define QIE_EPI_BIAS 0           /* y = bf16(x.W^T + b)                                        */
#define QIE_EPI_GELU 1           /* y = gelu_tanh(bf16(x.W^T + b))                             */
#define QIE_EPI_GATED_RESIDUAL 2 /* resid += bf16(gate[row/rows_per_batch] * bf16(x.W^T + b)) */
#define QIE_EPI_QKV 3            /* scatter into qkv[3][batch][heads][s_pad][head_dim]         */

typedef struct qie_epilogue {
  int kind;              /* QIE_EPI_* */
  void* out;             /* y (BIAS, GELU) / resid (GATED_RESIDUAL, in place) / qkv (QKV) */
  int64_t ldo;           /* row stride of y / resid in elements (unused for QKV) */
  const void* gate;      /* GATED_RESIDUAL: bf16 [batch][gate_bstride] */
  int64_t gate_bstride;
  int rows_per_batch;    /* GATED_RESIDUAL, QKV */
  int seq_offset;        /* QKV, as qie_linear_qkv_bf16 */
  int batch;
  int heads;
  int head_dim;
  int s_pad;
} qie_epilogue_t;

int qie_linear_splitk_bf16(const void* x, int64_t ldx, const void* w, const void* bias,
                           const qie_epilogue_t* epi, int M, int N, int K, int splits,
                           void* workspace, int64_t workspace_bytes, qie_stream_t stream);
int qie_linear_splitk_i8(const void* xq, int64_t ldx, const float* sx, const void* wq,
                         const float* sw, const void* bias, const qie_epilogue_t* epi, int M,
                         int N, int K, int splits, void* workspace, int64_t workspace_bytes,
                         qie_stream_t stream);

/* ------------------------------------------------------------------ VAE decoder
 * AutoencoderKLQwenImage.decode on one frame [U] (pipeline_qwenimage_edit_plus: unpack,
 * `latents / (1/std) + mean`, vae.decode(z)[:, :, 0], postprocess). On a single frame every
 * QwenImageCausalConv3d sees two zero frames of causal padding, so it is the 2-D convolution
 * with the last temporal slice of its kernel; Resample "upsample3d" skips its time_conv on the
 * first frame. Activations are NHWC bf16 [pixels][C]. */

/* 3x3 or 1x1 convolution as an implicit GEMM: y[p][n] = bf16(sum_{tap,c} x[src(p, tap)][c]
 * * w[n][tap*C + c] + bias[n]) with the input gathered per tap (no im2col buffer). mode 0: same
 * size, pad ksize/2; 1: a nearest-2x upsample folded into the gather (decoder Resample, output
 * 2H x 2W); 2: stride 2 after ZeroPad2d((0,1,0,1)) (encoder Resample, output H/2 x W/2, 3x3).
 * w: [N][ldw] bf16, K order [ky][kx][C], zero-padded to ldw >= roundup(ksize^2 * C, 64).
 * resid != NULL (must equal y): y = bf16(y + bf16(acc + bias)) (ResidualBlock x + h).
 * C % 8 == 0, N % 4 == 0. */
int qie_conv2d_bf16(const void* x, int H_in, int W_in, int C, int mode, int ksize, const void* w, int64_t ldw,
                    const void* bias, const void* resid, void* y, int N, qie_stream_t stream);

/* qie_conv2d_bf16 (no residual) followed by QwenImageRMS_norm (+ SiLU when silu != 0) of its output
 * with `gamma` [N] (the VAE ResidualBlock's conv1 + norm2, the bf16 rounding points of
 * qie_vae_rms_norm_bf16): fused into the convolution's epilogue where one wave holds every output
 * channel of a pixel (N = 96 on the halo-tiled kernel), otherwise the two launches. The fused form
 * divides through a reciprocal with one correction step and sums the squares in another order, so
 * it agrees with the two-launch form to within one bf16 ulp, not bit for bit. */
int qie_conv2d_rmsnorm_bf16(const void* x, int H_in, int W_in, int C, int mode, int ksize, const void* w,
                            int64_t ldw, const void* bias, const void* gamma, int silu, void* y, int N,
                            qie_stream_t stream);

/* y[M][N] = x[M][K] . w[N][K]^T as raw fp32 (row strides ldx, ldw elements): attention scores of
 * the VAE mid-block QwenImageAttentionBlock (one head over H*W tokens). K % 64 == 0. */
int qie_matmul_f32out_bf16(const void* x, int64_t ldx, const void* w, int64_t ldw, float* y, int M, int N,
                           int K, qie_stream_t stream);

/* Packed latents [batch][(h/2)(w/2)][64] -> NHWC [batch][h][w][16]: _unpack_latents, then
 * z = bf16(bf16(l / sinv[c]) + mean[c]) (sinv = bf16(1/std), mean bf16), then post_quant_conv
 * y = bf16(pq_w[16][16] . z + pq_b). */
int qie_vae_latents_in_bf16(const void* packed, int batch, int h, int w, const void* sinv, const void* mean,
                            const void* pq_w, const void* pq_b, void* y, qie_stream_t stream);

/* QwenImageRMS_norm over the C channels of each pixel (F.normalize * sqrt(C) * gamma, bf16
 * rounding after each op), then SiLU when silu != 0. C % 8 == 0, C <= 512. */
int qie_vae_rms_norm_bf16(const void* x, const void* gamma, void* y, int64_t pixels, int C, int silu,
                          qie_stream_t stream);

/* Row softmax of fp32 scores: p = bf16(exp(scale * (s - max)) / sum) for columns < N, zero in
 * [N, ldp) (the K padding of the P.V GEMM). Row strides lds (floats), ldp (bf16); N % 4 == 0.
 * causal != 0: row r keeps only columns 0..r (the prompt encoder's decoder mask). */
int qie_softmax_rows_f32_bf16(const float* s, int64_t lds, void* p, int64_t ldp, int rows, int N, float scale,
                              int causal, qie_stream_t stream);

/* As qie_softmax_rows_f32_bf16 with row r restricted to keys [ranges[2r], ranges[2r+1]) (device
 * int32 pairs): the vision tower's block-diagonal masks -- windows of cu_window_seqlens and
 * per-image full attention of cu_seqlens (transformers Qwen2_5_VLVisionAttention's per-chunk
 * split), and (0, r + 1) for the language model's causal mask. Row r uses pair r % period
 * (head-batched score blocks of `period` rows). Columns outside the range are written 0 up to ldp. */
int qie_softmax_rows_ranged_f32_bf16(const float* s, int64_t lds, void* p, int64_t ldp, int rows, int N,
                                     float scale, const int* ranges_dev, int period, qie_stream_t stream);

/* Head-batched product (the prompt encoder's attention, all heads in one launch): for z < batch,
 * y_z = x_z . w_{z / group}^T with x_z = x + z*bsx, w_g = w + g*bsw, y_z = y + z*bsy (elements;
 * group > 1 = grouped-query attention sharing k / v). out_f32 = 1: raw fp32 [M][N], ldy == N
 * (scores); out_f32 = 0: bf16(x.w^T + bias) with row stride ldy (P.V into a head's columns). */
int qie_matmul_batched_bf16(const void* x, int64_t ldx, int64_t bsx, const void* w, int64_t ldw, int64_t bsw,
                            int group, const void* bias, void* y, int64_t ldy, int64_t bsy, int M, int N, int K,
                            int batch, int out_f32, qie_stream_t stream);

/* VAE mid-block attention (QwenImageAttentionBlock: one head of C = 384 channels over P latent
 * pixels; replaces the qie_matmul_f32out_bf16 + qie_softmax_rows_f32_bf16 + P.V chain the
 * reference's F.scaled_dot_product_attention stands for, diffusers autoencoder_kl_qwenimage [U]):
 * out[q] = softmax(q . k^T / sqrt(C)) . v for the q / k column blocks of the to_qkv rows
 * (qkv[p][0..C) and [C..2C), row stride ldqkv) and v given transposed, vt [C][ldvt] with
 * ldvt >= P rounded up to 32 and ZERO past P. Flash form: fp32 online softmax, scores never
 * stored; key ranges split over workgroups meet through `workspace` (>=
 * qie_vae_attention_workspace(P, C) bytes, 16-byte aligned). C must be 384. */
int qie_vae_attention_bf16(const void* qkv, int64_t ldqkv, const void* vt, int64_t ldvt, int P, int C, void* out,
                           int64_t ldo, void* workspace, int64_t workspace_bytes, qie_stream_t stream);
int qie_vae_attention_workspace(int P, int C, int64_t* bytes);

/* y[c][r] = x[r][c] for an R x C bf16 block (row strides ldx, ldy elements). */
int qie_transpose_bf16(const void* x, int64_t ldx, void* y, int64_t ldy, int R, int C, qie_stream_t stream);

/* Encoder input: uint8 RGB [pixels][3] -> bf16(2 v/255 - 1) (VaeImageProcessor.preprocess, then
 * .to(bf16)) as NHWC [pixels][8], channels 3..7 zero (the conv gather reads 8-channel chunks). */
int qie_vae_rgb_in(const void* rgb, void* y, int64_t pixels, qie_stream_t stream);

/* Encoder output: quant_conv result NHWC [batch][h][w][ldx] bf16 -> its mode (channels 0..15, the
 * DiagonalGaussian mean; retrieve_latents(sample_mode="argmax")) -> bf16(bf16(mu - mean) / std)
 * -> packed [batch][(h/2)(w/2)][64] (_encode_vae_image + _pack_latents). */
int qie_vae_latents_out_bf16(const void* x, int64_t ldx, int batch, int h, int w, const void* mean,
                             const void* stdv, void* packed, qie_stream_t stream);

/* Decoder output [pixels][ldx] bf16 (channels 0..2) -> clamp(-1, 1) -> (x/2 + 0.5).clamp(0, 1)
 * -> round(255 v) as uint8 RGB [pixels][3] (VaeImageProcessor.postprocess, output_type="pil"). */
int qie_vae_rgb_out(const void* x, int64_t ldx, void* rgb, int64_t pixels, qie_stream_t stream);

/* ------------------------------------------------------------------ prompt encoder
 * The Qwen2.5-VL language model of the prompt encoder (text_encoder, transformers
 * Qwen2_5_VLTextModel [U]); its projections / norms / attention products use the entry points
 * above (qie_linear*, qie_rmsnorm_bf16, qie_matmul_f32out_bf16, qie_softmax_rows_f32_bf16). */

/* out[i] = table[ids[i]] (embed_tokens), D % 8 == 0; ids are device int32, clamped to the vocab. */
int qie_embed_rows_bf16(const void* table, const int* ids_dev, int rows, int D, int vocab, void* out,
                        qie_stream_t stream);

/* Rotate-half RoPE in place on heads [h0, h0 + nh) of each row (rotary width head_dim, heads
 * head_stride elements apart -- the vision tower pads its 80-wide heads to 128 slots), per-row
 * tables [rows][head_dim] with the sections already merged on the host:
 *   tab_f32 = 0: bf16 tables, apply_multimodal_rotary_pos_emb in the activation dtype,
 *                x = bf16(bf16(x cos) + bf16(rotate_half(x) sin));
 *   tab_f32 = 1: fp32 tables, apply_rotary_pos_emb_vision (upcast), x = bf16(x cos + rot(x) sin). */
int qie_rope_half_bf16(void* x, int64_t ld, int rows, int h0, int nh, int head_dim, int head_stride,
                       const void* cos_tab, const void* sin_tab, int tab_f32, qie_stream_t stream);

/* nn.GELU() (erf form) in place on a bf16 [rows][n] block (row stride ld): the patch merger. */
int qie_gelu_erf_bf16(void* x, int64_t ld, int rows, int n, qie_stream_t stream);

/* Qwen2MLP gating: y = bf16(bf16(silu(g)) * u) with [g | u] = gu[r][0..F) | gu[r][F..2F). */
int qie_silu_mul_bf16(const void* gu, int64_t ldg, int rows, int F, void* y, int64_t ldy, qie_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* QIE_H_ */
