// Diagnostic harness (not part of the product): builds the ping-pong attention kernel with
// s_memtime stamps around its phases and prints average cycles per tile per group.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DQIE_ATTN_STAMP -Iinclude \
//         tools/attn_stamp.hip -o tools/attn_stamp && ./tools/attn_stamp
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../qwen_image_edit_streamdiffusion_amd/csrc/attention.hip"

int main() {
  const int B = 2, H = 24, S_IMG = 8192, S_TXT = 216, S = S_IMG + S_TXT;
  const int s_pad = ((S + 255) / 256) * 256;
  const size_t n = (size_t)3 * B * H * s_pad * 128;
  std::vector<unsigned short> h(n);
  srand(1);
  for (size_t i = 0; i < n; ++i) {
    float f = ((rand() & 0xffff) / 32768.0f - 1.0f);
    unsigned int u;
    std::memcpy(&u, &f, 4);
    h[i] = (unsigned short)(u >> 16);
  }
  void *qkv, *oi, *ot;
  hipMalloc(&qkv, n * 2);
  hipMalloc(&oi, (size_t)B * S_IMG * H * 128 * 2);
  hipMalloc(&ot, (size_t)B * S_TXT * H * 128 * 2);
  hipMemcpy(qkv, h.data(), n * 2, hipMemcpyHostToDevice);
  int kv[2] = {S, S};
  for (int it = 0; it < 5; ++it)
    qie_attention_fwd_bf16(qkv, B, H, s_pad, kv, oi, ot, S_IMG, S_TXT, 0.0883883f, nullptr);
  hipDeviceSynchronize();
  unsigned long long z[2][6] = {};
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), z, sizeof(z));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  qie_attention_fwd_bf16(qkv, B, H, s_pad, kv, oi, ot, S_IMG, S_TXT, 0.0883883f, nullptr);
  hipEventRecord(b);
  hipDeviceSynchronize();
  float ms;
  hipEventElapsedTime(&ms, a, b);
  unsigned long long st[2][6];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamp), sizeof(st));
  printf("attention %.3f ms (stamped build)\n", ms);
  for (int g = 0; g < 2; ++g) {
    const double nt = (double)st[g][3];
    printf("group %d: tiles %.0f  M-body %.0f  M-end wait+barrier %.0f  V-phase %.0f  cycles/tile (s_memtime)\n",
           g, nt, st[g][0] / nt, st[g][1] / nt, st[g][2] / nt);
  }
  // the model's path: q pre-scaled by scale * log2(e), qie_attention_fwd_log2q_bf16
  const size_t qn = (size_t)B * H * s_pad * 128;
  for (size_t i = 0; i < qn; ++i) {
    unsigned int u = (unsigned int)h[i] << 16;
    float f;
    std::memcpy(&f, &u, 4);
    f *= 0.0883883f * 1.44269504f;
    std::memcpy(&u, &f, 4);
    h[i] = (unsigned short)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
  }
  hipMemcpy(qkv, h.data(), qn * 2, hipMemcpyHostToDevice);
  for (int it = 0; it < 5; ++it) qie_attention_fwd_log2q_bf16(qkv, B, H, s_pad, kv, oi, ot, S_IMG, S_TXT, nullptr, 0, nullptr);
  hipDeviceSynchronize();
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), z, sizeof(z));
  hipEventRecord(a);
  qie_attention_fwd_log2q_bf16(qkv, B, H, s_pad, kv, oi, ot, S_IMG, S_TXT, nullptr, 0, nullptr);
  hipEventRecord(b);
  hipDeviceSynchronize();
  hipEventElapsedTime(&ms, a, b);
  hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamp), sizeof(st));
  printf("attention log2q %.3f ms (stamped build)\n", ms);
  for (int g = 0; g < 2; ++g) {
    const double nt = (double)st[g][3];
    printf("group %d: tiles %.0f  M-body %.0f  M-end wait+barrier %.0f  V-phase %.0f  cycles/tile (s_memtime)\n",
           g, nt, st[g][0] / nt, st[g][1] / nt, st[g][2] / nt);
  }
  return 0;
}
