// Diagnostic harness (not part of the product): the ring GEMM with s_memtime stamps per K slice.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DQIE_GEMM_STAMP -Iinclude tools/gemm_stamp.hip -o tools/gemm_stamp
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../qwen_image_edit_streamdiffusion_amd/csrc/gemm.hip"

static void run(const char* name, int M, int N, int K) {
  std::vector<unsigned short> hx((size_t)M * K), hw((size_t)N * K);
  for (auto& v : hx) v = 0x3f80 ^ (rand() & 0x80ff);
  for (auto& v : hw) v = 0x3c00 ^ (rand() & 0x80ff);
  void *x, *w, *b, *y;
  hipMalloc(&x, hx.size() * 2);
  hipMalloc(&w, hw.size() * 2);
  hipMalloc(&b, N * 2);
  hipMalloc(&y, (size_t)M * N * 2);
  hipMemcpy(x, hx.data(), hx.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(w, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  hipMemset(b, 0, N * 2);
  for (int i = 0; i < 3; ++i) qie_linear_bf16(x, K, w, b, y, N, M, N, K, 0, nullptr);
  hipDeviceSynchronize();
  unsigned long long z[4] = {};
  hipMemcpyToSymbol(HIP_SYMBOL(g_gstamp), z, sizeof(z));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  qie_linear_bf16(x, K, w, b, y, N, M, N, K, 0, nullptr);
  hipEventRecord(e1);
  hipDeviceSynchronize();
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long st[4];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(g_gstamp), sizeof(st));
  printf("%s M=%d N=%d K=%d: %.3f ms (stamped)  per slice per wave: wait+barrier %.0f  total %.0f cycles  (%llu slices)\n",
         name, M, N, K, ms, (double)st[0] / st[2], (double)st[1] / st[2], st[2]);
  hipFree(x); hipFree(w); hipFree(b); hipFree(y);
}

int main() {
  run("up", 16384, 12288, 3072);
  run("qkv", 16384, 9216, 3072);
  run("down", 16384, 3072, 12288);
  return 0;
}
