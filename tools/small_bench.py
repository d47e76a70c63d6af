"""Time the DiT's bandwidth-bound small kernels at the bench shapes (B = 2 stream batch):
modulation GEMV (M = 2, N = 6 D, K = D), LayerNorm + modulate on the image rows."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from qwen_image_edit_streamdiffusion_amd import ops  # noqa: E402


def bench(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


dev = "cuda"
D = 3072
x = torch.randn(2, D, device=dev).to(torch.bfloat16)
# 12 distinct 113 MB matrices (1.36 GB, ~5x the MALL) cycled as the forward does, so every launch
# streams its weights from HBM; a single reused matrix would be served from the infinity cache
NW = 12
ws_ = [(torch.randn(6 * D, D, device=dev) / 60).to(torch.bfloat16) for _ in range(NW)]
w = ws_[0]
b = torch.zeros(6 * D, device=dev, dtype=torch.bfloat16)
out = torch.empty(2, 6 * D, device=dev, dtype=torch.bfloat16)
_i = [0]


def _next():
    _i[0] = (_i[0] + 1) % NW
    return ws_[_i[0]]


t = bench(lambda: ops.gemv(x, _next(), b, out=out), it=NW * 8)
print(f"gemv M=2 N={6 * D} K={D} (HBM-cold, {NW} matrices): {t:.1f} us, {w.numel() * 2 / t / 1e6:.2f} TB/s")
t = bench(lambda: ops.gemv(x, w, b, out=out))
print(f"gemv M=2 N={6 * D} K={D} (one matrix, cache-warm): {t:.1f} us, {w.numel() * 2 / t / 1e6:.2f} TB/s")
import ctypes  # noqa: E402
for so in sys.argv[1:]:  # A/B against other builds' gemv: python tools/small_bench.py a.so b.so ...
    lib = ctypes.CDLL(so)
    lib.qie_gemv_bf16.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p]
    st = torch.cuda.current_stream().cuda_stream
    t2 = bench(lambda: lib.qie_gemv_bf16(x.data_ptr(), D, _next().data_ptr(), b.data_ptr(), out.data_ptr(),
                                         6 * D, 2, 6 * D, D, st), it=NW * 8)
    print(f"  {so}: {t2:.1f} us, {w.numel() * 2 / t2 / 1e6:.2f} TB/s (HBM-cold)")
R = 2 * 8192
h = torch.randn(R, D, device=dev).to(torch.bfloat16)
mod = torch.randn(2, 6 * D, device=dev).to(torch.bfloat16)
o = torch.empty_like(h)
t = bench(lambda: ops.layernorm_modulate(h, mod[:, :D], mod[:, D:2 * D], 8192, out=o))
print(f"ln_mod rows={R} D={D}: {t:.1f} us, {2 * h.numel() * 2 / t / 1e6:.2f} TB/s")
for so in sys.argv[1:]:  # the same A/B for qie_layernorm_modulate_bf16
    lib = ctypes.CDLL(so)
    lib.qie_layernorm_modulate_bf16.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                                ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_void_p]
    st = torch.cuda.current_stream().cuda_stream
    t2 = bench(lambda: lib.qie_layernorm_modulate_bf16(h.data_ptr(), D, mod.data_ptr(), mod[:, D:].data_ptr(),
                                                       6 * D, 8192, o.data_ptr(), D, R, D, 1e-6, st))
    print(f"  {so}: ln_mod {t2:.1f} us, {2 * h.numel() * 2 / t2 / 1e6:.2f} TB/s")
