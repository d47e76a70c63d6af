"""Debug: where does the fused QKV+norm+RoPE epilogue differ from the two-launch path?"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import torch
from test_gpu_kernels import _qkv_nr_case, BF16
from qwen_image_edit_streamdiffusion_amd import ops
dev = torch.device("cuda:0")
B, rpb, H, K, off, s_pad, hw = 2, 2048, 8, 256, 0, 2304, (32, 32)
x, w, b, nq, nk, ic, is_, shapes = _qkv_nr_case(dev, B, rpb, H, K, off, s_pad, 70, hw)
fused = torch.zeros(3, B, H, s_pad, 128, dtype=BF16, device=dev)
ops.linear_qkv_norm_rope(x, w, b, fused, rpb, off, nq, nk, ic, is_, q_scale=1.0)
two = torch.zeros_like(fused)
ops.linear_qkv(x, w, b, two, rpb, off)
ops.qk_norm_rope(two, off, rpb, nq, nk, ic, is_, q_scale=1.0)
d = (fused.float() - two.float()).abs()[:, :, :, :rpb]
print("max", d.max().item())
bad = d > 0.05
print("bad count", bad.sum().item(), "of", bad.numel())
for wh in range(3):
    print("which", wh, "bad", bad[wh].sum().item())
idx = bad.nonzero()
print("first bad idx (which,b,h,s,d):", idx[:20].tolist())
if idx.numel():
    print("s mod 16 hist", torch.bincount(idx[:, 3] % 16, minlength=16).tolist())
    print("s //128 hist", torch.bincount(idx[:, 3] // 128).tolist())
    print("d hist /8", torch.bincount(idx[:, 4] // 8, minlength=16).tolist())
    print("h hist", torch.bincount(idx[:, 2], minlength=H).tolist())
