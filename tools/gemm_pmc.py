"""One DiT GEMM shape (mlp up: 16384 x 12288 x 3072) through libqie and through torch.mm
(hipBLASLt), 10 launches each, for a rocprofv3 --pmc pass that compares the two kernels."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from qwen_image_edit_streamdiffusion_amd import ops  # noqa: E402

M, N, K = 16384, 12288, 3072
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda") / 60).to(torch.bfloat16)
b = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(10):
    ops.linear(x, w, b, out=out)
for _ in range(10):
    torch.mm(x, w.t(), out=out)
torch.cuda.synchronize()
print("done")
