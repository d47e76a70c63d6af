#!/usr/bin/env python3
"""Time the VAE mid-block attention at 1024^2 (P = 16384 latent pixels, C = 384): the flash kernel
(qie_vae_attention_bf16) vs the materialised chain it replaced (fp32 scores, row softmax, P.V)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from qwen_image_edit_streamdiffusion_amd import ops  # noqa: E402

BF16 = torch.bfloat16


def timed(fn, n=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def main():
    dev = torch.device("cuda:0")
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    C = 384
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(P, 3 * C, generator=g, device=dev).to(BF16)
    kp = -(-P // 64) * 64
    vt = torch.zeros(C, kp, dtype=BF16, device=dev)
    ops.transpose(qkv[:, 2 * C:], out=vt[:, :P])
    ws = torch.empty(-(-ops.vae_attention_workspace_bytes(P, C) // 4), dtype=torch.float32, device=dev)
    out = torch.empty(P, C, dtype=BF16, device=dev)
    s = torch.empty(P, P, dtype=torch.float32, device=dev)
    p = torch.empty(P, kp, dtype=BF16, device=dev)
    out2 = torch.empty(P, C, dtype=BF16, device=dev)
    zb = torch.zeros(C, dtype=BF16, device=dev)

    def flash():
        ops.vae_attention(qkv, vt, out, ws)

    def chain():
        ops.matmul_f32out(qkv[:, :C], qkv[:, C:2 * C], out=s)
        ops.softmax_rows(s, 1.0 / math.sqrt(C), out=p)
        ops.linear(p, vt, zb, out=out2)
    flops = 4.0 * P * P * C
    tf, tc = timed(flash), timed(chain)
    d = (out.float() - out2.float()).abs().max().item()
    print(f"vae attention P={P}: flash {tf * 1e3:.1f} us ({flops / tf / 1e9:.0f} TF/s)  chain {tc * 1e3:.1f} us "
          f"({flops / tc / 1e9:.0f} TF/s)  max|flash-chain| {d:.3e}", flush=True)


if __name__ == "__main__":
    main()
