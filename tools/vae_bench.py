#!/usr/bin/env python3
"""Time the HIP VAE decoder at 1024^2 (128x128 latents, real architecture, random weights)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from qwen_image_edit_streamdiffusion_amd.vae import QwenImageVAEDecoder, QwenImageVAEEncoder  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dec = QwenImageVAEDecoder(device=dev).random_init_(0)
    g = torch.Generator(device=dev).manual_seed(1)
    packed = torch.randn(1, 4096, 64, generator=g, device=dev).to(torch.bfloat16)
    for _ in range(2):
        img = dec.decode(packed, 128, 128)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        img = dec.decode(packed, 128, 128)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / n
    f = dec.flops(128, 128)
    print(f"vae decode 1024^2: {ms:.2f} ms  {f / ms / 1e9:.0f} TFLOP/s  img {tuple(img.shape)} "
          f"mean {img.float().mean().item():.1f}")
    enc = QwenImageVAEEncoder(device=dev).random_init_(2)
    rgb = img
    for _ in range(2):
        z = enc.encode(rgb)
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        z = enc.encode(rgb)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / n
    f = enc.flops(1024, 1024)
    print(f"vae encode 1024^2: {ms:.2f} ms  {f / ms / 1e9:.0f} TFLOP/s  latents {tuple(z.shape)} "
          f"std {z.float().std().item():.3f}")


if __name__ == "__main__":
    main()
