#!/usr/bin/env python3
"""Time qie_conv2d_bf16 on the VAE's heavy shapes (TF/s per shape; optional second library for
a same-process A/B: python tools/conv_bench.py [libB.so])."""
import ctypes
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from qwen_image_edit_streamdiffusion_amd import ops  # noqa: E402
from qwen_image_edit_streamdiffusion_amd import _lib  # noqa: E402

BF16 = torch.bfloat16
SHAPES = [  # (H_in, W_in, C, N, mode)  mode 0 same, 1 up, 2 down
    (1024, 1024, 96, 96, 0), (512, 512, 192, 192, 0), (256, 256, 384, 384, 0), (128, 128, 384, 384, 0),
    (512, 512, 192, 96, 1), (1024, 1024, 96, 96, 2),
]


def main():
    dev = torch.device("cuda:0")
    libs = [("A", None)]
    if len(sys.argv) > 1:
        lb = ctypes.CDLL(sys.argv[1])
        lb.qie_conv2d_bf16.argtypes = _lib.SIGNATURES["qie_conv2d_bf16"]
        libs.append(("B", lb))
    st = torch.cuda.current_stream().cuda_stream
    for H, W, C, N, mode in SHAPES:
        x = torch.randn(H * W, C, device=dev).to(BF16)
        w = (torch.randn(N, ops.conv_kpad(C, 3), device=dev) / math.sqrt(9 * C)).to(BF16)
        b = torch.zeros(N, device=dev, dtype=BF16)
        Ho, Wo = (2 * H, 2 * W) if mode == 1 else (H // 2, W // 2) if mode == 2 else (H, W)
        ys = [torch.empty(Ho * Wo, N, device=dev, dtype=BF16) for _ in libs]
        flops = 2.0 * Ho * Wo * N * 9 * C

        def run(i):
            if libs[i][1] is None:
                ops.conv2d(x, H, W, w, b, up=mode == 1, down=mode == 2, out=ys[i])
            else:
                rc = libs[i][1].qie_conv2d_bf16(x.data_ptr(), H, W, C, mode, 3, w.data_ptr(), w.stride(0),
                                                b.data_ptr(), None, ys[i].data_ptr(), N, st)
                assert rc == 0, rc
        times = [[] for _ in libs]
        for i in range(len(libs)):
            run(i)
        torch.cuda.synchronize()
        for _ in range(5):
            for i in range(len(libs)):
                a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(3):
                    run(i)
                e.record()
                torch.cuda.synchronize()
                times[i].append(a.elapsed_time(e) / 3)
        line = f"conv {H}x{W} C{C}->N{N} mode{mode}:"
        for i, (nm, _) in enumerate(libs):
            ms = statistics.median(times[i])
            line += f"  {nm} {ms * 1e3:7.1f} us {flops / ms / 1e9:5.0f} TF/s"
        if len(libs) > 1:
            line += f"  max|A-B| {(ys[0].float() - ys[1].float()).abs().max().item():.2e}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
