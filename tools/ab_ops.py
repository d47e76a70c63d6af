#!/usr/bin/env python3
"""Same-process, interleaved A/B of op variants through the product wrappers (ops.py):
rounds of [A x5, B x5, C x5, ...], median and min per variant (cdna_hip_programming.md §5.4
rule 24). Shapes are the headline B=2 stream-batch forward (S_img 8192, D 3072, H 24).

    python tools/ab_ops.py qkv [rounds]     QKV projection: plain / scatter / +norm-rope / fused
    python tools/ab_ops.py epi [rounds]     epilogue kinds at the MLP-up and down shapes
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from qwen_image_edit_streamdiffusion_amd import ops  # noqa: E402
from qwen_image_edit_streamdiffusion_amd.rope import rope_tables  # noqa: E402

BF16 = torch.bfloat16
dev = torch.device("cuda:0")
B, S_IMG, S_TXT, D, H, F = 2, 8192, 216, 3072, 24, 12288


def rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(BF16)


def variants(what):
    M = B * S_IMG
    if what == "qkv":
        N, K = 3 * D, D
        x, w, b = rnd(M, K), rnd(N, K, scale=0.02), rnd(N, scale=0.02)
        s_pad = ((S_IMG + S_TXT + 255) // 256) * 256
        qkv = torch.zeros(3, B, H, s_pad, 128, dtype=BF16, device=dev)
        y = torch.empty(M, N, dtype=BF16, device=dev)
        ic, is_, _, _ = rope_tables([(1, 64, 64), (1, 64, 64)], S_TXT, dev)
        nw = (1 + rnd(128, scale=0.1).float()).to(BF16)

        def two():
            ops.linear_qkv(x, w, b, qkv, S_IMG, 0)
            ops.qk_norm_rope(qkv, 0, S_IMG, nw, nw, ic, is_)
        return 2.0 * M * N * K, {
            "plain": lambda: ops.linear(x, w, b, out=y),
            "scatter": lambda: ops.linear_qkv(x, w, b, qkv, S_IMG, 0),
            "scatter+norm_rope": two,
            "fused": lambda: ops.linear_qkv_norm_rope(x, w, b, qkv, S_IMG, 0, nw, nw, ic, is_)}
    if what == "epi":
        x, w, b = rnd(M, D), rnd(F, D, scale=0.02), rnd(F, scale=0.02)
        y = torch.empty(M, F, dtype=BF16, device=dev)
        xd, wd, bd = rnd(M, F), rnd(D, F, scale=0.02), rnd(D, scale=0.02)
        yd = torch.empty(M, D, dtype=BF16, device=dev)
        gate = rnd(B, 6 * D)
        resid = rnd(M, D)
        return 2.0 * M * F * D, {
            "up_plain": lambda: ops.linear(x, w, b, out=y),
            "up_gelu": lambda: ops.linear(x, w, b, out=y, act=ops.ACT_GELU),
            "down_plain": lambda: ops.linear(xd, wd, bd, out=yd),
            "down_gate": lambda: ops.linear_gated_residual(xd, wd, bd, gate[:, :D], S_IMG, resid)}
    raise SystemExit(f"unknown {what}")


def main():
    what = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    flops, vs = variants(what)
    names = list(vs)
    times = {n: [] for n in names}
    for _ in range(3):
        for n in names:
            vs[n]()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for n in names:
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                vs[n]()
            e.record()
            torch.cuda.synchronize()
            times[n].append(a.elapsed_time(e) / 5)
    for n in names:
        med, mn = statistics.median(times[n]), min(times[n])
        print(f"{what} {n}: median {med:.3f} ms  min {mn:.3f} ms  {flops / med / 1e9:.0f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
