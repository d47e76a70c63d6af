#!/usr/bin/env python3
"""Kernel microbenchmarks at the headline shapes (B=2 stream-batch forward,
1024^2: S_img=8192, S_txt=216, D=3072, H=24, F=12288), random data.

Prints one line per kernel: avg ms over N launches (HIP events on the launch
stream) and achieved TFLOP/s or GB/s.  Usage: python tools/kbench.py [names...]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from qwen_image_edit_streamdiffusion_amd import ops  # noqa: E402

BF16 = torch.bfloat16
dev = torch.device("cuda:0")
B, S_IMG, S_TXT, D, H, F = 2, 8192, 216, 3072, 24, 12288


def timeit(fn, n=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(BF16)


def bench_attention():
    S = S_IMG + S_TXT
    s_pad = ((S + 255) // 256) * 256
    qkv = rnd(3, B, H, s_pad, 128)
    qkv[:, :, :, S:] = 0
    oi = torch.empty(B * S_IMG, D, dtype=BF16, device=dev)
    ot = torch.empty(B * S_TXT, D, dtype=BF16, device=dev)
    ms = timeit(lambda: ops.attention(qkv, [S] * B, oi, ot, S_IMG, S_TXT))
    fl = 4.0 * B * S * S * D
    return f"attention B={B} S={S}: {ms:.3f} ms  {fl / ms / 1e9:.0f} TFLOP/s"


def bench_gemm(name, M, N, K, kind):
    x, w, b = rnd(M, K), rnd(N, K, scale=0.02), rnd(N, scale=0.02)
    if kind == "gelu":
        y = torch.empty(M, N, dtype=BF16, device=dev)
        fn = lambda: ops.linear(x, w, b, out=y, act=ops.ACT_GELU)
    elif kind == "plain":
        y = torch.empty(M, N, dtype=BF16, device=dev)
        fn = lambda: ops.linear(x, w, b, out=y)
    elif kind == "gate":
        g = rnd(B, 6 * N)
        r = rnd(M, N)
        fn = lambda: ops.linear_gated_residual(x, w, b, g[:, :N], M // B, r)
    elif kind == "qkv":
        qkv = torch.zeros(3, B, H, ((S_IMG + S_TXT + 255) // 256) * 256, 128, dtype=BF16, device=dev)
        fn = lambda: ops.linear_qkv(x, w, b, qkv, M // B, 0)
    ms = timeit(fn)
    return f"{name} M={M} N={N} K={K}: {ms:.3f} ms  {2.0 * M * N * K / ms / 1e9:.0f} TFLOP/s"


def bench_qkv_variants():
    """QKV projection at the image-stream shape: plain GEMM, QKV scatter, scatter + separate
    QK-norm/RoPE kernel, and the fused epilogue (same process, same inputs)."""
    from qwen_image_edit_streamdiffusion_amd.rope import rope_tables
    M, N, K = B * S_IMG, 3 * D, D
    x, w, b = rnd(M, K), rnd(N, K, scale=0.02), rnd(N, scale=0.02)
    s_pad = ((S_IMG + S_TXT + 255) // 256) * 256
    qkv = torch.zeros(3, B, H, s_pad, 128, dtype=BF16, device=dev)
    y = torch.empty(M, N, dtype=BF16, device=dev)
    ic, is_, _, _ = rope_tables([(1, 64, 64), (1, 64, 64)], S_TXT, dev)
    nw = rnd(128)
    fl = 2.0 * M * N * K
    out = []
    for name, fn in (("qkv_plain", lambda: ops.linear(x, w, b, out=y)),
                     ("qkv_scatter", lambda: ops.linear_qkv(x, w, b, qkv, S_IMG, 0)),
                     ("qkv_scatter+norm_rope", lambda: (ops.linear_qkv(x, w, b, qkv, S_IMG, 0),
                                                        ops.qk_norm_rope(qkv, 0, S_IMG, nw, nw, ic, is_))),
                     ("qkv_fused_norm_rope", lambda: ops.linear_qkv_norm_rope(x, w, b, qkv, S_IMG, 0, nw, nw,
                                                                              ic, is_))):
        ms = timeit(fn)
        out.append(f"{name} M={M} N={N} K={K}: {ms:.3f} ms  {fl / ms / 1e9:.0f} TFLOP/s")
    return out


def bench_i8(name, M, N, K, act=0):
    xq = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
    wq = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
    sx = torch.rand(M, device=dev) * 1e-2
    sw = torch.rand(N, device=dev) * 1e-3
    b = rnd(N, scale=0.02)
    y = torch.empty(M, N, dtype=BF16, device=dev)
    ms = timeit(lambda: ops.linear_i8(xq, sx, wq, sw, b, y, act=act))
    return f"{name} M={M} N={N} K={K}: {ms:.3f} ms  {2.0 * M * N * K / ms / 1e9:.0f} TOP/s"


def bench_misc():
    out = []
    x = rnd(B * S_IMG, D)
    mods = rnd(B, 6 * D)
    y = torch.empty_like(x)
    ms = timeit(lambda: ops.layernorm_modulate(x, mods[:, :D], mods[:, D:2 * D], S_IMG, out=y))
    out.append(f"ln_mod rows={B * S_IMG}: {ms * 1e3:.1f} us  {2 * x.numel() * 2 / ms / 1e6:.0f} GB/s")
    s_pad = ((S_IMG + S_TXT + 255) // 256) * 256
    qkv = rnd(3, B, H, s_pad, 128)
    from qwen_image_edit_streamdiffusion_amd.rope import rope_tables
    ic, is_, tc, ts = rope_tables([(1, 64, 64), (1, 64, 64)], S_TXT, dev)
    w = rnd(128)
    ms = timeit(lambda: ops.qk_norm_rope(qkv, 0, S_IMG, w, w, ic, is_))
    byt = 2 * 2 * B * H * S_IMG * 128 * 2
    out.append(f"qk_norm_rope img: {ms * 1e3:.1f} us  {byt / ms / 1e6:.0f} GB/s")
    xs = rnd(B, D)
    wm, bm = rnd(6 * D, D, scale=0.02), rnd(6 * D)
    ym = torch.empty(B, 6 * D, dtype=BF16, device=dev)
    ms = timeit(lambda: ops.gemv(xs, wm, bm, out=ym))
    out.append(f"gemv mod M={B} N={6 * D} K={D}: {ms * 1e3:.1f} us  {wm.numel() * 2 / ms / 1e6:.0f} GB/s")
    return out


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "one":  # single kernel, for rocprofv3 --pmc passes
        M = B * S_IMG
        shapes = {"mlp_up_plain": (M, F, D, "plain"), "mlp_down_gate": (M, D, F, "gate"),
                  "qkv": (M, 3 * D, D, "qkv"), "out_gate": (M, D, D, "gate")}
        if sys.argv[2] == "attention":
            print(bench_attention())
        else:
            print(bench_gemm(sys.argv[2], *shapes[sys.argv[2]]))
        return
    want = set(sys.argv[1:])
    res = []
    if not want or "attention" in want:
        res.append(bench_attention())
    if not want or "gemm" in want:
        M = B * S_IMG
        res.append(bench_gemm("qkv", M, 3 * D, D, "qkv"))
        res.append(bench_gemm("out_gate", M, D, D, "gate"))
        res.append(bench_gemm("mlp_up_gelu", M, F, D, "gelu"))
        res.append(bench_gemm("mlp_up_plain", M, F, D, "plain"))
        res.append(bench_gemm("mlp_down_gate", M, D, F, "gate"))
        Mt = B * S_TXT
        res.append(bench_gemm("txt_qkv", Mt, 3 * D, D, "qkv"))
        res.append(bench_gemm("txt_up", Mt, F, D, "gelu"))
        res.append(bench_gemm("txt_down", Mt, D, F, "gate"))
    if not want or "i8" in want:
        M = B * S_IMG
        res.append(bench_i8("i8_up", M, F, D, act=1))
        res.append(bench_i8("i8_down", M, D, F))
    if "i8x" in want:  # int8 per-tile overhead: K = 3072 (12 tiles per CU) vs K = 12288 (3 per CU)
        M = B * S_IMG
        res.append(bench_i8("i8_up_plain", M, F, D, act=0))
        res.append(bench_i8("i8_up_gelu", M, F, D, act=1))
        res.append(bench_i8("i8_down_plain", M, D, F, act=0))
        res.append(bench_i8("i8_out_plain", M, D, D, act=0))
        res.append(bench_gemm("mlp_up_plain", M, F, D, "plain"))
        res.append(bench_gemm("out_plain", M, D, D, "plain"))
    if "i8q" in want:  # per-row int8 quantisation of the GELU output / attention output (int8 path)
        for name, D_ in (("quant_mlp", F), ("quant_att", D)):
            xx = rnd(B * S_IMG, D_)
            qq = torch.empty(B * S_IMG, D_, dtype=torch.int8, device=dev)
            ss = torch.empty(B * S_IMG, dtype=torch.float32, device=dev)
            ms = timeit(lambda: ops.quantize_rows(xx, qq, ss))
            res.append(f"{name} rows={B * S_IMG} D={D_}: {ms * 1e3:.1f} us  {3.0 * B * S_IMG * D_ / ms / 1e9:.2f} TB/s")
    if not want or "qkv" in want:
        res += bench_qkv_variants()
    if not want or "misc" in want:
        res += bench_misc()
    for r in res:
        print(r, flush=True)


if __name__ == "__main__":
    main()
