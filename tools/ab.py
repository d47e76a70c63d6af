#!/usr/bin/env python3
"""Same-process A/B of two builds of a libqie kernel (cdna_hip_programming.md
§5.4 rule 24: interleaved rounds in ONE process, report median and min).

    python tools/ab.py attention path/to/libA.so path/to/libB.so [more.so ...] [rounds]

All libraries are loaded side by side with ctypes; launches alternate A, B, C, A, B, C ...
on the same random inputs (headline shapes: attention B=2, S=8408; the three DiT GEMMs)."""
import ctypes
import math
import os
import statistics
import sys

import torch

BF16 = torch.bfloat16


def load(path):
    lib = ctypes.CDLL(path)
    lib.qie_attention_fwd_bf16.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_int), ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_void_p]
    if hasattr(lib, "qie_attention_fwd_split_bf16"):
        lib.qie_attention_fwd_split_bf16.argtypes = lib.qie_attention_fwd_bf16.argtypes[:-1] + [
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    lib.qie_linear_splitk_bf16.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    lib.qie_linear_bf16.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_void_p]
    return lib


def main():
    what = sys.argv[1]
    # "lib.so@log2q": the attention entry for a q plane pre-multiplied by scale*log2(e)
    args = [a.split("@") for a in sys.argv[2:]]
    # "torch": the library reference (hipBLASLt through F.linear) for the gemm shapes
    paths = [a[0] for a in args if a[0].endswith(".so") or a[0] == "torch"]
    modes = [a[1] if len(a) > 1 else "" for a in args if a[0].endswith(".so") or a[0] == "torch"]
    rest = [a[0] for a in args if not (a[0].endswith(".so") or a[0] == "torch")]
    rounds = int(rest[0]) if rest else 10
    if not what.startswith("gemm"):  # the library arm exists for the plain GEMM shapes only
        keep = [i for i, p in enumerate(paths) if p != "torch"]
        paths, modes = [paths[i] for i in keep], [modes[i] for i in keep]
    libs = [load(p) if p != "torch" else None for p in paths]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    if what in ("attention", "attention_nosplit"):
        B, H, S_IMG, S_TXT = 2, 24, 8192, 216
        S = S_IMG + S_TXT
        s_pad = ((S + 255) // 256) * 256
        qkv = torch.randn(3, B, H, s_pad, 128, device=dev).to(BF16)
        qkv[:, :, :, S:] = 0
        if os.environ.get("AB_ZERO"):
            qkv.zero_()
        outs = [(torch.empty(B * S_IMG, H * 128, dtype=BF16, device=dev),
                 torch.empty(B * S_TXT, H * 128, dtype=BF16, device=dev)) for _ in libs]
        kv = (ctypes.c_int * B)(*[S] * B)
        flops = 4.0 * B * S * S * H * 128

        ws = torch.empty(B * H * 5 * 256 * 130, device=dev)  # QIE_ATTN_SPLIT = 5
        qkv2 = qkv.clone()
        qkv2[0] = (qkv[0].float() * (1.4426950408889634 / math.sqrt(128))).to(BF16)

        def run(i):
            lib = libs[i]
            if modes[i] == "log2q":
                lib.qie_attention_fwd_log2q_bf16.argtypes = lib.qie_attention_fwd_bf16.argtypes[:-2] + [
                    ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
                rc = lib.qie_attention_fwd_log2q_bf16(
                    qkv2.data_ptr(), B, H, s_pad, kv, outs[i][0].data_ptr(), outs[i][1].data_ptr(), S_IMG, S_TXT,
                    ws.data_ptr() if what == "attention" else None, ws.numel() * 4, st)
            elif what == "attention" and hasattr(lib, "qie_attention_fwd_split_bf16"):
                rc = lib.qie_attention_fwd_split_bf16(qkv.data_ptr(), B, H, s_pad, kv, outs[i][0].data_ptr(),
                                                      outs[i][1].data_ptr(), S_IMG, S_TXT, 1 / math.sqrt(128),
                                                      ws.data_ptr(), ws.numel() * 4, st)
            else:
                rc = lib.qie_attention_fwd_bf16(qkv.data_ptr(), B, H, s_pad, kv, outs[i][0].data_ptr(),
                                                outs[i][1].data_ptr(), S_IMG, S_TXT, 1 / math.sqrt(128), st)
            assert rc == 0, rc
    elif what.startswith("splitk:"):  # splitk:M:N:K:s_lib0:s_lib1:... (split count per library)
        parts = [int(v) for v in what.split(":")[1:]]
        M, N, K, spl = parts[0], parts[1], parts[2], parts[3:]
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from qwen_image_edit_streamdiffusion_amd import _lib as L
        x = torch.randn(M, K, device=dev).to(BF16)
        w = (torch.randn(N, K, device=dev) * 0.02).to(BF16)
        b = torch.zeros(N, device=dev, dtype=BF16)
        outs = [torch.empty(M, N, dtype=BF16, device=dev) for _ in libs]
        ws = torch.empty(max(spl) * M * N, device=dev)
        eps = [L.Epilogue(kind=0, out=o.data_ptr(), ldo=N) for o in outs]
        flops = 2.0 * M * N * K

        def run(i):
            rc = libs[i].qie_linear_splitk_bf16(x.data_ptr(), K, w.data_ptr(), b.data_ptr(), ctypes.addressof(eps[i]),
                                                M, N, K, spl[i], ws.data_ptr(), ws.numel() * 4, st)
            assert rc == 0, rc
    elif what.startswith("gate:"):  # gate:M:N:K -- gated-residual epilogue (resid += gate * y)
        M, N, K = (int(v) for v in what.split(":")[1:])
        x = torch.randn(M, K, device=dev).to(BF16)
        w = (torch.randn(N, K, device=dev) * 0.02).to(BF16)
        b = torch.zeros(N, device=dev, dtype=BF16)
        gate = (torch.randn(2, 6 * N, device=dev) * 0.1).to(BF16)
        r0 = torch.randn(M, N, device=dev).to(BF16)  # the same start residual for every build
        outs = [r0.clone() for _ in libs]
        flops = 2.0 * M * N * K
        for lib in libs:
            lib.qie_linear_gated_residual_bf16.argtypes = [
                ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]

        def run(i):
            rc = libs[i].qie_linear_gated_residual_bf16(x.data_ptr(), K, w.data_ptr(), b.data_ptr(), gate.data_ptr(),
                                                        6 * N, M // 2, outs[i].data_ptr(), N, M, N, K, st)
            assert rc == 0, rc
    elif what == "qkvnr":  # image QKV GEMM + QK RMSNorm + RoPE epilogue, headline shape (B = 2, S_img 8192)
        B, H, Dh, S_IMG, S_PAD, K = 2, 24, 128, 8192, 8448, 3072
        M, N = B * S_IMG, 3 * H * Dh
        x = torch.randn(M, K, device=dev).to(BF16)
        w = (torch.randn(N, K, device=dev) * 0.02).to(BF16)
        b = torch.zeros(N, device=dev, dtype=BF16)
        nq, nk = (1 + 0.1 * torch.randn(2, Dh, device=dev)).to(BF16)
        ang = torch.randn(S_IMG, Dh // 2, device=dev)
        cos_t, sin_t = ang.cos().contiguous(), ang.sin().contiguous()
        outs = [torch.zeros(3, B, H, S_PAD, Dh, device=dev, dtype=BF16) for _ in libs]
        flops = 2.0 * M * N * K
        for lib in libs:
            lib.qie_linear_qkv_norm_rope_bf16.argtypes = [
                ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p] + \
                [ctypes.c_int] * 8 + [ctypes.c_void_p] * 4 + [ctypes.c_float, ctypes.c_float, ctypes.c_void_p]

        def run(i):
            rc = libs[i].qie_linear_qkv_norm_rope_bf16(
                x.data_ptr(), K, w.data_ptr(), b.data_ptr(), outs[i].data_ptr(), M, K, S_IMG, 0, B, H, Dh, S_PAD,
                nq.data_ptr(), nk.data_ptr(), cos_t.data_ptr(), sin_t.data_ptr(), 1e-6, 1.0, st)
            assert rc == 0, rc
    elif what == "lnmod":  # LayerNorm + modulate of the image rows (B = 2 stream batch)
        M, D = 16384, 3072
        x = torch.randn(M, D, device=dev).to(BF16)
        mod = (torch.randn(2, 6 * D, device=dev) * 0.1).to(BF16)
        outs = [torch.empty(M, D, dtype=BF16, device=dev) for _ in libs]
        flops = 4.0 * M * D  # bytes moved (read + write), reported as "TFLOP/s" = TB/s here
        for lib in libs:
            lib.qie_layernorm_modulate_bf16.argtypes = [
                ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_void_p]

        def run(i):
            rc = libs[i].qie_layernorm_modulate_bf16(x.data_ptr(), D, mod.data_ptr(), mod[:, D:].data_ptr(), 6 * D,
                                                     M // 2, outs[i].data_ptr(), D, M, D, 1e-6, st)
            assert rc == 0, rc
    elif what.startswith("gemm"):
        if what.startswith("gemm:"):  # gemm:M:N:K
            M, N, K = (int(v) for v in what.split(":")[1:])
        else:
            M, N, K = {"gemm_up": (16384, 12288, 3072), "gemm_qkv": (16384, 9216, 3072),
                       "gemm_down": (16384, 3072, 12288)}[what]
        x = torch.randn(M, K, device=dev).to(BF16)
        w = (torch.randn(N, K, device=dev) * 0.02).to(BF16)
        b = torch.zeros(N, device=dev, dtype=BF16)
        if os.environ.get("AB_ZERO"):  # zero-filled operands: the DVFS ceiling (rule 25)
            x.zero_()
            w.zero_()
        outs = [torch.empty(M, N, dtype=BF16, device=dev) for _ in libs]
        flops = 2.0 * M * N * K

        def run(i):
            if libs[i] is None:
                torch.mm(x, w.t(), out=outs[i])
                return
            rc = libs[i].qie_linear_bf16(x.data_ptr(), K, w.data_ptr(), b.data_ptr(), outs[i].data_ptr(), N,
                                         M, N, K, 0, st)
            assert rc == 0, rc
    else:
        raise SystemExit(f"unknown kernel {what}")
    L = len(libs)
    times = [[] for _ in range(L)]
    for _ in range(3):
        for i in range(L):
            run(i)
    torch.cuda.synchronize()
    for _ in range(rounds):
        for i in range(L):
            a, bb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                run(i)
            bb.record()
            torch.cuda.synchronize()
            times[i].append(a.elapsed_time(bb) / 5)
    first = [o[0] if isinstance(o, tuple) else o for o in outs]
    for i in range(L):
        med, mn = statistics.median(times[i]), min(times[i])
        diff = (first[0].float() - first[i].float()).abs().max().item()
        print(f"{what} {paths[i]}: median {med:.3f} ms  min {mn:.3f} ms  {flops / med / 1e9:.0f} TFLOP/s"
              f"  max|diff vs first| {diff:.3e}")


if __name__ == "__main__":
    main()
