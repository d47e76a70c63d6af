"""ctypes binding of libqie.so (include/qie.h).

The product path has NO fallback: if the HIP library is missing or fails to
load, every op raises.  Build it with ``__graft_entry__.build()`` or
``make -C qwen_image_edit_streamdiffusion_amd/csrc``.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_int64, c_void_p, c_char_p, POINTER

_HERE = os.path.dirname(os.path.abspath(__file__))
# QIE_LIB_PATH: another build of the same library (same-box A/B of whole-model runs, tools/ab_bench.sh)
LIB_PATH = os.environ.get("QIE_LIB_PATH") or os.path.join(_HERE, "libqie.so")

P = c_void_p
I = c_int
L = c_int64
F = c_float
FP = POINTER(c_float)
IP = POINTER(c_int)



class Epilogue(ctypes.Structure):
    """``qie_epilogue_t`` (include/qie.h): epilogue of the split-K linears."""
    _fields_ = [("kind", c_int), ("out", c_void_p), ("ldo", c_int64), ("gate", c_void_p),
                ("gate_bstride", c_int64), ("rows_per_batch", c_int), ("seq_offset", c_int),
                ("batch", c_int), ("heads", c_int), ("head_dim", c_int), ("s_pad", c_int)]


EPI_BIAS, EPI_GELU, EPI_GATED_RESIDUAL, EPI_QKV = 0, 1, 2, 3

ABI_VERSION = 2  # include/qie.h QIE_ABI_VERSION

# name -> argtypes (return type is always c_int unless listed in _RESTYPES)
SIGNATURES = {
    "qie_abi_version": [],
    "qie_strerror": [I],
    "qie_linear_bf16": [P, L, P, P, P, L, I, I, I, I, P],
    "qie_linear_gated_residual_bf16": [P, L, P, P, P, L, I, P, L, I, I, I, P],
    "qie_linear_qkv_bf16": [P, L, P, P, P, I, I, I, I, I, I, I, I, P],
    "qie_linear_qkv_norm_rope_bf16": [P, L, P, P, P, I, I, I, I, I, I, I, I, P, P, P, P, F, F, P],
    "qie_gemv_bf16": [P, L, P, P, P, L, I, I, I, P],
    "qie_layernorm_modulate_bf16": [P, L, P, P, L, I, P, L, I, I, F, P],
    "qie_rmsnorm_bf16": [P, P, P, I, I, F, P],
    "qie_qk_norm_rope_bf16": [P, I, I, I, I, I, I, P, P, P, P, F, F, P],
    "qie_attention_fwd_bf16": [P, I, I, I, IP, P, P, I, I, F, P],
    "qie_attention_workspace_bytes": [I, I, I, I, I, POINTER(c_int64)],
    "qie_attention_fwd_split_bf16": [P, I, I, I, IP, P, P, I, I, F, P, L, P],
    "qie_attention_fwd_log2q_bf16": [P, I, I, I, IP, P, P, I, I, P, L, P],
    "qie_timestep_embed_bf16": [P, P, I, I, P],
    "qie_silu_bf16": [P, P, L, P],
    "qie_cfg_combine_bf16": [P, L, P, L, P, L, I, I, I, F, P],
    "qie_euler_step_bf16": [P, L, P, L, P, L, I, L, FP, P],
    "qie_copy_bf16": [P, L, P, L, I, L, P],
    "qie_pack_latents_bf16": [P, P, I, I, I, I, P],
    "qie_unpack_latents_bf16": [P, P, I, I, I, I, P],
    "qie_quantize_rows_i8": [P, L, P, L, P, I, I, P],
    "qie_layernorm_modulate_i8": [P, L, P, P, L, I, P, L, P, I, I, F, P],
    "qie_linear_i8": [P, L, P, P, P, P, P, L, I, I, I, I, P],
    "qie_linear_gated_residual_i8": [P, L, P, P, P, P, P, L, I, P, L, I, I, I, P],
    "qie_linear_qkv_i8": [P, L, P, P, P, P, P, I, I, I, I, I, I, I, I, P],
    "qie_linear_qkv_norm_rope_i8": [P, L, P, P, P, P, P, I, I, I, I, I, I, I, I, P, P, P, P, F, F, P],
    "qie_linear_splitk_bf16": [P, L, P, P, P, I, I, I, I, P, L, P],
    "qie_linear_splitk_i8": [P, L, P, P, P, P, P, I, I, I, I, P, L, P],
    "qie_conv2d_bf16": [P, I, I, I, I, I, P, L, P, P, P, I, P],
    "qie_conv2d_rmsnorm_bf16": [P, I, I, I, I, I, P, L, P, P, I, P, I, P],
    "qie_matmul_f32out_bf16": [P, L, P, L, P, I, I, I, P],
    "qie_vae_latents_in_bf16": [P, I, I, I, P, P, P, P, P, P],
    "qie_vae_rms_norm_bf16": [P, P, P, L, I, I, P],
    "qie_softmax_rows_f32_bf16": [P, L, P, L, I, I, F, I, P],
    "qie_transpose_bf16": [P, L, P, L, I, I, P],
    "qie_vae_attention_bf16": [P, L, P, L, I, I, P, L, P, L, P],
    "qie_vae_attention_workspace": [I, I, POINTER(c_int64)],
    "qie_vae_rgb_out": [P, L, P, L, P],
    "qie_vae_rgb_in": [P, P, L, P],
    "qie_vae_latents_out_bf16": [P, L, I, I, I, P, P, P, P],
    "qie_embed_rows_bf16": [P, P, I, I, I, P, P],
    "qie_softmax_rows_ranged_f32_bf16": [P, L, P, L, I, I, F, P, I, P],
    "qie_matmul_batched_bf16": [P, L, L, P, L, L, I, P, P, L, L, I, I, I, I, I, P],
    "qie_rope_half_bf16": [P, L, I, I, I, I, I, P, P, I, P],
    "qie_gelu_erf_bf16": [P, L, I, I, P],
    "qie_silu_mul_bf16": [P, L, I, I, P, L, P],
}
_RESTYPES = {"qie_strerror": c_char_p}

_lib = None


class QieError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load libqie.so once; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise QieError(
            f"libqie.so not found at {path}: the HIP extension is required (no CPU/eager "
            "fallback exists). Build it with `python -c 'import __graft_entry__ as g; g.build()'`.")
    lib = ctypes.CDLL(path)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, c_int)
    if lib.qie_abi_version() != ABI_VERSION:
        raise QieError("libqie.so ABI version mismatch")
    _lib = lib
    return lib


def call(name: str, *args) -> None:
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.qie_strerror(rc).decode()
        raise QieError(f"{name} failed ({rc}): {msg}")
