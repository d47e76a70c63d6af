"""CPU checks of the C ABI: libqie.so builds, loads, exports exactly the entry
points include/qie.h declares with matching arity, and rejects bad arguments
on the host (QIE_ERR_INVALID) before any GPU work -- no compute calls here."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "qie.h")


def header_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    funcs = {}
    for m in re.finditer(r"(?:int|const char\*)\s+(qie_\w+)\s*\(([^)]*)\)\s*;", src, flags=re.S):
        args = [a for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        funcs[m.group(1)] = len(args)
    return funcs


@pytest.fixture(scope="module")
def lib():
    from qwen_image_edit_streamdiffusion_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "qwen_image_edit_streamdiffusion_amd", "csrc"),
                        "-j8"], check=True, capture_output=True)
    return _lib.load()


def test_header_parses():
    f = header_functions()
    assert len(f) >= 20 and "qie_attention_fwd_bf16" in f and "qie_linear_i8" in f


def test_every_declared_symbol_exported(lib):
    for name in header_functions():
        assert hasattr(lib, name), name


def test_binding_table_matches_header(lib):
    from qwen_image_edit_streamdiffusion_amd import _lib
    hf = header_functions()
    assert set(_lib.SIGNATURES) == set(hf)
    for name, n in hf.items():
        assert len(_lib.SIGNATURES[name]) == n, name


def test_abi_version_and_strerror(lib):
    from qwen_image_edit_streamdiffusion_amd import _lib
    assert lib.qie_abi_version() == _lib.ABI_VERSION == 2
    assert lib.qie_strerror(0) == b"ok"
    assert b"invalid" in lib.qie_strerror(-1)


def test_invalid_arguments_rejected_on_host(lib):
    from qwen_image_edit_streamdiffusion_amd import _lib
    # null pointers / bad shapes return QIE_ERR_INVALID before any launch
    assert lib.qie_linear_bf16(None, 64, None, None, None, 64, 16, 16, 64, 0, None) == -1
    assert lib.qie_linear_bf16(1, 64, 1, 1, 1, 64, 16, 16, 63, 0, None) == -1      # K % 64
    assert lib.qie_gemv_bf16(16, 8, 16, 16, 16, 8, 17, 8, 8, None) == -1         # M > 16
    kv = (ctypes.c_int * 1)(100)
    assert lib.qie_attention_fwd_bf16(16, 1, 1, 300, kv, 16, 16, 256, 0, 0.1, None) == -1  # s_pad % 256
    dt = (ctypes.c_float * 1)(0.5)
    assert lib.qie_euler_step_bf16(16, 0, 16, 0, 16, 0, 17, 8, dt, None) == -1   # batch > 16
    assert lib.qie_qk_norm_rope_bf16(16, 1, 1, 64, 256, 0, 8, 16, 16, 16, 16, 1e-6, 1.0, None) == -1
    # fused QKV + QK-norm + RoPE: head_dim must be 128, norm/RoPE tables must be given
    assert lib.qie_linear_qkv_norm_rope_bf16(16, 256, 16, 16, 16, 512, 256, 256, 0, 2, 2, 64, 512,
                                             16, 16, 16, 16, 1e-6, 1.0, None) == -1
    assert lib.qie_linear_qkv_norm_rope_bf16(16, 256, 16, 16, 16, 512, 256, 256, 0, 2, 2, 128, 512,
                                             None, 16, 16, 16, 1e-6, 1.0, None) == -1
    with pytest.raises(_lib.QieError):
        _lib.call("qie_rmsnorm_bf16", None, None, None, 1, 8, 1e-6, None)
    # split-K: null epilogue, unknown kind, K not a multiple of splits * 64, workspace too small
    e = _lib.Epilogue(kind=0, out=16, ldo=256)
    ep = ctypes.addressof(e)
    assert lib.qie_linear_splitk_bf16(16, 256, 16, 16, None, 8, 256, 256, 2, 16, 1 << 20, None) == -1
    bad = _lib.Epilogue(kind=9, out=16, ldo=256)
    assert lib.qie_linear_splitk_bf16(16, 256, 16, 16, ctypes.addressof(bad), 8, 256, 256, 2, 16, 1 << 20, None) == -1
    assert lib.qie_linear_splitk_bf16(16, 256, 16, 16, ep, 8, 256, 192, 2, 16, 1 << 20, None) == -1
    assert lib.qie_linear_splitk_bf16(16, 256, 16, 16, ep, 8, 256, 256, 2, 16, 8 * 256 * 4, None) == -1
    assert lib.qie_linear_splitk_i8(16, 256, None, 16, 16, 16, ep, 8, 256, 256, 2, 16, 1 << 20, None) == -1
    # attention workspace query (host only) and the split entry's workspace check
    n = ctypes.c_int64(-1)
    assert lib.qie_attention_workspace_bytes(2, 24, 8448, 8192, 216, ctypes.byref(n)) == 0
    assert n.value == 2 * 24 * 5 * 256 * 130 * 4
    assert lib.qie_attention_workspace_bytes(1, 1, 256, 200, 0, ctypes.byref(n)) == 0 and n.value == 0
    assert lib.qie_attention_workspace_bytes(1, 1, 256, 200, 0, None) == -1
    kv = (ctypes.c_int * 1)(512)
    assert lib.qie_attention_fwd_split_bf16(16, 1, 1, 512, kv, 16, None, 512, 0, 0.1, None, 0, None) == -1
    # VAE flash attention: workspace query (host only), C must be 384, vt wide enough, workspace size
    assert lib.qie_vae_attention_workspace(16384, 384, ctypes.byref(n)) == 0
    assert n.value == 2 * 16384 * 386 * 4  # two key ranges of fp32 partials at 128 query blocks
    assert lib.qie_vae_attention_workspace(16384, 256, ctypes.byref(n)) == -1
    assert lib.qie_vae_attention_bf16(16, 1152, 16, 16384, 16384, 256, 16, 384, 16, 1 << 30, None) == -1
    assert lib.qie_vae_attention_bf16(16, 1152, 16, 100, 16384, 384, 16, 384, 16, 1 << 30, None) == -1
    assert lib.qie_vae_attention_bf16(16, 1152, 16, 16384, 16384, 384, 16, 384, 16, 1024, None) == -1
    # fused conv + RMS-norm: gamma required (and 16-byte aligned); the conv's own checks apply
    assert lib.qie_conv2d_rmsnorm_bf16(16, 64, 64, 96, 0, 3, 16, 896, 16, None, 1, 16, 96, None) == -1
    assert lib.qie_conv2d_rmsnorm_bf16(16, 64, 64, 96, 0, 3, 16, 896, 16, 18, 1, 16, 96, None) == -1
    assert lib.qie_conv2d_rmsnorm_bf16(16, 64, 64, 92, 0, 3, 16, 896, 16, 16, 1, 16, 96, None) == -1
