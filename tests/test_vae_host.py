"""VAE decoder host logic on the CPU (no GPU): the weight re-layout the conv kernel reads, the
causal-3-D -> 2-D reduction it relies on (checked against the oracle's real F.pad + conv3d),
the state_dict surface, and the FLOP count used by bench.py."""
import math

import pytest
import torch
import torch.nn.functional as F

from oracle import vae_ref as V
from qwen_image_edit_streamdiffusion_amd.vae import (QwenImageVAEDecoder, VAEConfig, conv_weight,
                                                     state_dict_shapes)
from qwen_image_edit_streamdiffusion_amd import ops

BF16 = torch.bfloat16


def _im2col_conv(x, w_rows, C, k):
    """The GEMM qie_conv2d_bf16 computes, in torch: rows of K = [ky][kx][C] (zero padded)."""
    _, H, W = x.shape
    xp = F.pad(x, (k // 2,) * 4)
    cols = []
    for ky in range(k):
        for kx in range(k):
            cols.append(xp[:, ky:ky + H, kx:kx + W].permute(1, 2, 0).reshape(H * W, C))
    a = torch.cat(cols, 1)
    a = F.pad(a, (0, w_rows.shape[1] - a.shape[1]))
    return a @ w_rows.float().T  # [H*W, N]


@pytest.mark.parametrize("C,N,k", [(16, 32, 3), (96, 40, 3), (24, 8, 1)])
def test_conv_weight_layout_equals_causal_conv3d(C, N, k):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(C, 10, 12, generator=g)
    w5 = torch.randn(N, C, k, k, k, generator=g).to(BF16)
    rows = conv_weight(w5)
    assert rows.shape == (N, ops.conv_kpad(C, k)) and rows.shape[1] % 64 == 0
    gemm = _im2col_conv(x, rows, C, k)
    ref = V.causal_conv3d(x[None, :, None], w5, torch.zeros(N), k // 2, V._R(False))[0, :, 0]
    assert torch.allclose(gemm, ref.permute(1, 2, 0).reshape(-1, N), atol=1e-3, rtol=1e-4)


def test_conv_out_padding_row():
    w5 = torch.randn(3, 96, 3, 3, 3).to(BF16)
    rows = conv_weight(w5, n_pad=1)
    assert rows.shape == (4, 896) and (rows[3] == 0).all() and (rows[:, 864:] == 0).all()


def test_state_dict_surface_matches_oracle():
    for base in (96, 32):
        assert state_dict_shapes(VAEConfig(base_dim=base)) == V.decoder_param_shapes(V.VAEConfig(base_dim=base))
    assert VAEConfig().up_blocks() == [(384, 384, "upsample3d"), (192, 384, "upsample3d"),
                                       (192, 192, "upsample2d"), (96, 96, None)]


def test_load_state_dict_strict():
    cfg = VAEConfig(base_dim=16)
    sd = V.random_params(V.VAEConfig(base_dim=16), 1)
    dec = QwenImageVAEDecoder(cfg, "cpu").load_state_dict(sd)
    assert dec.w["decoder.conv_out.weight"].shape == (4, ops.conv_kpad(16, 3))
    assert "decoder.up_blocks.0.upsamplers.0.time_conv.weight" not in dec.w  # skipped on frame 0
    bad = dict(sd)
    bad.pop("decoder.conv_in.bias")
    with pytest.raises(KeyError):
        QwenImageVAEDecoder(cfg, "cpu").load_state_dict(bad)
    bad = dict(sd)
    bad["decoder.conv_in.bias"] = torch.zeros(7)
    with pytest.raises(ValueError):
        QwenImageVAEDecoder(cfg, "cpu").load_state_dict(bad)


def test_decode_flops():
    assert abs(QwenImageVAEDecoder(VAEConfig(), "cpu").flops(128, 128) - V.decode_flops(V.VAEConfig(), 128, 128)) < 1
    # 1024^2 image: ~4.71 TFLOP, the mid-block attention 0.41 of it
    assert 4.6e12 < V.decode_flops(V.VAEConfig(), 128, 128) < 4.8e12


def test_oracle_decode_runs_small():
    """The oracle's decode itself on a tiny config: shape, range, the uint8 tail."""
    cfg = V.VAEConfig(base_dim=8)
    p = V.random_params(cfg, 2)
    packed = torch.randn(1, 16, 64).to(BF16)
    img = V.decode(p, packed, 8, 8, cfg)
    assert img.shape == (1, 3, 64, 64) and img.abs().max() <= 1.0
    u8 = V.to_uint8(img)
    assert u8.shape == (1, 64, 64, 3) and u8.dtype == torch.uint8
