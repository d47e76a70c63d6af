"""CPU restatement of the Qwen-Image VAE decoder (AutoencoderKLQwenImage.decode) on one frame.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): the checker for the HIP path, never the
product.  PARITY UNPINNED against diffusers (absent here).

What is restated, and where the reference invokes it:

* ``QwenImageEditPlusPipeline`` decode tail [U: diffusers pipelines/qwenimage/
  pipeline_qwenimage_edit_plus.py], reached through server.py:137-153 and
  qwen_realtime.py:247-255 (and the dead helper ``decode_latent`` at
  qwen_realtime.py:188-199): ``_unpack_latents``; ``latents / (1/std) + mean`` with both
  constants cast to the latents' bf16; ``vae.decode(z)[:, :, 0]``; ``postprocess``
  ((x/2 + 0.5).clamp(0, 1), (v*255).round() -> uint8).
* ``AutoencoderKLQwenImage`` [U: diffusers models/autoencoders/autoencoder_kl_qwenimage.py],
  the Wan-2.1 causal 3-D VAE: ``post_quant_conv`` (1x1x1), ``QwenImageDecoder3d``
  (conv_in 3x3x3, mid block = resnet + single-head attention + resnet, four up blocks of
  ``num_res_blocks + 1`` resnets with ``upsample3d, upsample3d, upsample2d, -`` resamplers,
  RMS_norm + SiLU + conv_out), ``clamp(-1, 1)``.

This module keeps the causal 3-D form on purpose -- ``F.pad`` of two zero frames in front and a
real ``conv3d`` -- so that the tests check the HIP path's reduction of each causal conv on the
first frame to a 2-D conv with the kernel's last temporal slice.  The ``upsample3d`` time_conv
is skipped on the first frame exactly as the reference does (``feat_cache[idx] is None`` ->
``"Rep"``).

Numerics: with ``emulate_bf16=True`` tensors are rounded to bf16 where the bf16 module graph
stores them (conv outputs, each op of F.normalize / * scale / * gamma, SiLU, residual sums,
attention output); reductions in fp32.  ``emulate_bf16=False`` is plain fp32.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

BF16 = torch.bfloat16

# AutoencoderKLQwenImage config defaults [U] (the Wan-2.1 VAE statistics)
LATENTS_MEAN = [-0.7571, -0.7089, -0.9113, 0.1075, -0.1745, 0.9653, -0.1517, 1.5508,
                0.4134, -0.0715, 0.5517, -0.3632, -0.1922, -0.9497, 0.2503, -0.2921]
LATENTS_STD = [2.8184, 1.4541, 2.3275, 2.6558, 1.2196, 1.7708, 2.6052, 2.0743,
               3.2687, 2.1526, 2.8652, 1.5579, 1.6382, 1.1253, 2.8251, 1.9160]


@dataclass
class VAEConfig:
    """Mirror of ``AutoencoderKLQwenImage.config`` (decoder half)."""

    base_dim: int = 96
    z_dim: int = 16
    dim_mult: Tuple[int, ...] = (1, 2, 4, 4)
    num_res_blocks: int = 2
    temperal_downsample: Tuple[bool, ...] = (False, True, True)

    @property
    def dims(self) -> List[int]:
        m = self.dim_mult
        return [self.base_dim * u for u in [m[-1]] + list(m[::-1])]

    def up_blocks(self) -> List[Tuple[int, int, Optional[str]]]:
        """(in_dim, out_dim, upsample mode) per up block (QwenImageDecoder3d.__init__)."""
        d = self.dims
        ups = list(self.temperal_downsample[::-1])
        out = []
        for i, (a, b) in enumerate(zip(d[:-1], d[1:])):
            if i > 0:
                a //= 2
            mode = None
            if i != len(self.dim_mult) - 1:
                mode = "upsample3d" if ups[i] else "upsample2d"
            out.append((a, b, mode))
        return out


def decoder_param_shapes(cfg: VAEConfig) -> Dict[str, Tuple[int, ...]]:
    """diffusers state_dict names and shapes of the decode path (decoder.* + post_quant_conv)."""
    z, d = cfg.z_dim, cfg.dims
    s: Dict[str, Tuple[int, ...]] = {
        "post_quant_conv.weight": (z, z, 1, 1, 1), "post_quant_conv.bias": (z,),
        "decoder.conv_in.weight": (d[0], z, 3, 3, 3), "decoder.conv_in.bias": (d[0],),
    }

    def res(prefix, a, b):
        s[f"{prefix}.norm1.gamma"] = (a, 1, 1, 1)
        s[f"{prefix}.conv1.weight"] = (b, a, 3, 3, 3)
        s[f"{prefix}.conv1.bias"] = (b,)
        s[f"{prefix}.norm2.gamma"] = (b, 1, 1, 1)
        s[f"{prefix}.conv2.weight"] = (b, b, 3, 3, 3)
        s[f"{prefix}.conv2.bias"] = (b,)
        if a != b:
            s[f"{prefix}.conv_shortcut.weight"] = (b, a, 1, 1, 1)
            s[f"{prefix}.conv_shortcut.bias"] = (b,)

    res("decoder.mid_block.resnets.0", d[0], d[0])
    res("decoder.mid_block.resnets.1", d[0], d[0])
    a = "decoder.mid_block.attentions.0"
    s[f"{a}.norm.gamma"] = (d[0], 1, 1)
    s[f"{a}.to_qkv.weight"] = (3 * d[0], d[0], 1, 1)
    s[f"{a}.to_qkv.bias"] = (3 * d[0],)
    s[f"{a}.proj.weight"] = (d[0], d[0], 1, 1)
    s[f"{a}.proj.bias"] = (d[0],)
    for i, (a_, b_, mode) in enumerate(cfg.up_blocks()):
        cur = a_
        for r in range(cfg.num_res_blocks + 1):
            res(f"decoder.up_blocks.{i}.resnets.{r}", cur, b_)
            cur = b_
        if mode is not None:
            s[f"decoder.up_blocks.{i}.upsamplers.0.resample.1.weight"] = (b_ // 2, b_, 3, 3)
            s[f"decoder.up_blocks.{i}.upsamplers.0.resample.1.bias"] = (b_ // 2,)
            if mode == "upsample3d":
                s[f"decoder.up_blocks.{i}.upsamplers.0.time_conv.weight"] = (2 * b_, b_, 3, 1, 1)
                s[f"decoder.up_blocks.{i}.upsamplers.0.time_conv.bias"] = (2 * b_,)
    s["decoder.norm_out.gamma"] = (d[-1], 1, 1, 1)
    s["decoder.conv_out.weight"] = (3, d[-1], 3, 3, 3)
    s["decoder.conv_out.bias"] = (3,)
    return s


def random_params(cfg: VAEConfig, seed: int = 0) -> Dict[str, torch.Tensor]:
    """Deterministic random weights of the decode path, bf16 (fan-in scaled normal, gammas near 1)."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name, shp in decoder_param_shapes(cfg).items():
        if name.endswith("gamma"):
            t = 1.0 + 0.05 * torch.randn(shp, generator=g)
        elif name.endswith("bias"):
            t = 0.02 * torch.randn(shp, generator=g)
        else:
            fan_in = math.prod(shp[1:])
            t = torch.randn(shp, generator=g) / math.sqrt(fan_in)
        out[name] = t.to(BF16)
    return out


class _R:
    def __init__(self, on: bool):
        self.on = on

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        return x.to(BF16).float() if self.on else x


def causal_conv3d(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, pad: int, r: _R) -> torch.Tensor:
    """QwenImageCausalConv3d on a clip with no cache: F.pad (space pad, 2*pad zero frames in front)
    then conv3d [U]. x: [B, C, T, H, W] fp32."""
    x = F.pad(x, (pad, pad, pad, pad, 2 * pad, 0))
    return r(F.conv3d(x, w.float(), b.float()))


def rms_norm(x: torch.Tensor, gamma: torch.Tensor, r: _R) -> torch.Tensor:
    """QwenImageRMS_norm(channel_first): F.normalize(x, dim=1) * sqrt(C) * gamma (+ 0.0) [U]."""
    C = x.shape[1]
    n = r(x.norm(p=2, dim=1, keepdim=True)).clamp_min(1e-12)
    y = r(x / n)
    y = r(y * math.sqrt(C))
    return r(y * gamma.float())


def silu(x: torch.Tensor, r: _R) -> torch.Tensor:
    return r(F.silu(x))


def residual_block(p, prefix: str, x: torch.Tensor, r: _R) -> torch.Tensor:
    """QwenImageResidualBlock: shortcut(x) + conv2(silu(norm2(conv1(silu(norm1(x))))))."""
    sc = p.get(f"{prefix}.conv_shortcut.weight")
    h = causal_conv3d(x, sc, p[f"{prefix}.conv_shortcut.bias"], 0, r) if sc is not None else x
    y = silu(rms_norm(x, p[f"{prefix}.norm1.gamma"], r), r)
    y = causal_conv3d(y, p[f"{prefix}.conv1.weight"], p[f"{prefix}.conv1.bias"], 1, r)
    y = silu(rms_norm(y, p[f"{prefix}.norm2.gamma"], r), r)
    y = causal_conv3d(y, p[f"{prefix}.conv2.weight"], p[f"{prefix}.conv2.bias"], 1, r)
    return r(y + h)


def attention_block(p, prefix: str, x: torch.Tensor, r: _R) -> torch.Tensor:
    """QwenImageAttentionBlock: RMS_norm, to_qkv 1x1, one-head SDPA over H*W, proj 1x1, + x."""
    B, C, T, H, W = x.shape
    xi = x.permute(0, 2, 1, 3, 4).reshape(B * T, C, H, W)
    y = rms_norm(xi, p[f"{prefix}.norm.gamma"], r)
    qkv = r(F.conv2d(y, p[f"{prefix}.to_qkv.weight"].float(), p[f"{prefix}.to_qkv.bias"].float()))
    qkv = qkv.reshape(B * T, 1, 3 * C, H * W).permute(0, 1, 3, 2)
    q, k, v = qkv.chunk(3, dim=-1)
    s = q @ k.transpose(-1, -2) / math.sqrt(C)
    a = r(torch.softmax(s, dim=-1) @ v)
    a = a.squeeze(1).permute(0, 2, 1).reshape(B * T, C, H, W)
    o = r(F.conv2d(a, p[f"{prefix}.proj.weight"].float(), p[f"{prefix}.proj.bias"].float()))
    o = o.view(B, T, C, H, W).permute(0, 2, 1, 3, 4)
    return r(o + x)


def resample_up(p, prefix: str, x: torch.Tensor, mode: str, r: _R) -> torch.Tensor:
    """QwenImageResample upsample2d / upsample3d on the first frame (time_conv skipped) [U]:
    nearest-exact 2x (== nearest for an integer factor) + Conv2d(dim, dim//2, 3, padding=1)."""
    B, C, T, H, W = x.shape
    xi = x.permute(0, 2, 1, 3, 4).reshape(B * T, C, H, W)
    xi = F.interpolate(xi, scale_factor=2.0, mode="nearest-exact")
    y = r(F.conv2d(xi, p[f"{prefix}.resample.1.weight"].float(), p[f"{prefix}.resample.1.bias"].float(), padding=1))
    return y.view(B, T, y.shape[1], 2 * H, 2 * W).permute(0, 2, 1, 3, 4)


def unpack_latents(packed: torch.Tensor, h: int, w: int) -> torch.Tensor:
    """_unpack_latents: [B, (h/2)(w/2), 64] -> [B, 16, 1, h, w] (h, w latent pixels) [U]."""
    B, _, Cp = packed.shape
    x = packed.view(B, h // 2, w // 2, Cp // 4, 2, 2).permute(0, 3, 1, 4, 2, 5)
    return x.reshape(B, Cp // 4, 1, h, w)


def decode(p: Dict[str, torch.Tensor], packed: torch.Tensor, h: int, w: int, cfg: VAEConfig = VAEConfig(),
           emulate_bf16: bool = True, mean=LATENTS_MEAN, std=LATENTS_STD) -> torch.Tensor:
    """Pipeline decode tail on packed latents -> image in [-1, 1], [B, 3, 8h, 8w] fp32."""
    r = _R(emulate_bf16)
    z = unpack_latents(packed.float(), h, w)
    mean_t = torch.tensor(mean).view(1, -1, 1, 1, 1).to(BF16).float()
    sinv = (1.0 / torch.tensor(std).view(1, -1, 1, 1, 1).to(BF16).float())
    sinv = r(sinv)
    z = r(r(z / sinv) + mean_t)
    x = causal_conv3d(z, p["post_quant_conv.weight"], p["post_quant_conv.bias"], 0, r)
    x = causal_conv3d(x, p["decoder.conv_in.weight"], p["decoder.conv_in.bias"], 1, r)
    x = residual_block(p, "decoder.mid_block.resnets.0", x, r)
    x = attention_block(p, "decoder.mid_block.attentions.0", x, r)
    x = residual_block(p, "decoder.mid_block.resnets.1", x, r)
    for i, (_, _, mode) in enumerate(cfg.up_blocks()):
        for j in range(cfg.num_res_blocks + 1):
            x = residual_block(p, f"decoder.up_blocks.{i}.resnets.{j}", x, r)
        if mode is not None:
            x = resample_up(p, f"decoder.up_blocks.{i}.upsamplers.0", x, mode, r)
    x = silu(rms_norm(x, p["decoder.norm_out.gamma"], r), r)
    x = causal_conv3d(x, p["decoder.conv_out.weight"], p["decoder.conv_out.bias"], 1, r)
    return x.clamp(-1.0, 1.0)[:, :, 0]


def to_uint8(img: torch.Tensor) -> torch.Tensor:
    """VaeImageProcessor.postprocess(output_type="pil") on a bf16 image: [B, 3, H, W] -> [B, H, W, 3]."""
    u = (img.to(BF16) / 2 + 0.5).clamp(0, 1).float()
    return torch.round(u * 255).to(torch.uint8).permute(0, 2, 3, 1)


def decode_flops(cfg: VAEConfig, h: int, w: int) -> float:
    """Algorithmic FLOPs of one decode (convs as 2-D on one frame, attention 4 P^2 C, 1x1s)."""
    f = 0.0
    d = cfg.dims
    H, W = h, w

    def conv(cin, cout, k, HH, WW):
        return 2.0 * HH * WW * cin * cout * k * k

    f += conv(cfg.z_dim, cfg.z_dim, 1, H, W) + conv(cfg.z_dim, d[0], 3, H, W)

    def res(a, b, HH, WW):
        return conv(a, b, 3, HH, WW) + conv(b, b, 3, HH, WW) + (conv(a, b, 1, HH, WW) if a != b else 0.0)

    f += 2 * res(d[0], d[0], H, W)
    P = H * W
    f += conv(d[0], 3 * d[0], 1, H, W) + 4.0 * P * P * d[0] + conv(d[0], d[0], 1, H, W)
    for a, b, mode in cfg.up_blocks():
        cur = a
        for _ in range(cfg.num_res_blocks + 1):
            f += res(cur, b, H, W)
            cur = b
        if mode is not None:
            H, W = 2 * H, 2 * W
            f += conv(b, b // 2, 3, H, W)
    f += conv(d[-1], 3, 3, H, W)
    return f


# ---------------------------------------------------------------------------- encoder
def encoder_param_shapes(cfg: VAEConfig) -> Dict[str, Tuple[int, ...]]:
    """diffusers names/shapes of the encode path: QwenImageEncoder3d (``encoder.*``; down_blocks is
    one flat ModuleList of resnets and Resample downsamplers) and ``quant_conv`` [U]."""
    dims = [cfg.base_dim * u for u in [1] + list(cfg.dim_mult)]
    z2 = 2 * cfg.z_dim
    s: Dict[str, Tuple[int, ...]] = {"encoder.conv_in.weight": (dims[0], 3, 3, 3, 3), "encoder.conv_in.bias": (dims[0],)}

    def res(prefix, a, b):
        s[f"{prefix}.norm1.gamma"] = (a, 1, 1, 1)
        s[f"{prefix}.conv1.weight"] = (b, a, 3, 3, 3)
        s[f"{prefix}.conv1.bias"] = (b,)
        s[f"{prefix}.norm2.gamma"] = (b, 1, 1, 1)
        s[f"{prefix}.conv2.weight"] = (b, b, 3, 3, 3)
        s[f"{prefix}.conv2.bias"] = (b,)
        if a != b:
            s[f"{prefix}.conv_shortcut.weight"] = (b, a, 1, 1, 1)
            s[f"{prefix}.conv_shortcut.bias"] = (b,)

    idx = 0
    for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
        for _ in range(cfg.num_res_blocks):
            res(f"encoder.down_blocks.{idx}", a, b)
            idx += 1
            a = b
        if i != len(cfg.dim_mult) - 1:
            s[f"encoder.down_blocks.{idx}.resample.1.weight"] = (b, b, 3, 3)
            s[f"encoder.down_blocks.{idx}.resample.1.bias"] = (b,)
            if cfg.temperal_downsample[i]:
                s[f"encoder.down_blocks.{idx}.time_conv.weight"] = (b, b, 3, 1, 1)
                s[f"encoder.down_blocks.{idx}.time_conv.bias"] = (b,)
            idx += 1
    top = dims[-1]
    res("encoder.mid_block.resnets.0", top, top)
    res("encoder.mid_block.resnets.1", top, top)
    a = "encoder.mid_block.attentions.0"
    s[f"{a}.norm.gamma"] = (top, 1, 1)
    s[f"{a}.to_qkv.weight"] = (3 * top, top, 1, 1)
    s[f"{a}.to_qkv.bias"] = (3 * top,)
    s[f"{a}.proj.weight"] = (top, top, 1, 1)
    s[f"{a}.proj.bias"] = (top,)
    s["encoder.norm_out.gamma"] = (top, 1, 1, 1)
    s["encoder.conv_out.weight"] = (z2, top, 3, 3, 3)
    s["encoder.conv_out.bias"] = (z2,)
    s["quant_conv.weight"] = (z2, z2, 1, 1, 1)
    s["quant_conv.bias"] = (z2,)
    return s


def random_encoder_params(cfg: VAEConfig, seed: int = 0) -> Dict[str, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name, shp in encoder_param_shapes(cfg).items():
        if name.endswith("gamma"):
            t = 1.0 + 0.05 * torch.randn(shp, generator=g)
        elif name.endswith("bias"):
            t = 0.02 * torch.randn(shp, generator=g)
        else:
            t = torch.randn(shp, generator=g) / math.sqrt(math.prod(shp[1:]))
        out[name] = t.to(BF16)
    return out


def resample_down(p, prefix: str, x: torch.Tensor, r: _R) -> torch.Tensor:
    """QwenImageResample downsample2d / downsample3d on the first frame (time_conv skipped: its
    feat_cache entry starts empty) [U]: ZeroPad2d((0, 1, 0, 1)) + Conv2d(dim, dim, 3, stride=2)."""
    B, C, T, H, W = x.shape
    xi = x.permute(0, 2, 1, 3, 4).reshape(B * T, C, H, W)
    xi = F.pad(xi, (0, 1, 0, 1))
    y = r(F.conv2d(xi, p[f"{prefix}.resample.1.weight"].float(), p[f"{prefix}.resample.1.bias"].float(), stride=2))
    return y.view(B, T, C, y.shape[2], y.shape[3]).permute(0, 2, 1, 3, 4)


def pack_latents(z: torch.Tensor) -> torch.Tensor:
    """_pack_latents: [B, 16, 1, h, w] -> [B, (h/2)(w/2), 64] [U]."""
    B, C, _, h, w = z.shape
    return z.view(B, C, h // 2, 2, w // 2, 2).permute(0, 2, 4, 1, 3, 5).reshape(B, (h // 2) * (w // 2), C * 4)


def encode(p: Dict[str, torch.Tensor], rgb: torch.Tensor, cfg: VAEConfig = VAEConfig(), emulate_bf16: bool = True,
           mean=LATENTS_MEAN, std=LATENTS_STD) -> torch.Tensor:
    """uint8 RGB [B, H, W, 3] -> packed normalised condition latents [B, (H/16)(W/16), 64]:
    preprocess (2 v/255 - 1, bf16), vae.encode (encoder + quant_conv), mode, (mu - mean) / std."""
    r = _R(emulate_bf16)
    x = r(2.0 * (rgb.float() / 255.0) - 1.0).permute(0, 3, 1, 2)[:, :, None]
    x = causal_conv3d(x, p["encoder.conv_in.weight"], p["encoder.conv_in.bias"], 1, r)
    dims = [cfg.base_dim * u for u in [1] + list(cfg.dim_mult)]
    idx = 0
    for i in range(len(dims) - 1):
        for _ in range(cfg.num_res_blocks):
            x = residual_block(p, f"encoder.down_blocks.{idx}", x, r)
            idx += 1
        if i != len(cfg.dim_mult) - 1:
            x = resample_down(p, f"encoder.down_blocks.{idx}", x, r)
            idx += 1
    x = residual_block(p, "encoder.mid_block.resnets.0", x, r)
    x = attention_block(p, "encoder.mid_block.attentions.0", x, r)
    x = residual_block(p, "encoder.mid_block.resnets.1", x, r)
    x = silu(rms_norm(x, p["encoder.norm_out.gamma"], r), r)
    x = causal_conv3d(x, p["encoder.conv_out.weight"], p["encoder.conv_out.bias"], 1, r)
    x = causal_conv3d(x, p["quant_conv.weight"], p["quant_conv.bias"], 0, r)
    mu = x[:, : cfg.z_dim]  # DiagonalGaussianDistribution.mode()
    mean_t = torch.tensor(mean).view(1, -1, 1, 1, 1).to(BF16).float()
    std_t = torch.tensor(std).view(1, -1, 1, 1, 1).to(BF16).float()
    z = r(r(mu - mean_t) / std_t)
    return pack_latents(z)
