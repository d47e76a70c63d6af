"""VAE decoder on the HIP path: AutoencoderKLQwenImage.decode for one frame.

Replaces the decode tail the reference reaches through ``QwenImageEditPlusPipeline.__call__``
(server.py:137-153, qwen_realtime.py:247-255) and its dead helper ``decode_latent``
(qwen_realtime.py:188-199): ``_unpack_latents``, ``latents / (1/std) + mean``,
``vae.decode(z)[:, :, 0]`` (post_quant_conv + QwenImageDecoder3d + clamp) and the image
processor's uint8 conversion [U: diffusers autoencoder_kl_qwenimage.py].

MI355X design:
  * activations NHWC bf16 ([pixels][channels]), so each per-pixel norm is one contiguous row and
    each convolution is a GEMM with K = (tap, channel);
  * a causal 3x3x3 conv on the first frame sees two zero frames in front, so it IS the 2-D conv
    with the kernel's last temporal slice -- weights are reduced and re-laid [Cout][ky][kx][Cin]
    (K zero-padded to 64) once at load;
  * every conv is qie_conv2d_bf16 (implicit GEMM, taps gathered per lane by LDS-DMA, no im2col
    buffer); the Resample nearest-2x upsample is folded into the gather of the conv after it;
    the ResidualBlock sum rides the second conv's epilogue;
  * the mid-block single-head attention (P = h*w tokens, C = 384): fp32 scores by one GEMM, a
    row softmax kernel, P.V by the bf16 GEMM against V^T;
  * the decode tail (clamp, (x/2+0.5).clamp(0,1), round(255 v)) writes uint8 RGB on the device.
The reference's ``upsample3d`` time_conv is skipped on the first frame (``feat_cache`` "Rep"),
so its weights are accepted but unused, as upstream.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

from . import ops

BF16 = torch.bfloat16

# AutoencoderKLQwenImage config defaults [U] (vae/config.json of Qwen-Image: Wan-2.1 statistics)
LATENTS_MEAN = (-0.7571, -0.7089, -0.9113, 0.1075, -0.1745, 0.9653, -0.1517, 1.5508,
                0.4134, -0.0715, 0.5517, -0.3632, -0.1922, -0.9497, 0.2503, -0.2921)
LATENTS_STD = (2.8184, 1.4541, 2.3275, 2.6558, 1.2196, 1.7708, 2.6052, 2.0743,
               3.2687, 2.1526, 2.8652, 1.5579, 1.6382, 1.1253, 2.8251, 1.9160)


@dataclass
class VAEConfig:
    """The decoder half of ``AutoencoderKLQwenImage.config``."""

    base_dim: int = 96
    z_dim: int = 16
    dim_mult: Tuple[int, ...] = (1, 2, 4, 4)
    num_res_blocks: int = 2
    temperal_downsample: Tuple[bool, ...] = (False, True, True)
    latents_mean: Tuple[float, ...] = LATENTS_MEAN
    latents_std: Tuple[float, ...] = LATENTS_STD
    scaling_factor: float = 1.0  # unused by the Qwen pipeline (it de-normalises with mean / std)

    @property
    def dims(self) -> List[int]:
        m = self.dim_mult
        return [self.base_dim * u for u in [m[-1]] + list(m[::-1])]

    def up_blocks(self) -> List[Tuple[int, int, Optional[str]]]:
        """(in_dim, out_dim, upsample mode) per up block, as QwenImageDecoder3d.__init__ builds them."""
        d, ups, out = self.dims, list(self.temperal_downsample[::-1]), []
        for i, (a, b) in enumerate(zip(d[:-1], d[1:])):
            if i > 0:
                a //= 2
            mode = None
            if i != len(self.dim_mult) - 1:
                mode = "upsample3d" if ups[i] else "upsample2d"
            out.append((a, b, mode))
        return out


def _res_names(prefix: str, a: int, b: int) -> Dict[str, Tuple[int, ...]]:
    s = {f"{prefix}.norm1.gamma": (a, 1, 1, 1), f"{prefix}.conv1.weight": (b, a, 3, 3, 3), f"{prefix}.conv1.bias": (b,),
         f"{prefix}.norm2.gamma": (b, 1, 1, 1), f"{prefix}.conv2.weight": (b, b, 3, 3, 3), f"{prefix}.conv2.bias": (b,)}
    if a != b:
        s[f"{prefix}.conv_shortcut.weight"] = (b, a, 1, 1, 1)
        s[f"{prefix}.conv_shortcut.bias"] = (b,)
    return s


def state_dict_shapes(cfg: VAEConfig) -> Dict[str, Tuple[int, ...]]:
    """diffusers state_dict names/shapes of the decode path (``decoder.*``, ``post_quant_conv.*``)."""
    z, d = cfg.z_dim, cfg.dims
    s: Dict[str, Tuple[int, ...]] = {"post_quant_conv.weight": (z, z, 1, 1, 1), "post_quant_conv.bias": (z,),
                                     "decoder.conv_in.weight": (d[0], z, 3, 3, 3), "decoder.conv_in.bias": (d[0],)}
    s.update(_res_names("decoder.mid_block.resnets.0", d[0], d[0]))
    s.update(_res_names("decoder.mid_block.resnets.1", d[0], d[0]))
    a = "decoder.mid_block.attentions.0"
    s.update({f"{a}.norm.gamma": (d[0], 1, 1), f"{a}.to_qkv.weight": (3 * d[0], d[0], 1, 1),
              f"{a}.to_qkv.bias": (3 * d[0],), f"{a}.proj.weight": (d[0], d[0], 1, 1), f"{a}.proj.bias": (d[0],)})
    for i, (a_, b_, mode) in enumerate(cfg.up_blocks()):
        cur = a_
        for r in range(cfg.num_res_blocks + 1):
            s.update(_res_names(f"decoder.up_blocks.{i}.resnets.{r}", cur, b_))
            cur = b_
        if mode is not None:
            u = f"decoder.up_blocks.{i}.upsamplers.0"
            s[f"{u}.resample.1.weight"] = (b_ // 2, b_, 3, 3)
            s[f"{u}.resample.1.bias"] = (b_ // 2,)
            if mode == "upsample3d":
                s[f"{u}.time_conv.weight"] = (2 * b_, b_, 3, 1, 1)
                s[f"{u}.time_conv.bias"] = (2 * b_,)
    s.update({"decoder.norm_out.gamma": (d[-1], 1, 1, 1), "decoder.conv_out.weight": (3, d[-1], 3, 3, 3),
              "decoder.conv_out.bias": (3,)})
    return s


def conv_weight(w: torch.Tensor, n_pad: int = 0, cin_pad: int = 0) -> torch.Tensor:
    """A causal conv3d [Cout, Cin, kt, k, k] / conv2d [Cout, Cin, k, k] weight as the
    [Cout (+n_pad)][conv_kpad] bf16 rows qie_conv2d_bf16 reads: the last temporal slice (the only
    tap a first frame meets behind its causal zero padding), K order [ky][kx][Cin (+cin_pad zero
    channels)], zero padded to a multiple of 64."""
    if w.dim() == 5:
        w = w[:, :, -1]
    if cin_pad:
        w = torch.cat([w, torch.zeros(w.shape[0], cin_pad, *w.shape[2:], dtype=w.dtype, device=w.device)], 1)
    co, ci, k, _ = w.shape
    rows = w.permute(0, 2, 3, 1).reshape(co, k * k * ci)
    out = torch.zeros(co + n_pad, ops.conv_kpad(ci, k), dtype=BF16, device=w.device)
    out[:co, : k * k * ci] = rows.to(BF16)
    return out


def _random_sd(shapes: Dict[str, Tuple[int, ...]], seed: int) -> Dict[str, torch.Tensor]:
    """Random weights of the real architecture (fan-in scaled normal; gammas near 1)."""
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for name, shp in shapes.items():
        if name.endswith("gamma"):
            t = 1.0 + 0.05 * torch.randn(shp, generator=g)
        elif name.endswith("bias"):
            t = 0.02 * torch.randn(shp, generator=g)
        else:
            t = torch.randn(shp, generator=g) / math.sqrt(math.prod(shp[1:]))
        sd[name] = t.to(BF16)
    return sd


def _convert(sd: Dict[str, torch.Tensor], shapes: Dict[str, Tuple[int, ...]], dev, strict: bool, what: str,
             special: Dict[str, dict]) -> Dict[str, torch.Tensor]:
    """Check names/shapes and convert a (de|en)coder state_dict to the kernel layouts: gammas and
    biases flat bf16, convs to conv_weight rows (``special[name]`` = its extra kwargs), the
    upsample3d / downsample3d time_conv dropped (never applied to a first frame)."""
    missing = [k for k in shapes if k not in sd]
    if strict and missing:
        raise KeyError(f"missing VAE {what} weights: {missing[:5]}{'...' if len(missing) > 5 else ''}")
    w = {}
    for k, shp in shapes.items():
        t = sd[k]
        if tuple(t.shape) != shp:
            raise ValueError(f"{k}: shape {tuple(t.shape)} != {shp}")
        t = t.to(dev)
        if k.endswith("gamma"):
            w[k] = t.reshape(-1).to(BF16).contiguous()
        elif k.endswith("bias"):
            w[k] = t.to(BF16).contiguous()
        elif "time_conv" in k:
            continue
        else:
            w[k] = conv_weight(t, **special.get(k, {}))
    return w


class _VAEBlocks:
    """The resnet / attention blocks both VAE halves share (NHWC, on the workspace buffers
    "t", "y", "qkv", "vt", "att", the flash-attention workspace "attn_ws" (or, for C != 384, the
    materialised "s", "p", "zero_b") and the free activation buffer named)."""

    w: Dict[str, torch.Tensor]

    @staticmethod
    def _view(buf: torch.Tensor, P: int, C: int) -> torch.Tensor:
        return buf[: P * C].view(P, C)

    # ------------------------------------------------------------------ forward
    def _resnet(self, ws, prefix: str, x: torch.Tensor, H: int, W: int, a: int, b: int, free: List[str]):
        """QwenImageResidualBlock on NHWC x [H*W, a] -> [H*W, b]; returns (out, its buffer name)."""
        P = H * W
        wt = self.w
        t = self._view(ws["t"], P, a)
        ops.vae_rms_norm(x, wt[f"{prefix}.norm1.gamma"], True, out=t)
        y = self._view(ws["y"], P, b)
        ops.conv2d_rmsnorm(t, H, W, wt[f"{prefix}.conv1.weight"], wt[f"{prefix}.conv1.bias"],
                           wt[f"{prefix}.norm2.gamma"], True, out=y)  # conv1 + norm2 (+ SiLU)
        if a != b:  # shortcut into a free buffer; conv2 adds onto it
            name = free[0]
            h = self._view(ws[name], P, b)
            ops.conv2d(x, H, W, wt[f"{prefix}.conv_shortcut.weight"], wt[f"{prefix}.conv_shortcut.bias"], ksize=1,
                       out=h)
        else:
            name, h = None, x
        ops.conv2d(y, H, W, wt[f"{prefix}.conv2.weight"], wt[f"{prefix}.conv2.bias"], out=h, residual=True)
        return h, name

    def _attention(self, ws, prefix: str, x: torch.Tensor, H: int, W: int, C: int):
        """QwenImageAttentionBlock: x += proj(SDPA(to_qkv(norm(x)))), one head over H*W tokens."""
        P = H * W
        wt = self.w
        t = self._view(ws["t"], P, C)
        ops.vae_rms_norm(x, wt[f"{prefix}.norm.gamma"], False, out=t)
        qkv = ws["qkv"][:P]
        ops.conv2d(t, H, W, wt[f"{prefix}.to_qkv.weight"], wt[f"{prefix}.to_qkv.bias"], ksize=1, out=qkv)
        q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
        vt = ws["vt"]  # [C, roundup(P, 64)], zero past column P
        ops.transpose(v, out=vt[:, :P])
        att = ws["att"][:P]
        if "attn_ws" in ws:  # flash form (C = 384, the real model): no score matrix
            ops.vae_attention(qkv, vt, att, ws["attn_ws"])
        else:
            s = ws["s"]
            ops.matmul_f32out(q, k, out=s)
            p = ws["p"]  # [P, roundup(P, 64)], zero past column P
            ops.softmax_rows(s, 1.0 / math.sqrt(C), out=p)
            ops.linear(p, vt, ws["zero_b"][:C], out=att)
        ops.conv2d(att, H, W, wt[f"{prefix}.proj.weight"], wt[f"{prefix}.proj.bias"], ksize=1, out=x, residual=True)


    @staticmethod
    def _attn_buffers(P0: int, C0: int, dev) -> Dict[str, torch.Tensor]:
        """Mid-block attention over P0 tokens of C0 channels: K of P.V padded to 64 (zero P
        columns from the softmax kernel, zero V^T columns here)."""
        e = dict(dtype=BF16, device=dev)
        kp = -(-P0 // 64) * 64
        bufs = {"qkv": torch.empty(P0, 3 * C0, **e), "vt": torch.zeros(C0, kp, **e), "att": torch.empty(P0, C0, **e)}
        if C0 == 384:  # qie_vae_attention_bf16: fp32 partials of the key-range splits only
            nb = ops.vae_attention_workspace_bytes(P0, C0)
            bufs["attn_ws"] = torch.empty(-(-nb // 4), dtype=torch.float32, device=dev)
        else:
            bufs.update({"s": torch.empty(P0, P0, dtype=torch.float32, device=dev), "p": torch.empty(P0, kp, **e),
                         "zero_b": torch.zeros(C0, **e)})
        return bufs


class QwenImageVAEDecoder(_VAEBlocks):
    """``vae.decode`` + pipeline decode tail on the HIP path. ``decode(packed, h, w)`` takes the
    pipeline's packed latents [B, (h/2)(w/2), 64] (h, w in latent pixels) and returns uint8 RGB
    [B, 8h, 8w, 3] on the device (``output="pt"``: the clamped bf16 image [B, 3, 8h, 8w])."""

    def __init__(self, config: Optional[VAEConfig] = None, device="cuda"):
        self.config = config or VAEConfig()
        self.device = torch.device(device)
        if any(c % 8 for c in self.config.dims) or self.config.z_dim != 16:
            raise NotImplementedError("the conv kernels need channel counts % 8 == 0 and z_dim 16")
        self.w: Dict[str, torch.Tensor] = {}
        self._ws: Dict[Tuple[int, int], Dict[str, torch.Tensor]] = {}

    # ------------------------------------------------------------------ weights
    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True) -> "QwenImageVAEDecoder":
        """diffusers AutoencoderKLQwenImage state_dict (``decoder.*`` / ``post_quant_conv.*``; the
        encoder half is ignored)."""
        dev = self.device
        w = _convert(sd, state_dict_shapes(self.config), dev, strict, "decoder",
                     {"decoder.conv_out.weight": {"n_pad": 1}})  # 3 -> 4 output channels (N % 4)
        pq = sd["post_quant_conv.weight"]
        w["post_quant_conv.weight"] = pq.reshape(pq.shape[0], pq.shape[1]).to(dev).to(BF16).contiguous()
        w["decoder.conv_out.bias"] = torch.cat([w["decoder.conv_out.bias"], torch.zeros(1, dtype=BF16, device=dev)])
        c = self.config
        std = torch.tensor(c.latents_std, dtype=torch.float32).to(BF16)
        w["sinv"] = (1.0 / std.float()).to(BF16).to(dev)  # 1.0 / bf16 tensor -> bf16 (pipeline)
        w["mean"] = torch.tensor(c.latents_mean, dtype=torch.float32).to(BF16).to(dev)
        self.w = w
        return self

    def random_init_(self, seed: int = 0) -> "QwenImageVAEDecoder":
        """Random weights of the real architecture (fan-in scaled normal; gammas near 1)."""
        return self.load_state_dict(_random_sd(state_dict_shapes(self.config), seed))

    # ------------------------------------------------------------------ workspace
    def _workspace(self, h: int, w: int) -> Dict[str, torch.Tensor]:
        key = (h, w)
        if key not in self._ws:
            c, dev = self.config, self.device
            P0 = h * w
            # activation buffers hold the largest pixels x channels of any stage
            sizes, P = [P0 * c.dims[0]], P0
            for a, b, mode in c.up_blocks():
                sizes.append(P * max(a, b))
                if mode is not None:
                    P *= 4
                    sizes.append(P * (b // 2))
            n = max(sizes)
            e = dict(dtype=BF16, device=dev)
            C0 = c.dims[0]
            self._ws[key] = {
                "a": torch.empty(n, **e), "b": torch.empty(n, **e), "t": torch.empty(n, **e), "y": torch.empty(n, **e),
                "z": torch.empty(P0, 16, **e), "out": torch.empty(P, 4, **e), **self._attn_buffers(P0, C0, dev)}
        return self._ws[key]

    def decode(self, packed: torch.Tensor, h: int, w: int, output: str = "uint8") -> torch.Tensor:
        c, wt = self.config, self.w
        if not wt:
            raise RuntimeError("VAE weights not loaded (load_state_dict / random_init_)")
        B = packed.shape[0]
        ws = self._workspace(h, w)
        outs = []
        for bi in range(B):
            z = ws["z"]
            ops.vae_latents_in(packed[bi:bi + 1].contiguous(), h, w, wt["sinv"], wt["mean"],
                               wt["post_quant_conv.weight"], wt["post_quant_conv.bias"], out=z)
            H, W = h, w
            C = c.dims[0]
            cur, other = "a", "b"
            x = self._view(ws[cur], H * W, C)
            ops.conv2d(z, H, W, wt["decoder.conv_in.weight"], wt["decoder.conv_in.bias"], out=x)
            x, _ = self._resnet(ws, "decoder.mid_block.resnets.0", x, H, W, C, C, [other])
            self._attention(ws, "decoder.mid_block.attentions.0", x, H, W, C)
            x, _ = self._resnet(ws, "decoder.mid_block.resnets.1", x, H, W, C, C, [other])
            for i, (a, b, mode) in enumerate(c.up_blocks()):
                for r in range(c.num_res_blocks + 1):
                    x, name = self._resnet(ws, f"decoder.up_blocks.{i}.resnets.{r}", x, H, W, a if r == 0 else b, b,
                                           [other])
                    if name is not None:
                        cur, other = name, cur
                if mode is not None:
                    u = f"decoder.up_blocks.{i}.upsamplers.0.resample.1"
                    nx = self._view(ws[other], 4 * H * W, b // 2)
                    ops.conv2d(x, H, W, wt[f"{u}.weight"], wt[f"{u}.bias"], up=True, out=nx)
                    cur, other = other, cur
                    x = nx
                    H, W = 2 * H, 2 * W
            Cl = c.dims[-1]
            t = self._view(ws["t"], H * W, Cl)
            ops.vae_rms_norm(x, wt["decoder.norm_out.gamma"], True, out=t)
            o = ws["out"][: H * W]
            ops.conv2d(t, H, W, wt["decoder.conv_out.weight"], wt["decoder.conv_out.bias"], out=o)
            if output == "uint8":
                outs.append(ops.vae_rgb_out(o).view(H, W, 3))
            else:
                outs.append(o[:, :3].clamp(-1, 1).reshape(H, W, 3).permute(2, 0, 1).clone())
        return torch.stack(outs)

    def flops(self, h: int, w: int) -> float:
        """Algorithmic FLOPs of one decode at latent size h x w (2-D convs, attention 4 P^2 C)."""
        c = self.config
        d = c.dims

        def conv(ci, co, k, P):
            return 2.0 * P * ci * co * k * k

        def res(a, b, P):
            return conv(a, b, 3, P) + conv(b, b, 3, P) + (conv(a, b, 1, P) if a != b else 0.0)

        P = h * w
        f = conv(16, 16, 1, P) + conv(16, d[0], 3, P) + 2 * res(d[0], d[0], P)
        f += conv(d[0], 3 * d[0], 1, P) + 4.0 * P * P * d[0] + conv(d[0], d[0], 1, P)
        for a, b, mode in c.up_blocks():
            cur = a
            for _ in range(c.num_res_blocks + 1):
                f += res(cur, b, P)
                cur = b
            if mode is not None:
                P *= 4
                f += conv(b, b // 2, 3, P)
        return f + conv(d[-1], 3, 3, P)


# ============================================================================ encoder
def encoder_plan(cfg: VAEConfig) -> List[Tuple]:
    """QwenImageEncoder3d.down_blocks as a flat list (the diffusers ModuleList indices):
    ("res", idx, in, out) and ("down", idx, C, mode)."""
    dims = [cfg.base_dim * u for u in (1,) + tuple(cfg.dim_mult)]
    plan, idx = [], 0
    for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
        for _ in range(cfg.num_res_blocks):
            plan.append(("res", idx, a, b))
            idx += 1
            a = b
        if i != len(cfg.dim_mult) - 1:
            plan.append(("down", idx, b, "downsample3d" if cfg.temperal_downsample[i] else "downsample2d"))
            idx += 1
    return plan


def encoder_state_dict_shapes(cfg: VAEConfig) -> Dict[str, Tuple[int, ...]]:
    """diffusers state_dict names/shapes of the encode path (``encoder.*``, ``quant_conv.*``)."""
    z2 = 2 * cfg.z_dim
    d0 = cfg.base_dim
    s: Dict[str, Tuple[int, ...]] = {"encoder.conv_in.weight": (d0, 3, 3, 3, 3), "encoder.conv_in.bias": (d0,)}
    top = d0
    for op in encoder_plan(cfg):
        if op[0] == "res":
            s.update(_res_names(f"encoder.down_blocks.{op[1]}", op[2], op[3]))
            top = op[3]
        else:
            u = f"encoder.down_blocks.{op[1]}"
            s[f"{u}.resample.1.weight"] = (op[2], op[2], 3, 3)
            s[f"{u}.resample.1.bias"] = (op[2],)
            if op[3] == "downsample3d":
                s[f"{u}.time_conv.weight"] = (op[2], op[2], 3, 1, 1)
                s[f"{u}.time_conv.bias"] = (op[2],)
    s.update(_res_names("encoder.mid_block.resnets.0", top, top))
    s.update(_res_names("encoder.mid_block.resnets.1", top, top))
    a = "encoder.mid_block.attentions.0"
    s.update({f"{a}.norm.gamma": (top, 1, 1), f"{a}.to_qkv.weight": (3 * top, top, 1, 1),
              f"{a}.to_qkv.bias": (3 * top,), f"{a}.proj.weight": (top, top, 1, 1), f"{a}.proj.bias": (top,)})
    s.update({"encoder.norm_out.gamma": (top, 1, 1, 1), "encoder.conv_out.weight": (z2, top, 3, 3, 3),
              "encoder.conv_out.bias": (z2,), "quant_conv.weight": (z2, z2, 1, 1, 1), "quant_conv.bias": (z2,)})
    return s


class QwenImageVAEEncoder(_VAEBlocks):
    """``vae.encode`` + the pipeline's ``_encode_vae_image`` tail on the HIP path, one frame:
    uint8 RGB [B, H, W, 3] (device) -> image processor normalisation -> QwenImageEncoder3d
    (conv_in, down blocks with stride-2 Resamples folded into the conv gather, mid block,
    RMS_norm + SiLU + conv_out) -> quant_conv -> DiagonalGaussian mode (mu) ->
    ``(mu - mean) / std`` -> packed latents [B, (H/16)(W/16), 64] (the
    reference reaches it through QwenImageEditPlusPipeline.__call__ at server.py:137-153 and
    the dead helper ``encode_image`` at qwen_realtime.py:167-186). The ``downsample3d`` time_conv
    is skipped on a first frame, as upstream (its feat_cache starts empty)."""

    def __init__(self, config: Optional[VAEConfig] = None, device="cuda"):
        self.config = config or VAEConfig()
        self.device = torch.device(device)
        if self.config.base_dim % 8 or self.config.z_dim != 16:
            raise NotImplementedError("the conv kernels need channel counts % 8 == 0 and z_dim 16")
        self.w: Dict[str, torch.Tensor] = {}
        self._ws: Dict[Tuple[int, int], Dict[str, torch.Tensor]] = {}

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True) -> "QwenImageVAEEncoder":
        """diffusers AutoencoderKLQwenImage state_dict (``encoder.*`` / ``quant_conv.*``)."""
        dev = self.device
        w = _convert(sd, encoder_state_dict_shapes(self.config), dev, strict, "encoder",
                     {"encoder.conv_in.weight": {"cin_pad": 5}})  # RGB -> 8 gathered channels
        c = self.config
        w["mean"] = torch.tensor(c.latents_mean, dtype=torch.float32).to(BF16).to(dev)
        w["std"] = torch.tensor(c.latents_std, dtype=torch.float32).to(BF16).to(dev)
        self.w = w
        return self

    def random_init_(self, seed: int = 0) -> "QwenImageVAEEncoder":
        return self.load_state_dict(_random_sd(encoder_state_dict_shapes(self.config), seed))

    def _workspace(self, H: int, W: int) -> Dict[str, torch.Tensor]:
        key = (H, W)
        if key not in self._ws:
            c, dev = self.config, self.device
            P, sizes, top = H * W, [H * W * 8], c.base_dim
            for op in encoder_plan(c):
                if op[0] == "res":
                    sizes.append(P * max(op[2], op[3]))
                    top = op[3]
                else:
                    P //= 4
            e = dict(dtype=BF16, device=dev)
            n = max(sizes + [H * W * c.base_dim])
            self._ws[key] = {"a": torch.empty(n, **e), "b": torch.empty(n, **e), "t": torch.empty(n, **e),
                             "y": torch.empty(n, **e), "rgb8": torch.empty(H * W, 8, **e),
                             "zq": torch.empty(P, 2 * c.z_dim, **e), "zo": torch.empty(P, 2 * c.z_dim, **e),
                             **self._attn_buffers(P, top, dev)}
        return self._ws[key]

    def encode(self, rgb: torch.Tensor) -> torch.Tensor:
        """uint8 RGB [B, H, W, 3] on the device (H, W multiples of 16) -> packed latents."""
        c, wt = self.config, self.w
        if not wt:
            raise RuntimeError("VAE encoder weights not loaded (load_state_dict / random_init_)")
        B, H0, W0, _ = rgb.shape
        if H0 % 16 or W0 % 16:
            raise ValueError("image height and width must be multiples of 16")
        ws = self._workspace(H0, W0)
        outs = []
        for bi in range(B):
            x8 = ops.vae_rgb_in(rgb[bi].reshape(-1, 3).contiguous(), out=ws["rgb8"])
            H, W, C = H0, W0, c.base_dim
            cur, other = "a", "b"
            x = self._view(ws[cur], H * W, C)
            ops.conv2d(x8, H, W, wt["encoder.conv_in.weight"], wt["encoder.conv_in.bias"], out=x)
            for op in encoder_plan(c):
                if op[0] == "res":
                    x, name = self._resnet(ws, f"encoder.down_blocks.{op[1]}", x, H, W, op[2], op[3], [other])
                    if name is not None:
                        cur, other = name, cur
                    C = op[3]
                else:
                    u = f"encoder.down_blocks.{op[1]}.resample.1"
                    nx = self._view(ws[other], (H // 2) * (W // 2), C)
                    ops.conv2d(x, H, W, wt[f"{u}.weight"], wt[f"{u}.bias"], down=True, out=nx)
                    cur, other = other, cur
                    x = nx
                    H, W = H // 2, W // 2
            x, _ = self._resnet(ws, "encoder.mid_block.resnets.0", x, H, W, C, C, [other])
            self._attention(ws, "encoder.mid_block.attentions.0", x, H, W, C)
            x, _ = self._resnet(ws, "encoder.mid_block.resnets.1", x, H, W, C, C, [other])
            t = self._view(ws["t"], H * W, C)
            ops.vae_rms_norm(x, wt["encoder.norm_out.gamma"], True, out=t)
            zo = ws["zo"]
            ops.conv2d(t, H, W, wt["encoder.conv_out.weight"], wt["encoder.conv_out.bias"], out=zo)
            zq = ws["zq"]
            ops.conv2d(zo, H, W, wt["quant_conv.weight"], wt["quant_conv.bias"], ksize=1, out=zq)
            outs.append(ops.vae_latents_out(zq, 1, H, W, wt["mean"], wt["std"]))
        return torch.cat(outs)

    def flops(self, H: int, W: int) -> float:
        """Algorithmic FLOPs of one encode of an H x W image."""
        c = self.config

        def conv(ci, co, k, P):
            return 2.0 * P * ci * co * k * k

        P = H * W
        f = conv(3, c.base_dim, 3, P)
        top = c.base_dim
        for op in encoder_plan(c):
            if op[0] == "res":
                a, b = op[2], op[3]
                f += conv(a, b, 3, P) + conv(b, b, 3, P) + (conv(a, b, 1, P) if a != b else 0.0)
                top = b
            else:
                P //= 4
                f += conv(op[2], op[2], 3, P)
        f += 2 * (2 * conv(top, top, 3, P)) + conv(top, 3 * top, 1, P) + 4.0 * P * P * top + conv(top, top, 1, P)
        z2 = 2 * c.z_dim
        return f + conv(top, z2, 3, P) + conv(z2, z2, 1, P)
