"""CPU restatement of the Qwen-Image-Edit-2509 DiT forward + denoise loop.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): the checker for the HIP
path, never the product.  PARITY UNPINNED against diffusers (absent here).

What is restated, and where the reference invokes it:

* ``QwenImageTransformer2DModel.forward`` [U: diffusers
  models/transformers/transformer_qwenimage.py], reached through
  ``QwenImageEditPlusPipeline.__call__`` at server.py:137-153,
  qwen_realtime.py:247-255, benchmark_lightning.py:41-49, and swapped as a
  module at benchmark_compile.py:102-106.
* ``FlowMatchEulerDiscreteScheduler.set_timesteps/step`` + ``calculate_shift``
  [U].
* the true-CFG combine + norm rescale of the Edit-Plus pipeline [U],
  switched on by ``true_cfg_scale=4.0, negative_prompt=" "``
  at benchmark_lightning.py:28-29.
* ``_pack_latents`` / ``_unpack_latents`` [U].

Numerics: the reference runs the model in bf16 (``torch_dtype=torch.bfloat16``,
server.py:66-69).  With ``emulate_bf16=True`` every tensor that diffusers stores
in bf16 is rounded to bf16 at the same point (module outputs, the bf16
elementwise ops of ``_modulate`` / gated residuals / CFG), while reductions run
in fp32 -- i.e. cuBLAS/SDPA semantics.  With ``emulate_bf16=False`` everything
is plain fp32 (the "math" reference).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch

BF16 = torch.bfloat16


# ----------------------------------------------------------------------------
# configuration
# ----------------------------------------------------------------------------
@dataclass
class DiTConfig:
    """Mirror of ``QwenImageTransformer2DModel.config``."""

    patch_size: int = 2
    in_channels: int = 64
    out_channels: int = 16
    num_layers: int = 60
    attention_head_dim: int = 128
    num_attention_heads: int = 24
    joint_attention_dim: int = 3584
    guidance_embeds: bool = False
    axes_dims_rope: Tuple[int, int, int] = (16, 56, 56)
    timestep_dim: int = 256      # Timesteps(num_channels=256)
    mlp_ratio: int = 4           # FeedForward inner_dim = 4*dim
    eps: float = 1e-6

    @property
    def inner_dim(self) -> int:
        return self.num_attention_heads * self.attention_head_dim


def tiny_config(**kw) -> DiTConfig:
    """Small config for fast CPU/GPU parity cases."""
    base = dict(num_layers=2, num_attention_heads=2, joint_attention_dim=128)
    base.update(kw)
    return DiTConfig(**base)


# ----------------------------------------------------------------------------
# parameters (diffusers state_dict names)
# ----------------------------------------------------------------------------
def param_shapes(cfg: DiTConfig) -> List[Tuple[str, Tuple[int, ...]]]:
    """Ordered (name, shape) list using diffusers' state_dict names [U]."""
    D, Dh = cfg.inner_dim, cfg.attention_head_dim
    F = cfg.mlp_ratio * D
    out = [
        ("img_in.weight", (D, cfg.in_channels)), ("img_in.bias", (D,)),
        ("txt_norm.weight", (cfg.joint_attention_dim,)),
        ("txt_in.weight", (D, cfg.joint_attention_dim)), ("txt_in.bias", (D,)),
        ("time_text_embed.timestep_embedder.linear_1.weight", (D, cfg.timestep_dim)),
        ("time_text_embed.timestep_embedder.linear_1.bias", (D,)),
        ("time_text_embed.timestep_embedder.linear_2.weight", (D, D)),
        ("time_text_embed.timestep_embedder.linear_2.bias", (D,)),
    ]
    for i in range(cfg.num_layers):
        p = f"transformer_blocks.{i}."
        for s in ("img", "txt"):
            out += [(p + f"{s}_mod.1.weight", (6 * D, D)), (p + f"{s}_mod.1.bias", (6 * D,))]
        for n in ("to_q", "to_k", "to_v", "add_q_proj", "add_k_proj", "add_v_proj"):
            out += [(p + f"attn.{n}.weight", (D, D)), (p + f"attn.{n}.bias", (D,))]
        for n in ("norm_q", "norm_k", "norm_added_q", "norm_added_k"):
            out += [(p + f"attn.{n}.weight", (Dh,))]
        out += [(p + "attn.to_out.0.weight", (D, D)), (p + "attn.to_out.0.bias", (D,)),
                (p + "attn.to_add_out.weight", (D, D)), (p + "attn.to_add_out.bias", (D,))]
        for s in ("img", "txt"):
            out += [(p + f"{s}_mlp.net.0.proj.weight", (F, D)), (p + f"{s}_mlp.net.0.proj.bias", (F,)),
                    (p + f"{s}_mlp.net.2.weight", (D, F)), (p + f"{s}_mlp.net.2.bias", (D,))]
    out += [("norm_out.linear.weight", (2 * D, D)), ("norm_out.linear.bias", (2 * D,)),
            ("proj_out.weight", (cfg.patch_size ** 2 * cfg.out_channels, D)),
            ("proj_out.bias", (cfg.patch_size ** 2 * cfg.out_channels,))]
    return out


def random_params(cfg: DiTConfig, seed: int = 0, std: float = 0.02) -> Dict[str, torch.Tensor]:
    """Seeded random init: Linear weights/biases N(0, std),
    RMSNorm weights 1 + N(0, std); drawn in parameter order from one CPU
    generator, then rounded to bf16 (the model's storage dtype)."""
    g = torch.Generator().manual_seed(seed)
    params = {}
    for name, shape in param_shapes(cfg):
        t = torch.randn(shape, generator=g, dtype=torch.float32) * std
        if name == "txt_norm.weight" or ".attn.norm_" in name:
            t = t + 1.0
        params[name] = t.to(BF16)
    return params


# ----------------------------------------------------------------------------
# primitives
# ----------------------------------------------------------------------------
class _R:
    """Rounding helper: r(x) rounds to bf16 (kept as fp32) when emulating."""

    def __init__(self, emulate_bf16: bool):
        self.on = emulate_bf16

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        return x.to(BF16).float() if self.on else x


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], r: _R) -> torch.Tensor:
    """nn.Linear in bf16: fp32 accumulate, one rounding of (acc + bias)."""
    y = x.float() @ w.float().t()
    if b is not None:
        y = y + b.float()
    return r(y)


def silu(x: torch.Tensor, r: _R) -> torch.Tensor:
    return r(torch.nn.functional.silu(x.float()))


def gelu_tanh(x: torch.Tensor, r: _R) -> torch.Tensor:
    return r(torch.nn.functional.gelu(x.float(), approximate="tanh"))


def layer_norm(x: torch.Tensor, eps: float, r: _R) -> torch.Tensor:
    """nn.LayerNorm(elementwise_affine=False): fp32 statistics, bf16 output."""
    x = x.float()
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return r((x - mu) * torch.rsqrt(var + eps))


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, r: _R) -> torch.Tensor:
    """diffusers RMSNorm(elementwise_affine=True) [U]: variance in fp32,
    ``(x * rsqrt(var+eps)).to(bf16) * weight`` -> two bf16 roundings."""
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    y = r(xf * torch.rsqrt(var + eps))
    return r(y * w.float())


def modulate(x: torch.Tensor, shift: torch.Tensor, scale: torch.Tensor, r: _R) -> torch.Tensor:
    """``x * (1 + scale) + shift`` evaluated in bf16 tensors [U] (_modulate)."""
    one_p = r(1.0 + scale.float())
    return r(r(x * one_p[:, None, :]) + shift.float()[:, None, :])


def gated_residual(x: torch.Tensor, gate: torch.Tensor, y: torch.Tensor, r: _R) -> torch.Tensor:
    """``x + gate * y`` in bf16 tensors (two roundings)."""
    return r(x + r(gate.float()[:, None, :] * y))


# ----------------------------------------------------------------------------
# timestep embedding (Timesteps(256, flip_sin_to_cos=True, shift=0, scale=1000))
# ----------------------------------------------------------------------------
def timestep_sinusoid(t: torch.Tensor, dim: int = 256, max_period: float = 10000.0,
                      scale: float = 1000.0) -> torch.Tensor:
    """get_timestep_embedding [U] -> fp32 [B, dim] = [cos | sin]."""
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(0, half, dtype=torch.float32) / half
    emb = torch.exp(exponent)
    emb = t.float()[:, None] * emb[None, :]
    emb = scale * emb
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    return torch.cat([emb[:, half:], emb[:, :half]], dim=-1)


def time_embed(params, t_scaled: torch.Tensor, cfg: DiTConfig, r: _R) -> torch.Tensor:
    """QwenTimestepProjEmbeddings [U]: Linear(SiLU(Linear(sinus(t))))."""
    p = "time_text_embed.timestep_embedder."
    proj = r(timestep_sinusoid(t_scaled, cfg.timestep_dim))
    h = linear(proj, params[p + "linear_1.weight"], params[p + "linear_1.bias"], r)
    h = silu(h, r)
    return linear(h, params[p + "linear_2.weight"], params[p + "linear_2.bias"], r)


# ----------------------------------------------------------------------------
# RoPE (QwenEmbedRope, theta=10000, axes (16,56,56), scale_rope=True) [U]
# ----------------------------------------------------------------------------
def _rope_axis_phase(index: torch.Tensor, dim: int, theta: float = 10000.0) -> torch.Tensor:
    inv = 1.0 / torch.pow(torch.tensor(theta, dtype=torch.float32),
                          torch.arange(0, dim, 2).to(torch.float32).div(dim))
    return torch.outer(index.to(torch.float32), inv)


def rope_phases(img_shapes: Sequence[Tuple[int, int, int]], txt_len: int,
                axes: Sequence[int] = (16, 56, 56), theta: float = 10000.0):
    """Return (img_phase [S_img, Dh/2], txt_phase [txt_len, Dh/2]) fp32 angles.

    Image i (frame index i) uses frame-axis position i and h/w positions
    centred as [-(h - h//2) .. -1] ++ [0 .. h//2 - 1]; text token n uses
    position max_i(max(h_i//2, w_i//2)) + n on all three axes.
    """
    imgs = []
    max_vid = 0
    for idx, (f, h, w) in enumerate(img_shapes):
        fr = _rope_axis_phase(torch.arange(idx, idx + f), axes[0], theta)
        hi = torch.cat([torch.arange(-(h - h // 2), 0), torch.arange(0, h // 2)])
        wi = torch.cat([torch.arange(-(w - w // 2), 0), torch.arange(0, w // 2)])
        ph = _rope_axis_phase(hi, axes[1], theta)
        pw = _rope_axis_phase(wi, axes[2], theta)
        fr = fr.view(f, 1, 1, -1).expand(f, h, w, -1)
        ph = ph.view(1, h, 1, -1).expand(f, h, w, -1)
        pw = pw.view(1, 1, w, -1).expand(f, h, w, -1)
        imgs.append(torch.cat([fr, ph, pw], dim=-1).reshape(f * h * w, -1))
        max_vid = max(h // 2, w // 2, max_vid)
    tpos = torch.arange(max_vid, max_vid + txt_len)
    txt = torch.cat([_rope_axis_phase(tpos, a, theta) for a in axes], dim=-1)
    return torch.cat(imgs, dim=0), txt


def apply_rope(x: torch.Tensor, phase: torch.Tensor, r: _R) -> torch.Tensor:
    """apply_rotary_emb_qwen(use_real=False) [U]: pairs (x[2j], x[2j+1]) as a
    complex number times e^{i*phase_j}, in fp32; x: [B, S, H, Dh]."""
    xf = x.float().reshape(*x.shape[:-1], -1, 2)
    c = torch.cos(phase)[None, :, None, :]
    s = torch.sin(phase)[None, :, None, :]
    re = xf[..., 0] * c - xf[..., 1] * s
    im = xf[..., 0] * s + xf[..., 1] * c
    return r(torch.stack([re, im], dim=-1).flatten(-2))


# ----------------------------------------------------------------------------
# attention
# ----------------------------------------------------------------------------
def joint_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor,
                    kv_valid: Optional[torch.Tensor], r: _R) -> torch.Tensor:
    """SDPA(non-causal, scale 1/sqrt(Dh)) on [B, S, H, Dh]; kv_valid [B, S]
    bool masks padded keys (batched CFG with unequal text lengths)."""
    qh, kh, vh = (t.float().transpose(1, 2) for t in (q, k, v))  # [B,H,S,Dh]
    B, H, S, Dh = qh.shape
    o = torch.empty(B, H, S, Dh, dtype=torch.float32)
    for b in range(B):          # one (b, h) score matrix at a time: bounded memory
        for h in range(H):
            s = qh[b, h] @ kh[b, h].transpose(-1, -2) / math.sqrt(Dh)
            if kv_valid is not None:
                s = s.masked_fill(~kv_valid[b][None, :], float("-inf"))
            o[b, h] = torch.softmax(s, dim=-1) @ vh[b, h]
    return r(o.transpose(1, 2).flatten(2))


# ----------------------------------------------------------------------------
# block / model
# ----------------------------------------------------------------------------
def block_forward(params, i: int, img: torch.Tensor, txt: torch.Tensor, temb: torch.Tensor,
                  img_phase: torch.Tensor, txt_phase: torch.Tensor, cfg: DiTConfig, r: _R,
                  txt_valid: Optional[torch.Tensor] = None):
    """QwenImageTransformerBlock.forward [U]."""
    p = f"transformer_blocks.{i}."
    D, H, Dh, eps = cfg.inner_dim, cfg.num_attention_heads, cfg.attention_head_dim, cfg.eps
    B, S_img, S_txt = img.shape[0], img.shape[1], txt.shape[1]
    st = silu(temb, r)
    img_mod = linear(st, params[p + "img_mod.1.weight"], params[p + "img_mod.1.bias"], r)
    txt_mod = linear(st, params[p + "txt_mod.1.weight"], params[p + "txt_mod.1.bias"], r)
    ish1, isc1, ig1, ish2, isc2, ig2 = img_mod.chunk(6, dim=-1)
    tsh1, tsc1, tg1, tsh2, tsc2, tg2 = txt_mod.chunk(6, dim=-1)

    img_m = modulate(layer_norm(img, eps, r), ish1, isc1, r)
    txt_m = modulate(layer_norm(txt, eps, r), tsh1, tsc1, r)

    def proj(x, n):
        return linear(x, params[p + f"attn.{n}.weight"], params[p + f"attn.{n}.bias"], r)

    iq, ik, iv = (proj(img_m, n).view(B, S_img, H, Dh) for n in ("to_q", "to_k", "to_v"))
    tq, tk, tv = (proj(txt_m, n).view(B, S_txt, H, Dh) for n in ("add_q_proj", "add_k_proj", "add_v_proj"))
    iq = rms_norm(iq, params[p + "attn.norm_q.weight"], eps, r)
    ik = rms_norm(ik, params[p + "attn.norm_k.weight"], eps, r)
    tq = rms_norm(tq, params[p + "attn.norm_added_q.weight"], eps, r)
    tk = rms_norm(tk, params[p + "attn.norm_added_k.weight"], eps, r)
    iq, ik = apply_rope(iq, img_phase, r), apply_rope(ik, img_phase, r)
    tq, tk = apply_rope(tq, txt_phase, r), apply_rope(tk, txt_phase, r)

    jq, jk, jv = torch.cat([tq, iq], 1), torch.cat([tk, ik], 1), torch.cat([tv, iv], 1)
    kv_valid = None
    if txt_valid is not None:
        kv_valid = torch.cat([txt_valid, torch.ones(B, S_img, dtype=torch.bool)], dim=1)
    o = joint_attention(jq, jk, jv, kv_valid, r)
    t_att, i_att = o[:, :S_txt], o[:, S_txt:]
    i_att = linear(i_att, params[p + "attn.to_out.0.weight"], params[p + "attn.to_out.0.bias"], r)
    t_att = linear(t_att, params[p + "attn.to_add_out.weight"], params[p + "attn.to_add_out.bias"], r)
    img = gated_residual(img, ig1, i_att, r)
    txt = gated_residual(txt, tg1, t_att, r)

    def mlp(x, s):
        h = linear(x, params[p + f"{s}_mlp.net.0.proj.weight"], params[p + f"{s}_mlp.net.0.proj.bias"], r)
        h = gelu_tanh(h, r)
        return linear(h, params[p + f"{s}_mlp.net.2.weight"], params[p + f"{s}_mlp.net.2.bias"], r)

    img = gated_residual(img, ig2, mlp(modulate(layer_norm(img, eps, r), ish2, isc2, r), "img"), r)
    txt = gated_residual(txt, tg2, mlp(modulate(layer_norm(txt, eps, r), tsh2, tsc2, r), "txt"), r)
    return img, txt


def transformer_forward(params, cfg: DiTConfig, hidden_states: torch.Tensor,
                        encoder_hidden_states: torch.Tensor, timestep: torch.Tensor,
                        img_shapes: Sequence[Tuple[int, int, int]], txt_seq_lens: Sequence[int],
                        emulate_bf16: bool = True, num_layers: Optional[int] = None) -> torch.Tensor:
    """QwenImageTransformer2DModel.forward [U] -> sample [B, S_img, 64] (fp32
    tensor holding bf16 values when emulating).

    ``timestep`` is what the pipeline passes: bf16(t)/1000 in bf16.
    ``txt_seq_lens`` gives each row's valid text length; rows shorter than
    ``encoder_hidden_states.shape[1]`` are key-masked (batched CFG)."""
    r = _R(emulate_bf16)
    B, S_txt = encoder_hidden_states.shape[:2]
    img = linear(hidden_states.float(), params["img_in.weight"], params["img_in.bias"], r)
    t = r(timestep.float())
    txt = rms_norm(encoder_hidden_states, params["txt_norm.weight"], cfg.eps, r)
    txt = linear(txt, params["txt_in.weight"], params["txt_in.bias"], r)
    temb = time_embed(params, t, cfg, r)
    img_phase, txt_phase = rope_phases(img_shapes, S_txt, cfg.axes_dims_rope)
    txt_valid = None
    if any(int(l) != S_txt for l in txt_seq_lens):
        txt_valid = torch.arange(S_txt)[None, :] < torch.tensor([int(l) for l in txt_seq_lens])[:, None]
    L = cfg.num_layers if num_layers is None else num_layers
    for i in range(L):
        img, txt = block_forward(params, i, img, txt, temb, img_phase, txt_phase, cfg, r, txt_valid)
    emb = linear(silu(temb, r), params["norm_out.linear.weight"], params["norm_out.linear.bias"], r)
    scale, shift = emb.chunk(2, dim=-1)
    x = layer_norm(img, cfg.eps, r)
    x = r(r(x * r(1.0 + scale)[:, None, :]) + shift[:, None, :])
    return linear(x, params["proj_out.weight"], params["proj_out.bias"], r)


# ----------------------------------------------------------------------------
# scheduler (FlowMatchEulerDiscreteScheduler, Qwen-Image config) [U]
# ----------------------------------------------------------------------------
@dataclass
class SchedulerConfig:
    num_train_timesteps: int = 1000
    base_image_seq_len: int = 256
    max_image_seq_len: int = 8192
    base_shift: float = 0.5
    max_shift: float = 0.9
    shift_terminal: Optional[float] = 0.02
    use_dynamic_shifting: bool = True


def calculate_shift(image_seq_len: int, c: SchedulerConfig) -> float:
    m = (c.max_shift - c.base_shift) / (c.max_image_seq_len - c.base_image_seq_len)
    b = c.base_shift - m * c.base_image_seq_len
    return image_seq_len * m + b


def sigma_schedule(num_steps: int, image_seq_len: int, c: SchedulerConfig = SchedulerConfig()):
    """set_timesteps(sigmas=linspace(1, 1/N, N), mu=calculate_shift(seq)):
    exponential time shift, stretch to shift_terminal, append 0.
    Returns (sigmas fp32 [N+1], timesteps fp32 [N] = 1000*sigma)."""
    import numpy as np
    sig = np.linspace(1.0, 1.0 / num_steps, num_steps).astype(np.float32)
    mu = calculate_shift(image_seq_len, c)
    sig = (math.exp(mu) / (math.exp(mu) + (1.0 / sig - 1.0) ** 1.0)).astype(np.float32) \
        if c.use_dynamic_shifting else sig
    if c.shift_terminal:
        one_minus = 1.0 - sig
        scale = one_minus[-1] / (1.0 - c.shift_terminal)
        sig = (1.0 - one_minus / scale).astype(np.float32)
    s = torch.from_numpy(np.asarray(sig)).to(torch.float32)
    return torch.cat([s, torch.zeros(1)]), s * c.num_train_timesteps


def model_timestep(t: torch.Tensor) -> torch.Tensor:
    """Pipeline: ``timestep = t.expand(B).to(latents.dtype)`` then ``/1000``,
    both in bf16 [U]."""
    return (t.to(BF16) / 1000).to(BF16)


def euler_step(sample: torch.Tensor, v: torch.Tensor, sigma: float, sigma_next: float) -> torch.Tensor:
    """FlowMatchEulerDiscreteScheduler.step [U]: ``sample.float() + (s1 - s0) * v``
    where the 0-d fp32 factor times the bf16 ``v`` yields a bf16 product; the
    sum is fp32, cast back to bf16.  Returns bf16."""
    dt = torch.tensor(sigma_next, dtype=torch.float32) - torch.tensor(sigma, dtype=torch.float32)
    prod = (dt * v.to(BF16).float()).to(BF16).float()
    return (sample.to(BF16).float() + prod).to(BF16)


def cfg_combine(cond: torch.Tensor, uncond: torch.Tensor, scale: float) -> torch.Tensor:
    """True-CFG + norm rescale of the Edit-Plus pipeline [U], bf16 tensors:
    comb = u + s*(c-u); out = comb * (||c|| / ||comb||) over the last dim."""
    r = _R(True)
    c, u = cond.to(BF16).float(), uncond.to(BF16).float()
    comb = r(u + r(scale * r(c - u)))
    cn = r(torch.linalg.vector_norm(c, dim=-1, keepdim=True))
    nn_ = r(torch.linalg.vector_norm(comb, dim=-1, keepdim=True))
    return r(comb * r(cn / nn_)).to(BF16)


# ----------------------------------------------------------------------------
# latent packing [U] (_pack_latents / _unpack_latents)
# ----------------------------------------------------------------------------
def pack_latents(x: torch.Tensor) -> torch.Tensor:
    """[B, 1, C, H, W] / [B, C, 1, H, W] / [B, C, H, W] -> [B, (H/2)(W/2), C*4]
    (diffusers views the 5-D tensor as [B, C, H/2, 2, W/2, 2] by memory order)."""
    if x.dim() == 5:
        x = x.reshape(x.shape[0], x.shape[1] * x.shape[2], x.shape[3], x.shape[4])
    B, C, H, W = x.shape
    x = x.view(B, C, H // 2, 2, W // 2, 2).permute(0, 2, 4, 1, 3, 5)
    return x.reshape(B, (H // 2) * (W // 2), C * 4)


def unpack_latents(x: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """[B, (H/2)(W/2), C*4] -> [B, C, 1, H, W] (H, W in latent pixels)."""
    B, N, C4 = x.shape
    C = C4 // 4
    x = x.view(B, H // 2, W // 2, C, 2, 2).permute(0, 3, 1, 4, 2, 5)
    return x.reshape(B, C, 1, H, W)


# ----------------------------------------------------------------------------
# full denoise (sequential true-CFG, the reference's own loop) [U]
# ----------------------------------------------------------------------------
def denoise(params, cfg: DiTConfig, latents: torch.Tensor, cond_latents: torch.Tensor,
            prompt_embeds: torch.Tensor, img_shapes, num_steps: int,
            neg_embeds: Optional[torch.Tensor] = None, true_cfg_scale: float = 4.0,
            emulate_bf16: bool = True, num_layers: Optional[int] = None) -> torch.Tensor:
    """Edit-Plus denoise loop on packed latents [B, S_noise, 64] (bf16)."""
    sig, ts = sigma_schedule(num_steps, latents.shape[1])
    x = latents.to(BF16)
    for i in range(num_steps):
        t = model_timestep(ts[i].expand(x.shape[0]))
        inp = torch.cat([x, cond_latents.to(BF16)], dim=1)
        out = transformer_forward(params, cfg, inp, prompt_embeds, t, img_shapes,
                                  [prompt_embeds.shape[1]] * x.shape[0], emulate_bf16, num_layers)
        v = out[:, : x.shape[1]].to(BF16)
        if neg_embeds is not None and true_cfg_scale > 1.0:
            outn = transformer_forward(params, cfg, inp, neg_embeds, t, img_shapes,
                                       [neg_embeds.shape[1]] * x.shape[0], emulate_bf16, num_layers)
            v = cfg_combine(v, outn[:, : x.shape[1]].to(BF16), true_cfg_scale)
        x = euler_step(x, v, float(sig[i]), float(sig[i + 1]))
    return x


def flops_per_forward(S_img: int, S_txt: int, cfg: DiTConfig = DiTConfig(), layers: Optional[int] = None) -> float:
    """Algorithmic FLOPs of one B=1 forward."""
    D, L = cfg.inner_dim, (cfg.num_layers if layers is None else layers)
    S = S_img + S_txt
    return (L * (24 * S * D * D + 4 * S * S * D + 24 * D * D) + 2 * S_img * 64 * D
            + 2 * S_txt * cfg.joint_attention_dim * D + 2 * (256 * D + D * D) + 4 * D * D
            + 2 * S_img * D * 64)
