"""The prompt encoder's vision tower on the HIP path.

The reference feeds each condition image (resized to a 384^2 area) through
Qwen2.5-VL's vision transformer [U: transformers 5.15 models/qwen2_5_vl/modeling_qwen2_5_vl.py,
Qwen2_5_VisionTransformerPretrainedModel; window / position helpers in transformers/vision_utils.py]:
a 2x14x14 patch embedding (Conv3d with kernel == stride, i.e. one linear over 1176 inputs), the
patches permuted so that each 112-pixel window is contiguous, 32 blocks (RMSNorm, q|k|v with bias,
2-D rotate-half RoPE in fp32, window attention -- full attention per image on blocks 7/15/23/31 --,
proj + residual, RMSNorm, SwiGLU MLP with bias + residual), then the 2x2 patch merger (RMSNorm,
Linear 5120 -> 5120, GELU, Linear -> 3584) and the inverse window permutation. The output rows
replace the ``<|image_pad|>`` tokens of the prompt (text_encoder.QwenVLEncoder).

MI355X mapping: every linear is one GEMM; the 80-wide heads sit in 128-wide zero-padded slots
(the fp32 score GEMM needs K % 64; zeros leave q.k and P.V unchanged) and the SwiGLU width 3420 is
zero-padded to 3456, both once at load time. Attention runs all heads per launch: head-batched fp32
score GEMM over all rows, one softmax that keeps each row's window (or image) range, head-batched
P.V against V^T. The
window permutation and its inverse are row gathers (the embedding kernel).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import torch

from . import ops

BF16 = torch.bfloat16


def _ru(x: int, m: int) -> int:
    return -(-x // m) * m


@dataclass
class VisionConfig:
    """Qwen2_5_VLVisionConfig fields the forward uses (defaults: Qwen2.5-VL-7B's vision_config)."""

    depth: int = 32
    hidden_size: int = 1280
    intermediate_size: int = 3420
    num_heads: int = 16
    in_channels: int = 3
    patch_size: int = 14
    temporal_patch_size: int = 2
    spatial_merge_size: int = 2
    window_size: int = 112
    out_hidden_size: int = 3584
    fullatt_block_indexes: Tuple[int, ...] = (7, 15, 23, 31)
    rms_norm_eps: float = 1e-6

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_heads

    @property
    def patch_dim(self) -> int:
        return self.in_channels * self.temporal_patch_size * self.patch_size ** 2


def vision_state_dict_shapes(c: VisionConfig) -> Dict[str, Tuple[int, ...]]:
    """Qwen2_5_VisionTransformerPretrainedModel parameter names (tower relative) and shapes."""
    D, F, m = c.hidden_size, c.intermediate_size, c.spatial_merge_size ** 2
    out = {"patch_embed.proj.weight": (D, c.in_channels, c.temporal_patch_size, c.patch_size, c.patch_size),
           "merger.ln_q.weight": (D,), "merger.mlp.0.weight": (m * D, m * D), "merger.mlp.0.bias": (m * D,),
           "merger.mlp.2.weight": (c.out_hidden_size, m * D), "merger.mlp.2.bias": (c.out_hidden_size,)}
    for i in range(c.depth):
        p = f"blocks.{i}."
        out.update({p + "norm1.weight": (D,), p + "norm2.weight": (D,), p + "attn.qkv.weight": (3 * D, D),
                    p + "attn.qkv.bias": (3 * D,), p + "attn.proj.weight": (D, D), p + "attn.proj.bias": (D,),
                    p + "mlp.gate_proj.weight": (F, D), p + "mlp.gate_proj.bias": (F,),
                    p + "mlp.up_proj.weight": (F, D), p + "mlp.up_proj.bias": (F,),
                    p + "mlp.down_proj.weight": (D, F), p + "mlp.down_proj.bias": (D,)})
    return out


# ---------------------------------------------------------------------------- host index logic
def vision_position_ids(grid_thw: Sequence[Sequence[int]], merge: int) -> torch.Tensor:
    """(h, w) patch coordinates [S, 2], block-major over merge x merge blocks, repeated per frame
    (vision_utils.get_vision_position_ids, include_temporal=False)."""
    out = []
    for t, h, w in grid_thw:
        hh = torch.arange(h).view(h // merge, merge, 1, 1).expand(h // merge, merge, w // merge, merge)
        ww = torch.arange(w).view(1, 1, w // merge, merge).expand(h // merge, merge, w // merge, merge)
        hh = hh.permute(0, 2, 1, 3).reshape(-1)
        ww = ww.permute(0, 2, 1, 3).reshape(-1)
        out.append(torch.stack([hh, ww], -1).repeat(t, 1))
    return torch.cat(out)


def window_index(grid_thw: Sequence[Sequence[int]], merge: int, window_size: int, patch_size: int
                 ) -> Tuple[torch.Tensor, List[int]]:
    """(merged-unit permutation making every window contiguous, cumulative window lengths in
    patches with empty windows dropped) -- vision_utils.get_vision_window_index. Windows are
    window_size / merge / patch_size merged units on a side; the edge windows are ragged."""
    vw = window_size // merge // patch_size
    unit = merge * merge
    index, cu, base = [], [0], 0
    for t, h, w in grid_thw:
        lh, lw = h // merge, w // merge
        nh, nw = lh // vw + 1, lw // vw + 1  # the reference pads by vw - (l % vw): one extra window if exact
        for tt in range(t):
            for wy in range(nh):
                for wx in range(nw):
                    ys = range(wy * vw, min((wy + 1) * vw, lh))
                    xs = range(wx * vw, min((wx + 1) * vw, lw))
                    ids = [base + (tt * lh + y) * lw + x for y in ys for x in xs]
                    if ids:
                        index.extend(ids)
                        cu.append(cu[-1] + len(ids) * unit)
        base += t * lh * lw
    return torch.tensor(index, dtype=torch.long), cu


def frame_seqlens(grid_thw: Sequence[Sequence[int]]) -> List[int]:
    """Cumulative per-frame lengths (full-attention blocks): vision_utils.get_vision_cu_seqlens."""
    cu = [0]
    for t, h, w in grid_thw:
        for _ in range(t):
            cu.append(cu[-1] + h * w)
    return cu


def _row_ranges(cu: List[int], S: int, Sp: int) -> torch.Tensor:
    """[Sp, 2] int32 key ranges: row r of segment [a, b) keeps keys [a, b); padding rows keep themselves."""
    r = torch.empty(Sp, 2, dtype=torch.int32)
    for a, b in zip(cu[:-1], cu[1:]):
        r[a:b, 0], r[a:b, 1] = a, b
    pad = torch.arange(S, Sp, dtype=torch.int32)
    r[S:, 0], r[S:, 1] = pad, pad + 1
    return r


def rotary_tables(cfg: VisionConfig, grid_thw, perm_units: torch.Tensor, rows: int
                  ) -> Tuple[torch.Tensor, torch.Tensor]:
    """fp32 cos / sin [rows, head_dim] in window order: Qwen2_5_VisionRotaryEmbedding(head_dim/2)
    on the (h, w) positions, emb = cat(freqs, freqs)."""
    dim = cfg.head_dim // 2
    inv = 1.0 / (10000.0 ** (torch.arange(0, dim, 2, dtype=torch.float) / dim))
    pos = vision_position_ids(grid_thw, cfg.spatial_merge_size)
    rpe = (pos[:, :, None].float() * inv).flatten(1)                      # [S, dim]
    unit = cfg.spatial_merge_size ** 2
    rpe = rpe.view(-1, unit, dim)[perm_units].reshape(-1, dim)
    emb = torch.cat([rpe, rpe], -1)
    cos = torch.zeros(rows, cfg.head_dim)
    sin = torch.zeros(rows, cfg.head_dim)
    cos[:emb.shape[0]], sin[:emb.shape[0]] = emb.cos(), emb.sin()
    return cos, sin


# ---------------------------------------------------------------------------- the tower
class QwenVLVisionTower:
    """``Qwen2_5_VisionTransformerPretrainedModel`` forward (pooler output) on the HIP path."""

    SLOT = 128  # zero-padded head slot

    def __init__(self, config: VisionConfig = None, device="cuda"):
        self.config = config or VisionConfig()
        self.device = torch.device(device)
        c = self.config
        if c.hidden_size % 64 or c.out_hidden_size % 64 or c.head_dim > self.SLOT or c.head_dim % 2:
            raise NotImplementedError("hidden sizes must be multiples of 64 and head_dim <= 128")
        self.Fp = _ru(c.intermediate_size, 64)
        self.Kp = _ru(c.patch_dim, 64)
        self.blocks: List[Dict[str, torch.Tensor]] = []
        self.w: Dict[str, torch.Tensor] = {}
        from .text_encoder import EncoderLinears
        self.lin = EncoderLinears(self.device)

    @staticmethod
    def _strip(sd):
        for pre in ("model.visual.", "visual."):
            if any(k.startswith(pre) for k in sd):
                return {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)}
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> "QwenVLVisionTower":
        sd = self._strip(sd)
        c, dev, S = self.config, self.device, self.SLOT
        D, H, Dh, F = c.hidden_size, c.num_heads, c.head_dim, c.intermediate_size
        g = lambda k: sd[k].to(dev).to(BF16)  # noqa: E731
        z = lambda *s: torch.zeros(*s, dtype=BF16, device=dev)  # noqa: E731
        pw = g("patch_embed.proj.weight").reshape(D, -1)
        if pw.shape[1] != c.patch_dim:
            raise ValueError("patch_embed does not match the config")
        w_patch = z(D, self.Kp)
        w_patch[:, :c.patch_dim] = pw
        self.w = {"patch": w_patch, "zero_d": z(D), "zero_slot": z(S), "ones": torch.ones(1, D, dtype=BF16, device=dev),
                  "ln_q": g("merger.ln_q.weight").contiguous(),
                  "m0_w": g("merger.mlp.0.weight").contiguous(), "m0_b": g("merger.mlp.0.bias").contiguous(),
                  "m2_w": g("merger.mlp.2.weight").contiguous(), "m2_b": g("merger.mlp.2.bias").contiguous()}
        self.blocks = []
        for i in range(c.depth):
            p = f"blocks.{i}."
            qkv_w, qkv_b = g(p + "attn.qkv.weight"), g(p + "attn.qkv.bias")
            w_qkv, b_qkv = z(3 * H * S, D), z(3 * H * S)
            for j in range(3 * H):  # q heads, k heads, v heads, each in a 128-row slot
                w_qkv[j * S:j * S + Dh] = qkv_w[j * Dh:(j + 1) * Dh]
                b_qkv[j * S:j * S + Dh] = qkv_b[j * Dh:(j + 1) * Dh]
            pj = g(p + "attn.proj.weight")
            w_proj = z(D, H * S)
            for h in range(H):
                w_proj[:, h * S:h * S + Dh] = pj[:, h * Dh:(h + 1) * Dh]
            w_gu, b_gu = z(2 * self.Fp, D), z(2 * self.Fp)
            w_gu[:F], b_gu[:F] = g(p + "mlp.gate_proj.weight"), g(p + "mlp.gate_proj.bias")
            w_gu[self.Fp:self.Fp + F], b_gu[self.Fp:self.Fp + F] = g(p + "mlp.up_proj.weight"), g(p + "mlp.up_proj.bias")
            w_down = z(D, self.Fp)
            w_down[:, :F] = g(p + "mlp.down_proj.weight")
            self.blocks.append({"n1": g(p + "norm1.weight").contiguous(), "n2": g(p + "norm2.weight").contiguous(),
                                "w_qkv": w_qkv, "b_qkv": b_qkv, "w_proj": w_proj,
                                "b_proj": g(p + "attn.proj.bias").contiguous(),
                                "w_gu": w_gu, "b_gu": b_gu, "w_down": w_down,
                                "b_down": g(p + "mlp.down_proj.bias").contiguous()})
        return self

    def forward(self, pixel_values: torch.Tensor, grid_thw) -> torch.Tensor:
        """pixel_values [S, in_channels * temporal_patch * patch^2] (the processor's flattened
        patches), grid_thw [(t, h, w)] per image -> merged image embeddings [S / 4, out_hidden]
        bf16, image after image."""
        c, w, dev, SL = self.config, self.w, self.device, self.SLOT
        if not self.blocks:
            raise RuntimeError("vision tower weights not loaded")
        grid = [tuple(int(v) for v in g) for g in (grid_thw.tolist() if torch.is_tensor(grid_thw) else grid_thw)]
        m = c.spatial_merge_size
        unit = m * m
        S = sum(t * h * wd for t, h, wd in grid)
        if pixel_values.shape != (S, c.patch_dim):
            raise ValueError(f"pixel_values {tuple(pixel_values.shape)} != ({S}, {c.patch_dim}) for grid {grid}")
        if any(h % m or wd % m for _, h, wd in grid):
            raise ValueError("grid h / w must be multiples of spatial_merge_size")
        Sp = _ru(S, 64)
        D, H, Dh = c.hidden_size, c.num_heads, c.head_dim
        perm, cu_win = window_index(grid, m, c.window_size, c.patch_size)
        rows = (perm[:, None] * unit + torch.arange(unit)).reshape(-1)
        rows_dev = rows.to(torch.int32).to(dev)
        inv_dev = torch.argsort(perm).to(torch.int32).to(dev)
        cos, sin = (t.to(dev) for t in rotary_tables(c, grid, perm, Sp))
        rng_win = _row_ranges(cu_win, S, Sp).to(dev)
        rng_full = _row_ranges(frame_seqlens(grid), S, Sp).to(dev)

        xin = torch.zeros(Sp, self.Kp, dtype=BF16, device=dev)
        xin[:S, :c.patch_dim] = pixel_values.to(dev).to(BF16)
        x0 = ops.linear(xin, w["patch"], w["zero_d"])
        x = torch.zeros(Sp, D, dtype=BF16, device=dev)
        ops.embed_rows(x0, rows_dev, out=x[:S])  # window order
        h = torch.empty(Sp, D, dtype=BF16, device=dev)
        qkv = torch.empty(Sp, 3 * H * SL, dtype=BF16, device=dev)
        att = torch.empty(Sp, H * SL, dtype=BF16, device=dev)
        s = torch.empty(H * Sp, Sp, dtype=torch.float32, device=dev)  # all heads' scores
        p = torch.empty(H * Sp, Sp, dtype=BF16, device=dev)
        vt = torch.empty(H * SL, Sp, dtype=BF16, device=dev)
        gu = torch.empty(Sp, 2 * self.Fp, dtype=BF16, device=dev)
        a = torch.empty(Sp, self.Fp, dtype=BF16, device=dev)
        scale = Dh ** -0.5
        for i, B in enumerate(self.blocks):
            rng = rng_full if i in c.fullatt_block_indexes else rng_win
            ops.rmsnorm(x, B["n1"], out=h, eps=c.rms_norm_eps)
            self.lin.linear(h, B["w_qkv"], B["b_qkv"], qkv)
            ops.rope_half(qkv, 0, 2 * H, Dh, cos, sin, head_stride=SL)
            ops.transpose(qkv[:, 2 * H * SL:], out=vt)
            ops.matmul_heads(qkv[:, :SL], SL, qkv[:, H * SL:(H + 1) * SL], SL, s[:Sp], Sp * Sp, H)
            ops.softmax_rows(s, scale, out=p, ranges=rng)
            ops.matmul_heads(p[:Sp], Sp * Sp, vt[:SL], SL * Sp, att[:, :SL], SL, H, bias=w["zero_slot"])
            self.lin.residual(att, B["w_proj"], B["b_proj"], w["ones"], x)
            ops.rmsnorm(x, B["n2"], out=h, eps=c.rms_norm_eps)
            self.lin.linear(h, B["w_gu"], B["b_gu"], gu)
            ops.silu_mul(gu, out=a)
            self.lin.residual(a, B["w_down"], B["b_down"], w["ones"], x)
        ops.rmsnorm(x, w["ln_q"], out=h, eps=c.rms_norm_eps)
        hm = h.view(Sp // unit, unit * D)
        m1 = self.lin.linear(hm, w["m0_w"], w["m0_b"], torch.empty(Sp // unit, unit * D, dtype=BF16, device=dev))
        ops.gelu_erf_(m1)
        m2 = self.lin.linear(m1, w["m2_w"], w["m2_b"],
                             torch.empty(Sp // unit, c.out_hidden_size, dtype=BF16, device=dev))
        out = torch.empty(S // unit, c.out_hidden_size, dtype=BF16, device=dev)
        ops.embed_rows(m2, inv_dev, out=out)  # back to raster (merge-block) order
        return out

    __call__ = forward

    def flops(self, S: int) -> float:
        """Dense GEMM FLOPs of one forward over S patches (padded widths, as executed)."""
        c, SL = self.config, self.SLOT
        D, H = c.hidden_size, c.num_heads
        Sp = _ru(S, 64)
        per = 2 * Sp * D * (3 * H * SL + H * SL + 3 * self.Fp) + H * 2 * 2 * Sp * Sp * SL
        merge = 2 * (Sp // 4) * (4 * D) * (4 * D + c.out_hidden_size)
        return float(c.depth * per + merge + 2 * Sp * self.Kp * D)
