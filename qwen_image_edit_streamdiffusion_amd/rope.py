"""Host-side RoPE tables (QwenEmbedRope, theta=10000, axes (16,56,56), scale_rope=True) [U].

Built once per (img_shapes, txt_len) on the host in fp32 exactly as diffusers
builds its ``pos_freqs``/``neg_freqs`` (outer(index, theta^(-2j/d)) then
polar -> cos/sin), uploaded to HBM and consumed by ``qie_qk_norm_rope_bf16``.
The reference invokes it through every pipeline call
(server.py:137-153) with ``img_shapes=[[(1,64,64),(1,64,64)]]`` at 1024^2.
"""
from __future__ import annotations

from typing import Sequence, Tuple

import torch


def _axis_angles(index: torch.Tensor, dim: int, theta: float) -> torch.Tensor:
    inv = 1.0 / torch.pow(torch.tensor(theta, dtype=torch.float32),
                          torch.arange(0, dim, 2).to(torch.float32).div(dim))
    return torch.outer(index.to(torch.float32), inv)


def rope_angles(img_shapes: Sequence[Tuple[int, int, int]], txt_len: int,
                axes: Sequence[int] = (16, 56, 56), theta: float = 10000.0):
    """(img [S_img, Dh/2], txt [txt_len, Dh/2]) fp32 rotation angles."""
    parts = []
    max_vid = 0
    for idx, (f, h, w) in enumerate(img_shapes):
        fa = _axis_angles(torch.arange(idx, idx + f), axes[0], theta).view(f, 1, 1, -1).expand(f, h, w, -1)
        hi = torch.cat([torch.arange(-(h - h // 2), 0), torch.arange(0, h // 2)])
        wi = torch.cat([torch.arange(-(w - w // 2), 0), torch.arange(0, w // 2)])
        ha = _axis_angles(hi, axes[1], theta).view(1, h, 1, -1).expand(f, h, w, -1)
        wa = _axis_angles(wi, axes[2], theta).view(1, 1, w, -1).expand(f, h, w, -1)
        parts.append(torch.cat([fa, ha, wa], dim=-1).reshape(f * h * w, -1))
        max_vid = max(max_vid, h // 2, w // 2)
    pos = torch.arange(max_vid, max_vid + txt_len)
    txt = torch.cat([_axis_angles(pos, a, theta) for a in axes], dim=-1)
    return torch.cat(parts, dim=0), txt


def rope_tables(img_shapes, txt_len: int, device, axes=(16, 56, 56), theta: float = 10000.0):
    """Device fp32 (img_cos, img_sin, txt_cos, txt_sin), each [rows, Dh/2]."""
    ia, ta = rope_angles(img_shapes, txt_len, axes, theta)
    out = []
    for a in (ia, ta):
        out += [torch.cos(a).contiguous().to(device), torch.sin(a).contiguous().to(device)]
    return tuple(out)
