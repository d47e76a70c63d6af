"""The prompt encoder's language model on the HIP path (first half).

The reference encodes each prompt (and its condition image) with the pipeline's ``text_encoder``,
Qwen2.5-VL-7B [U: diffusers QwenImageEditPlusPipeline.encode_prompt -> transformers
Qwen2_5_VLForConditionalGeneration, hidden_states[-1]], invoked through server.py:137-153 and
qwen_realtime.py:140-165 (the prompt cache).  This module is its decoder-only language model
(``Qwen2_5_VLTextModel``): embed_tokens, N x (RMSNorm, q|k|v with bias, multimodal rotate-half
RoPE on 3-D positions, causal GQA attention, o_proj + residual, RMSNorm, SwiGLU MLP + residual),
final RMSNorm -- the hidden states the DiT consumes as ``encoder_hidden_states``.  The vision tower
that turns the condition image into the ``<|image_pad|>`` embeddings is the next half of f2;
``forward`` already takes those embeddings (``inputs_embeds`` rows) and their 3-D positions.

MI355X mapping: every projection is one GEMM (q|k|v packed, gate|up packed; o_proj and down_proj
carry the residual add in their epilogue), RMSNorm / RoPE / SwiGLU / embedding are HIP kernels,
attention is per query head: fp32 scores by GEMM, causal softmax, P.V by GEMM against V^T (prompt
lengths are a few hundred tokens; the GQA group shares its V^T).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

from . import ops

BF16 = torch.bfloat16


@dataclass
class TextEncoderConfig:
    """Qwen2_5_VLTextConfig fields the forward uses (defaults: Qwen2.5-VL-7B)."""

    vocab_size: int = 152064
    hidden_size: int = 3584
    intermediate_size: int = 18944
    num_hidden_layers: int = 28
    num_attention_heads: int = 28
    num_key_value_heads: int = 4
    rms_norm_eps: float = 1e-6
    rope_theta: float = 1000000.0
    mrope_section: Tuple[int, ...] = (16, 24, 24)

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads


def mrope_tables(cfg: TextEncoderConfig, position_ids: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """cos / sin [S, head_dim] for 3-D positions [3, S] (temporal, height, width), as
    Qwen2_5_VLRotaryEmbedding + apply_multimodal_rotary_pos_emb build them: fp32 freqs =
    pos * inv_freq, emb = cat(freqs, freqs), cos / sin in fp32, section i of the doubled
    mrope_section taken from axis i % 3, cast to bf16."""
    Dh = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, Dh, 2, dtype=torch.float) / Dh))
    pos = position_ids.to(torch.float32).cpu()                       # [3, S]
    freqs = pos[:, :, None] * inv[None, None, :]                     # [3, S, Dh/2]
    emb = torch.cat([freqs, freqs], dim=-1)                          # [3, S, Dh]
    cos, sin = emb.cos(), emb.sin()
    sec = list(cfg.mrope_section) * 2
    parts_c, parts_s, o = [], [], 0
    for i, n in enumerate(sec):
        parts_c.append(cos[i % 3, :, o:o + n])
        parts_s.append(sin[i % 3, :, o:o + n])
        o += n
    return torch.cat(parts_c, -1).to(BF16), torch.cat(parts_s, -1).to(BF16)


class QwenVLTextModel:
    """``Qwen2_5_VLTextModel`` forward on the HIP path (one prompt at a time: no padding mask)."""

    def __init__(self, config: Optional[TextEncoderConfig] = None, device="cuda"):
        self.config = config or TextEncoderConfig()
        self.device = torch.device(device)
        c = self.config
        if c.head_dim % 64 or c.hidden_size % 64 or c.intermediate_size % 64:
            raise NotImplementedError("head_dim, hidden_size and intermediate_size must be multiples of 64")
        if sum(c.mrope_section) * 2 != c.head_dim:
            raise ValueError("mrope_section must cover head_dim / 2")
        self.layers: List[Dict[str, torch.Tensor]] = []
        self.w: Dict[str, torch.Tensor] = {}

    # ------------------------------------------------------------------ weights
    @staticmethod
    def _strip(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """Accept the text model's own names and the checkpoint prefixes around it."""
        for pre in ("model.language_model.", "language_model.model.", "language_model.", "model."):
            if any(k.startswith(pre + "layers.") for k in sd):
                return {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)}
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> "QwenVLTextModel":
        sd = self._strip(sd)
        c, dev = self.config, self.device
        g = lambda k: sd[k].to(dev).to(BF16).contiguous()  # noqa: E731
        if tuple(sd["embed_tokens.weight"].shape) != (c.vocab_size, c.hidden_size):
            raise ValueError("embed_tokens shape does not match the config")
        self.w = {"embed": g("embed_tokens.weight"), "norm": g("norm.weight"),
                  "ones": torch.ones(1, c.hidden_size, dtype=BF16, device=dev),
                  "zero_d": torch.zeros(c.hidden_size, dtype=BF16, device=dev),
                  "zero_hd": torch.zeros(c.head_dim, dtype=BF16, device=dev),
                  "zero_2f": torch.zeros(2 * c.intermediate_size, dtype=BF16, device=dev)}
        self.layers = []
        for i in range(c.num_hidden_layers):
            p = f"layers.{i}."
            a = p + "self_attn."
            self.layers.append({
                "ln1": g(p + "input_layernorm.weight"), "ln2": g(p + "post_attention_layernorm.weight"),
                "w_qkv": torch.cat([g(a + "q_proj.weight"), g(a + "k_proj.weight"), g(a + "v_proj.weight")]).contiguous(),
                "b_qkv": torch.cat([g(a + "q_proj.bias"), g(a + "k_proj.bias"), g(a + "v_proj.bias")]).contiguous(),
                "w_o": g(a + "o_proj.weight"),
                "w_gu": torch.cat([g(p + "mlp.gate_proj.weight"), g(p + "mlp.up_proj.weight")]).contiguous(),
                "w_down": g(p + "mlp.down_proj.weight"),
            })
        return self

    # ------------------------------------------------------------------ forward
    def forward(self, input_ids: Optional[torch.Tensor] = None, position_ids: Optional[torch.Tensor] = None,
                inputs_embeds: Optional[torch.Tensor] = None) -> torch.Tensor:
        """input_ids [S] (or inputs_embeds [S, D] bf16, e.g. text embeddings with the vision rows
        spliced in), position_ids [3, S] (default: 0..S-1 on all three axes) -> last hidden state
        after the final norm, [S, D] bf16."""
        c, w, dev = self.config, self.w, self.device
        if not self.layers:
            raise RuntimeError("text encoder weights not loaded")
        D, H, Hk, Dh, F = c.hidden_size, c.num_attention_heads, c.num_key_value_heads, c.head_dim, c.intermediate_size
        S = int(input_ids.numel()) if inputs_embeds is None else int(inputs_embeds.shape[0])
        Sp = -(-S // 64) * 64  # padded rows: GEMM N / K alignment; causal masking keeps rows < S exact
        if position_ids is None:
            position_ids = torch.arange(S).view(1, S).expand(3, S)
        pos = torch.zeros(3, Sp, dtype=torch.long)
        pos[:, :S] = position_ids.cpu()
        cos, sin = (t.to(dev).contiguous() for t in mrope_tables(c, pos))
        x = torch.zeros(Sp, D, dtype=BF16, device=dev)
        if inputs_embeds is None:
            ids = torch.zeros(Sp, dtype=torch.int32, device=dev)
            ids[:S] = input_ids.reshape(-1).to(dev).to(torch.int32)
            ops.embed_rows(w["embed"], ids, out=x)
        else:
            x[:S] = inputs_embeds.to(dev).to(BF16)
        h = torch.empty(Sp, D, dtype=BF16, device=dev)
        qkv = torch.empty(Sp, (H + 2 * Hk) * Dh, dtype=BF16, device=dev)
        att = torch.empty(Sp, H * Dh, dtype=BF16, device=dev)
        s = torch.empty(Sp, Sp, dtype=torch.float32, device=dev)
        p = torch.empty(Sp, Sp, dtype=BF16, device=dev)
        vt = torch.empty(Dh, Sp, dtype=BF16, device=dev)
        gu = torch.empty(Sp, 2 * F, dtype=BF16, device=dev)
        a = torch.empty(Sp, F, dtype=BF16, device=dev)
        scale = 1.0 / math.sqrt(Dh)
        for L in self.layers:
            ops.rmsnorm(x, L["ln1"], out=h, eps=c.rms_norm_eps)
            ops.linear(h, L["w_qkv"], L["b_qkv"], out=qkv)
            ops.rope_half(qkv, 0, H + Hk, Dh, cos, sin)  # q heads, then the k heads right after them
            for kv in range(Hk):
                k = qkv[:, (H + kv) * Dh:(H + kv + 1) * Dh]
                ops.transpose(qkv[:, (H + Hk + kv) * Dh:(H + Hk + kv + 1) * Dh], out=vt)
                for hq in range(kv * (H // Hk), (kv + 1) * (H // Hk)):
                    ops.matmul_f32out(qkv[:, hq * Dh:(hq + 1) * Dh], k, out=s)
                    ops.softmax_rows(s, scale, out=p, causal=True)
                    ops.linear(p, vt, w["zero_hd"], out=att[:, hq * Dh:(hq + 1) * Dh])
            ops.linear_gated_residual(att, L["w_o"], w["zero_d"], w["ones"], Sp, x)
            ops.rmsnorm(x, L["ln2"], out=h, eps=c.rms_norm_eps)
            ops.linear(h, L["w_gu"], w["zero_2f"], out=gu)
            ops.silu_mul(gu, out=a)
            ops.linear_gated_residual(a, L["w_down"], w["zero_d"], w["ones"], Sp, x)
        ops.rmsnorm(x, w["norm"], out=h, eps=c.rms_norm_eps)
        return h[:S]

    __call__ = forward
