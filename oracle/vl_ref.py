"""Prompt-encoder checker: the reference's text encoder is transformers'
Qwen2.5-VL (un-vendored third-party code the reference pulls in through diffusers'
QwenImageEditPlusPipeline.encode_prompt [U]; pinned here: transformers 5.15.0, importable in this
image).  TEST INFRASTRUCTURE ONLY: this module builds small random-init instances of
``Qwen2_5_VLTextModel`` as the oracle the HIP language model is compared with.  No Qwen2.5-VL
weights exist offline, so parity is on random weights of reduced width (the same code path the
7B checkpoint runs)."""
from __future__ import annotations

from typing import Dict, Tuple

import torch

BF16 = torch.bfloat16


def tiny_text_model(seed: int = 0, hidden: int = 256, heads: int = 2, kv_heads: int = 1, layers: int = 2,
                    intermediate: int = 512, vocab: int = 1000, mrope=(16, 24, 24)):
    """A random transformers Qwen2_5_VLTextModel (fp32, eager attention) whose weights are exactly
    bf16-representable, and its state_dict."""
    import transformers  # noqa: F401
    from transformers import Qwen2_5_VLTextConfig
    from transformers.models.qwen2_5_vl.modeling_qwen2_5_vl import Qwen2_5_VLTextModel
    cfg = Qwen2_5_VLTextConfig(vocab_size=vocab, hidden_size=hidden, intermediate_size=intermediate,
                               num_hidden_layers=layers, num_attention_heads=heads, num_key_value_heads=kv_heads,
                               rms_norm_eps=1e-6, max_position_embeddings=8192, bos_token_id=0, eos_token_id=1,
                               rope_parameters={"rope_type": "default", "rope_theta": 1e6,
                                                "mrope_section": list(mrope)})
    cfg._attn_implementation = "eager"
    torch.manual_seed(seed)
    m = Qwen2_5_VLTextModel(cfg).eval()
    with torch.no_grad():
        for name, p in m.named_parameters():
            if name.endswith("norm.weight") or "layernorm" in name:
                p.copy_(1.0 + 0.1 * torch.randn_like(p))
            elif name.endswith("bias"):
                p.copy_(0.1 * torch.randn_like(p))
            else:
                p.copy_(torch.randn_like(p) / (p.shape[-1] ** 0.5))
            p.copy_(p.to(BF16).float())
    return m, {k: v.to(BF16) for k, v in m.state_dict().items()}


@torch.no_grad()
def text_forward(m, input_ids=None, position_ids=None, inputs_embeds=None) -> torch.Tensor:
    """Last hidden state (after the final norm) of one sequence, fp32 [S, D]."""
    kw = {}
    if position_ids is not None:
        kw["position_ids"] = position_ids.view(3, 1, -1)
    if inputs_embeds is not None:
        out = m(inputs_embeds=inputs_embeds.float()[None], **kw)
    else:
        out = m(input_ids=input_ids.view(1, -1), **kw)
    return out.last_hidden_state[0]


def rotary_reference(hidden: int, heads: int, mrope, position_ids: torch.Tensor, q: torch.Tensor
                     ) -> torch.Tensor:
    """transformers' own M-RoPE on q [S, heads, Dh] (fp32): Qwen2_5_VLRotaryEmbedding +
    apply_multimodal_rotary_pos_emb."""
    from transformers import Qwen2_5_VLTextConfig
    from transformers.models.qwen2_5_vl.modeling_qwen2_5_vl import (Qwen2_5_VLRotaryEmbedding,
                                                                    apply_multimodal_rotary_pos_emb)
    cfg = Qwen2_5_VLTextConfig(hidden_size=hidden, num_attention_heads=heads, num_key_value_heads=heads,
                               rope_parameters={"rope_type": "default", "rope_theta": 1e6,
                                                "mrope_section": list(mrope)})
    rot = Qwen2_5_VLRotaryEmbedding(cfg)
    x = q.float().permute(1, 0, 2)[None]  # [1, heads, S, Dh]
    cos, sin = rot(x, position_ids.view(3, 1, -1))
    qe, _ = apply_multimodal_rotary_pos_emb(x, x, cos, sin, list(mrope))
    return qe[0].permute(1, 0, 2)
