"""Prompt-encoder checker: the reference's text encoder is transformers'
Qwen2.5-VL (un-vendored third-party code the reference pulls in through diffusers'
QwenImageEditPlusPipeline.encode_prompt [U]; pinned here: transformers 5.15.0, importable in this
image).  TEST INFRASTRUCTURE ONLY: this module builds small random-init instances of
``Qwen2_5_VLTextModel`` as the oracle the HIP language model is compared with.  No Qwen2.5-VL
weights exist offline, so parity is on random weights of reduced width (the same code path the
7B checkpoint runs)."""
from __future__ import annotations


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


def tiny_vl_model(seed: int = 0, text_hidden: int = 256, vis_hidden: int = 320, vis_heads: int = 4,
                  vis_intermediate: int = 200, depth: int = 4, fullatt=(1, 3), image_token_id: int = 990,
                  text_heads: int = 2, text_kv_heads: int = 1, text_layers: int = 2, text_intermediate: int = 512):
    """A random transformers Qwen2_5_VLModel (vision tower + language model, fp32 eager) whose
    weights are bf16-representable, and its state_dict. The vision head_dim is 80 (as in the 7B
    checkpoint) and the MLP width 200 is not a multiple of 64 (the HIP path pads both)."""
    from transformers import Qwen2_5_VLConfig
    from transformers.models.qwen2_5_vl.modeling_qwen2_5_vl import Qwen2_5_VLModel
    cfg = Qwen2_5_VLConfig(
        text_config=dict(vocab_size=1000, hidden_size=text_hidden, bos_token_id=0, eos_token_id=1,
                         intermediate_size=text_intermediate, num_hidden_layers=text_layers,
                         num_attention_heads=text_heads, num_key_value_heads=text_kv_heads, rms_norm_eps=1e-6,
                         rope_parameters={"rope_type": "default", "rope_theta": 1e6, "mrope_section": [16, 24, 24]}),
        vision_config=dict(depth=depth, hidden_size=vis_hidden, intermediate_size=vis_intermediate,
                           num_heads=vis_heads, out_hidden_size=text_hidden, fullatt_block_indexes=list(fullatt),
                           window_size=112, patch_size=14, spatial_merge_size=2, temporal_patch_size=2),
        bos_token_id=0, eos_token_id=1, image_token_id=image_token_id, video_token_id=991, vision_start_token_id=992, vision_end_token_id=993)
    cfg._attn_implementation = "eager"
    cfg.text_config._attn_implementation = "eager"
    cfg.vision_config._attn_implementation = "eager"
    torch.manual_seed(seed)
    m = Qwen2_5_VLModel(cfg).eval()
    with torch.no_grad():
        for name, p in m.named_parameters():
            if "norm" in name or "ln_q" in name:
                p.copy_(1.0 + 0.1 * torch.randn_like(p))
            elif name.endswith("bias"):
                p.copy_(0.1 * torch.randn_like(p))
            else:
                p.copy_(torch.randn_like(p) / (p[0].numel() ** 0.5))
            p.copy_(p.to(BF16).float())
    return m, {k: v.to(BF16) for k, v in m.state_dict().items()}


@torch.no_grad()
def vision_forward(m, pixel_values: torch.Tensor, grid_thw: torch.Tensor) -> torch.Tensor:
    """The tower's pooler output (merged embeddings, raster order), fp32."""
    return m.visual(pixel_values.float(), grid_thw=grid_thw).pooler_output


@torch.no_grad()
def vl_forward(m, input_ids: torch.Tensor, pixel_values=None, image_grid_thw=None) -> torch.Tensor:
    """Qwen2_5_VLModel last hidden state for one prompt (the reference's hidden_states[-1])."""
    ids = input_ids.view(1, -1)
    kw = {}
    if pixel_values is not None:
        kw = dict(pixel_values=pixel_values.float(), image_grid_thw=image_grid_thw,
                  mm_token_type_ids=(ids == m.config.image_token_id).int())
    out = m(input_ids=ids, output_hidden_states=True, **kw)
    return out.hidden_states[-1][0], out.last_hidden_state[0]
