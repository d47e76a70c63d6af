"""Prompt encoder (§8 f2) host logic on the CPU: the 3-D M-RoPE tables against transformers' own
rotary embedding (oracle/vl_ref.py), the weight packing and config checks."""
import pytest
import torch

from qwen_image_edit_streamdiffusion_amd.text_encoder import QwenVLTextModel, TextEncoderConfig, mrope_tables

BF16 = torch.bfloat16


def _apply(q, cos, sin):  # rotate-half with the merged tables, fp32
    half = q.shape[-1] // 2
    rot = torch.cat([-q[..., half:], q[..., :half]], -1)
    return q * cos[:, None] + rot * sin[:, None]


def test_mrope_tables_match_transformers():
    vl = pytest.importorskip("oracle.vl_ref")
    cfg = TextEncoderConfig(hidden_size=256, num_attention_heads=2, num_key_value_heads=1)
    S = 40
    g = torch.Generator().manual_seed(0)
    pos = torch.stack([torch.arange(S), torch.arange(S) * 2 % 17, torch.arange(S) * 3 % 11])  # distinct t/h/w
    q = torch.randn(S, 2, 128, generator=g)
    want = vl.rotary_reference(256, 2, (16, 24, 24), pos, q)
    cos, sin = mrope_tables(cfg, pos)
    got = _apply(q, cos.float(), sin.float())
    # the tables are bf16 (transformers casts cos / sin to the activation dtype): 2^-8 relative
    assert ((got - want).norm() / want.norm()).item() < 4e-3


def test_text_model_weight_packing_and_config_checks():
    vl = pytest.importorskip("oracle.vl_ref")
    m, sd = vl.tiny_text_model(1)
    cfg = TextEncoderConfig(vocab_size=1000, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                            num_attention_heads=2, num_key_value_heads=1)
    te = QwenVLTextModel(cfg, "cpu").load_state_dict({"model.language_model." + k: v for k, v in sd.items()})
    L = te.layers[0]
    assert L["w_qkv"].shape == (256 + 2 * 128, 256) and L["b_qkv"].shape == (512,)
    assert torch.equal(L["w_gu"][:512], sd["layers.0.mlp.gate_proj.weight"])
    with pytest.raises(ValueError):
        QwenVLTextModel(TextEncoderConfig(hidden_size=256, num_attention_heads=2, mrope_section=(8, 8, 8)), "cpu")
