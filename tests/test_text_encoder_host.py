"""Prompt encoder host logic on the CPU: the 3-D M-RoPE tables against transformers' own
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


GRIDS = [[(1, 20, 28)], [(1, 16, 16)], [(2, 8, 12)], [(1, 28, 28), (1, 10, 36)]]


@pytest.mark.parametrize("grid", GRIDS)
def test_vision_index_logic_matches_transformers(grid):
    """Window permutation, window / frame boundaries and (h, w) positions vs transformers.vision_utils."""
    pytest.importorskip("transformers")
    from transformers import vision_utils as vu
    from qwen_image_edit_streamdiffusion_amd.vision import frame_seqlens, vision_position_ids, window_index
    g = torch.tensor(grid)
    wi, cu = window_index(grid, 2, 112, 14)
    wi_ref, cu_ref = vu.get_vision_window_index(g, spatial_merge_size=2, window_size=112, patch_size=14)
    assert torch.equal(wi, wi_ref) and cu == cu_ref.tolist()
    assert torch.equal(vision_position_ids(grid, 2), vu.get_vision_position_ids(g, 2))
    ref = vu.get_vision_cu_seqlens(g).tolist()  # one full-attention block per frame
    assert frame_seqlens(grid) == ref


def test_rope_index_matches_transformers():
    vl = pytest.importorskip("oracle.vl_ref")
    from qwen_image_edit_streamdiffusion_amd.text_encoder import rope_index
    m, _ = vl.tiny_vl_model(0, depth=2, fullatt=(1,))
    grid = torch.tensor([[1, 20, 28], [1, 8, 12]])
    ids = torch.cat([torch.arange(5), torch.full((140,), 990), torch.arange(7) + 10, torch.full((24,), 990),
                     torch.arange(3) + 20]).view(1, -1)
    want, _ = m.get_rope_index(ids, (ids == 990).int(), image_grid_thw=grid)
    got = rope_index(ids[0], 990, grid, 2)
    assert torch.equal(got, want[:, 0])
    with pytest.raises(ValueError):
        rope_index(ids[0, :100], 990, grid, 2)


def test_condition_size_and_prompt_hook_host():
    from qwen_image_edit_streamdiffusion_amd.text_encoder import (PROMPT_TEMPLATE, QwenImageEditPromptEncoder,
                                                                  condition_size)
    assert condition_size(1024, 1024) == (384, 384)
    assert condition_size(1920, 1080) == (512, 288)
    seen = {}

    class Proc:  # records what the hook hands to the processor
        def __call__(self, text, images=None, return_tensors=None):
            seen["text"], seen["images"] = text, images
            return {"input_ids": torch.arange(80).view(1, -1), "attention_mask": torch.ones(1, 80, dtype=torch.long)}

    class Enc:
        def __call__(self, ids, pv, grid):
            return torch.arange(ids.numel(), dtype=torch.float).view(-1, 1).expand(-1, 4).to(torch.bfloat16)

    from PIL import Image
    e, mask = QwenImageEditPromptEncoder(Enc(), Proc())("make it red", Image.new("RGB", (1024, 768)))
    assert seen["text"] == [PROMPT_TEMPLATE.format("Picture 1: <|vision_start|><|image_pad|><|vision_end|>make it red")]
    assert seen["images"][0].size == (448, 320)
    assert e.shape == (1, 16, 4) and e[0, 0, 0].item() == 64 and mask.sum().item() == 16


def test_state_dict_shapes_match_transformers():
    vl = pytest.importorskip("oracle.vl_ref")
    from qwen_image_edit_streamdiffusion_amd.text_encoder import text_state_dict_shapes
    from qwen_image_edit_streamdiffusion_amd.vision import VisionConfig, vision_state_dict_shapes
    _, sd = vl.tiny_vl_model(0)
    tc = TextEncoderConfig(vocab_size=1000, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                           num_attention_heads=2, num_key_value_heads=1)
    vc = VisionConfig(depth=4, hidden_size=320, intermediate_size=200, num_heads=4, out_hidden_size=256)
    want = {k: tuple(v.shape) for k, v in sd.items()}
    got = {"language_model." + k: v for k, v in text_state_dict_shapes(tc).items()}
    got.update({"visual." + k: v for k, v in vision_state_dict_shapes(vc).items()})
    assert got == want


def test_load_prompt_encoder_from_snapshot(tmp_path):
    """text_encoder/config.json + safetensors (transformers 4.x key layout, lm_head present) -> the
    encoder's configs and packed weights (loaded on the CPU; the forward needs the GPU)."""
    import json
    from safetensors.torch import save_file
    vl = pytest.importorskip("oracle.vl_ref")
    from qwen_image_edit_streamdiffusion_amd.weights import load_prompt_encoder
    m, sd = vl.tiny_vl_model(3)
    d = tmp_path / "text_encoder"
    d.mkdir()
    old = {("model." + k[len("language_model."):] if k.startswith("language_model.") else k): v.contiguous()
           for k, v in sd.items()}
    old["lm_head.weight"] = torch.zeros(1000, 256, dtype=BF16)
    save_file(old, str(d / "model.safetensors"))
    cfg = m.config.to_dict()
    tcd = cfg.pop("text_config")
    cfg.update(tcd)  # 4.x layout: text fields at the top level
    (d / "config.json").write_text(json.dumps(cfg))
    enc = load_prompt_encoder(str(tmp_path), device="cpu")
    assert enc.text.config.hidden_size == 256 and enc.text.config.num_key_value_heads == 1
    assert enc.vision.config.hidden_size == 320 and enc.vision.config.fullatt_block_indexes == (1, 3)
    assert enc.vision.config.intermediate_size == 200 and enc.image_token_id == 990
    assert torch.equal(enc.text.w["embed"], sd["language_model.embed_tokens.weight"])
    assert torch.equal(enc.vision.blocks[1]["w_down"][:, :200], sd["visual.blocks.1.mlp.down_proj.weight"])


def test_from_pretrained_wires_snapshot_prompt_encoder(tmp_path, monkeypatch):
    """A snapshot with text_encoder/ + processor/ gives pipe.prompt_encoder (loaded on the CPU here;
    the processor is stubbed -- the tokenizer files come with a real checkpoint)."""
    import json
    import transformers
    from safetensors.torch import save_file
    vl = pytest.importorskip("oracle.vl_ref")
    from qwen_image_edit_streamdiffusion_amd.pipeline import QwenImageEditPlusPipeline
    from qwen_image_edit_streamdiffusion_amd.text_encoder import QwenImageEditPromptEncoder
    m, sd = vl.tiny_vl_model(6)
    d = tmp_path / "text_encoder"
    d.mkdir()
    (tmp_path / "processor").mkdir()
    save_file({"model." + k: v.contiguous() for k, v in sd.items()}, str(d / "model.safetensors"))
    (d / "config.json").write_text(json.dumps(m.config.to_dict()))
    seen = {}

    def fake_from_pretrained(path, **kw):
        seen["path"], seen["kw"] = path, kw
        return "processor"

    monkeypatch.setattr(transformers.AutoProcessor, "from_pretrained", staticmethod(fake_from_pretrained))
    hook = QwenImageEditPlusPipeline._snapshot_prompt_encoder(str(tmp_path), "cpu")
    assert isinstance(hook, QwenImageEditPromptEncoder) and hook.processor == "processor"
    assert seen["path"].endswith("processor") and seen["kw"].get("local_files_only") is True
    assert hook.encoder.text.config.hidden_size == 256 and hook.encoder.image_token_id == 990


def test_prompt_hook_cache():
    """Repeated (prompt, image) pairs are served from the embedding cache; a new prompt or new
    image contents miss it; the LRU bound holds."""
    from PIL import Image
    from qwen_image_edit_streamdiffusion_amd.text_encoder import QwenImageEditPromptEncoder
    calls = []

    class Proc:
        def __call__(self, text, images=None, return_tensors=None):
            calls.append(text[0])
            return {"input_ids": torch.arange(70).view(1, -1)}

    class Enc:
        def __call__(self, ids, pv, grid):
            return torch.full((ids.numel(), 4), float(len(calls)), dtype=torch.bfloat16)

    hook = QwenImageEditPromptEncoder(Enc(), Proc(), cache_size=2)
    a, b = Image.new("RGB", (64, 64), "red"), Image.new("RGB", (64, 64), "blue")
    e1, _ = hook("x", a)
    e2, _ = hook("x", Image.new("RGB", (64, 64), "red"))  # same contents, new object
    assert len(calls) == 1 and e2 is e1
    hook("x", b)
    hook("y", a)
    assert len(calls) == 3
    hook("x", a)  # evicted by the bound of 2
    assert len(calls) == 4


def test_condition_image_resized_lanczos():
    """The processor gets the condition image resized with LANCZOS (Edit-Plus'
    VaeImageProcessor.resize default), not PIL's default BICUBIC."""
    import numpy as np
    from PIL import Image
    from qwen_image_edit_streamdiffusion_amd.text_encoder import QwenImageEditPromptEncoder
    seen = {}

    class Proc:
        def __call__(self, text, images=None, return_tensors=None):
            seen["images"] = images
            return {"input_ids": torch.arange(80).view(1, -1)}

    class Enc:
        def __call__(self, ids, pv, grid):
            return torch.zeros(ids.numel(), 4, dtype=torch.bfloat16)

    rng = np.random.default_rng(1)
    im = Image.fromarray(rng.integers(0, 255, (480, 640, 3), dtype=np.uint8))
    QwenImageEditPromptEncoder(Enc(), Proc())("p", im)
    got = np.asarray(seen["images"][0])
    w, h = seen["images"][0].size
    assert np.array_equal(got, np.asarray(im.resize((w, h), Image.LANCZOS)))
    assert not np.array_equal(got, np.asarray(im.resize((w, h), Image.BICUBIC)))
