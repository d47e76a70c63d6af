"""The /edit app over the HIP pipeline on the GPU (the serving surface of server.py:43-55, 99-120,
183-230): the real request path -- base64 decode -> 512x512 -> QwenImageEditPlusPipeline (batched
true CFG when use_cfg) -> JPEG q90 -- with every model stage on the HIP path: the VAE encoder
and decoder (reduced width, random weights), the Qwen2.5-VL prompt encoder (a tiny vision tower +
language model behind a stub of the processor's contract: a prompt-dependent token sequence and
image-dependent patches) and a tiny-config DiT. Checks determinism, that the prompt, the image and
true CFG each change the result, and that the served image is exactly a direct pipeline call's."""
import base64
import hashlib
import io

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import dit_ref as R
from oracle import vl_ref as VL

pytestmark = pytest.mark.gpu


def _b64(img):
    buf = io.BytesIO()
    img.save(buf, format="PNG")
    return base64.b64encode(buf.getvalue()).decode()


class _Processor:
    """The HF processor's contract (input_ids, attention_mask, pixel_values, image_grid_thw) on
    synthetic vocabulary: 64 template tokens, one 8x8-patch image block (16 merged image tokens),
    then tokens derived from the text; patches derived from the condition image's pixels."""

    def __init__(self):
        self.calls = []

    def __call__(self, text, images=None, return_tensors=None):
        self.calls.append((text[0], None if images is None else [im.size for im in images]))
        body = [b * 3 for b in hashlib.sha1(text[0].encode()).digest()]  # 20 tokens < 900, from the whole text
        ids = list(range(100, 164)) + [992] + [990] * 16 + [993] + body
        out = {"input_ids": torch.tensor(ids).view(1, -1), "attention_mask": torch.ones(1, len(ids), dtype=torch.long)}
        if images:
            im = np.asarray(images[0].convert("RGB").resize((112, 112)), dtype=np.float32) / 127.5 - 1
            pv = torch.from_numpy(im).reshape(-1)[: 64 * 588].view(64, 588)
            out["pixel_values"] = torch.cat([pv, pv], 1)  # 64 patches x 1176 (two temporal copies)
            out["image_grid_thw"] = torch.tensor([[1, 8, 8]])
        return out


def _make_pipeline(dev):
    from qwen_image_edit_streamdiffusion_amd import QwenImageEditPlusPipeline, QwenImageTransformer2DModel
    from qwen_image_edit_streamdiffusion_amd.text_encoder import (QwenImageEditPromptEncoder, QwenVLEncoder,
                                                                  TextEncoderConfig)
    from qwen_image_edit_streamdiffusion_amd.vae import QwenImageVAEDecoder, QwenImageVAEEncoder, VAEConfig
    from qwen_image_edit_streamdiffusion_amd.vision import VisionConfig
    cfg = R.tiny_config()
    m = QwenImageTransformer2DModel(num_layers=cfg.num_layers, num_attention_heads=cfg.num_attention_heads,
                                    joint_attention_dim=cfg.joint_attention_dim, device=dev)
    m.load_diffusers_state_dict(R.random_params(cfg, seed=0))
    _, sd = VL.tiny_vl_model(5, text_hidden=cfg.joint_attention_dim, text_heads=1)
    enc = QwenVLEncoder(TextEncoderConfig(vocab_size=1000, hidden_size=cfg.joint_attention_dim, intermediate_size=512,
                                          num_hidden_layers=2, num_attention_heads=1, num_key_value_heads=1),
                        VisionConfig(depth=4, hidden_size=320, intermediate_size=200, num_heads=4,
                                     out_hidden_size=cfg.joint_attention_dim, fullatt_block_indexes=(1, 3)),
                        dev, image_token_id=990).load_state_dict(sd)
    proc = _Processor()
    pipe = QwenImageEditPlusPipeline(m, prompt_encoder=QwenImageEditPromptEncoder(enc, proc))
    pipe.vae = QwenImageVAEDecoder(VAEConfig(base_dim=16), dev).random_init_(7)
    pipe.vae_encoder = QwenImageVAEEncoder(VAEConfig(base_dim=16), dev).random_init_(8)
    return pipe, proc


def test_edit_over_hip_pipeline(dev):
    from fastapi.testclient import TestClient
    from qwen_image_edit_streamdiffusion_amd import server as S
    pipe, proc = _make_pipeline(dev)
    rng = np.random.default_rng(3)
    src = Image.fromarray(rng.integers(0, 256, (200, 300, 3), dtype=np.uint8))
    other = Image.fromarray(rng.integers(0, 256, (200, 300, 3), dtype=np.uint8))
    with TestClient(S.create_app(loader=lambda: pipe, do_warmup=True)) as c:
        r1 = c.post("/edit", json={"image": _b64(src), "prompt": "oil painting"})
        r2 = c.post("/edit", json={"image": _b64(src), "prompt": "oil painting"})
        r3 = c.post("/edit", json={"image": _b64(src), "prompt": "oil painting", "use_cfg": True})
        r4 = c.post("/edit", json={"image": _b64(src), "prompt": "pencil sketch"})
        r5 = c.post("/edit", json={"image": _b64(other), "prompt": "oil painting"})
    for r in (r1, r2, r3, r4, r5):
        assert r.status_code == 200, r.text
    img = lambda r: r.json()["image"]  # noqa: E731
    assert img(r1) == img(r2), "served result not deterministic (seed 42, same kernels)"
    out = Image.open(io.BytesIO(base64.b64decode(img(r1))))
    assert out.size == (1024, 1024)  # Edit-Plus' default 1024^2-area output for a square 512^2 input
    # the processor saw the Edit-Plus template with one picture block and the 384^2-area condition image
    text, sizes = proc.calls[-1]
    assert "Picture 1: <|vision_start|><|image_pad|><|vision_end|>oil painting" in text and sizes == [(384, 384)]
    direct = S.process_image_sync(pipe, src, "oil painting", 2, False)
    assert img(r1) == S.pil_to_base64(direct), "served image != direct pipeline call"
    # true CFG, the prompt (through the HIP prompt encoder) and the image (through the HIP VAE encoder
    # and the vision tower) each reach the result. Compared on the latents the decoder is fed: a
    # random-weight decoder moves its uint8 output by less than one level for any latent change.
    def latents(image, prompt, use_cfg):
        kw = dict(image=[image.resize((S.SERVE_SIZE, S.SERVE_SIZE), Image.LANCZOS)], prompt=prompt,
                  num_inference_steps=2, generator=torch.Generator(device="cuda").manual_seed(S.SEED),
                  output_type="latent")
        if use_cfg:
            kw["negative_prompt"] = ""
        return pipe(**kw).images.clone()

    base = latents(src, "oil painting", False)
    assert base.shape == (1, 4096, 64) and torch.isfinite(base.float()).all()
    assert torch.equal(base, latents(src, "oil painting", False))
    for what, args in (("use_cfg", (src, "oil painting", True)), ("prompt", (src, "pencil sketch", False)),
                       ("image", (other, "oil painting", False))):
        assert not torch.equal(latents(*args), base), f"{what} does not change the latents"
