"""The /edit app over the HIP pipeline on the GPU: a tiny-config DiT behind the
real request path (decode -> 512x512 -> pipeline (batched true CFG when use_cfg) -> JPEG), with
deterministic stand-in encoders for the text encoder / VAE (§8 f1/f2 are not built yet). Checks
determinism and that the served image is exactly the image of a direct pipeline call."""
import base64
import io

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import dit_ref as R

pytestmark = pytest.mark.gpu


def _b64(img):
    buf = io.BytesIO()
    img.save(buf, format="PNG")
    return base64.b64encode(buf.getvalue()).decode()


def _make_pipeline(dev):
    from qwen_image_edit_streamdiffusion_amd import QwenImageEditPlusPipeline, QwenImageTransformer2DModel
    cfg = R.tiny_config()
    m = QwenImageTransformer2DModel(num_layers=cfg.num_layers, num_attention_heads=cfg.num_attention_heads,
                                    joint_attention_dim=cfg.joint_attention_dim, device=dev)
    m.load_diffusers_state_dict(R.random_params(cfg, seed=0))
    pipe = QwenImageEditPlusPipeline(m)
    jd = cfg.joint_attention_dim

    def prompt_encoder(prompt, images):
        g = torch.Generator().manual_seed(sum(map(ord, prompt or "")) + 1)
        n = 8 + len(prompt or "") % 8
        return torch.randn(1, n, jd, generator=g).to(torch.bfloat16).to(dev), torch.ones(1, n, dtype=torch.long, device=dev)

    def image_encoder(images):
        im = images[-1].resize((32, 32))
        x = torch.from_numpy(np.asarray(im, dtype=np.float32)).view(1, 1024, 3) / 127.5 - 1
        return x.repeat(1, 1, 22)[:, :, :64].to(torch.bfloat16).to(dev)

    def latent_decoder(lat, h, w):
        v = lat[0, :, :3].float().view(int(h) // 2, int(w) // 2, 3)
        v = ((v.clamp(-3, 3) + 3) * (255 / 6)).to(torch.uint8).cpu().numpy()
        return [Image.fromarray(v, "RGB")]

    pipe.prompt_encoder, pipe.image_encoder, pipe.latent_decoder = prompt_encoder, image_encoder, latent_decoder
    return pipe


def test_edit_over_hip_pipeline(dev):
    from fastapi.testclient import TestClient
    from qwen_image_edit_streamdiffusion_amd import server as S
    pipe = _make_pipeline(dev)
    src = Image.new("RGB", (300, 200), (120, 30, 200))
    with TestClient(S.create_app(loader=lambda: pipe, do_warmup=True)) as c:
        r1 = c.post("/edit", json={"image": _b64(src), "prompt": "oil painting"})
        r2 = c.post("/edit", json={"image": _b64(src), "prompt": "oil painting"})
        r3 = c.post("/edit", json={"image": _b64(src), "prompt": "oil painting", "use_cfg": True})
    for r in (r1, r2, r3):
        assert r.status_code == 200, r.text
    assert r1.json()["image"] == r2.json()["image"]       # deterministic (seed 42, same kernels)
    assert r1.json()["image"] != r3.json()["image"]       # true CFG changes the result
    direct = S.process_image_sync(pipe, src, "oil painting", 2, False)
    assert r1.json()["image"] == S.pil_to_base64(direct)
