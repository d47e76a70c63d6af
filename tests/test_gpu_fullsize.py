"""Parity at the headline sizes (BASELINE configs[2]: 60 blocks, D = 3072, 1024^2 -> 8192 image +
216 text tokens, B = 2 stream-batch rows) through size-independent properties. The CPU oracle
cannot run these sizes in seconds, so the checks are:
  * attention at the full joint shape (B = 2, H = 24, S = 8408, row 1 with 5 padded text keys,
    log2-q + split tail, the model path) vs fp32 softmax on sampled query rows: rel-L2 <= 1e-2;
  * the 60-block forward: finite, bitwise deterministic, and row-independent (row b of a B = 2
    forward == the same row run alone, bitwise -- what makes batched CFG equal sequential CFG);
  * the stream-batch engine (depth 2) == the serial 2-step pipeline per frame, bitwise;
  * the VAE at 1024^2: encode and decode finite and bitwise deterministic.
Random-init weights of the real architecture (no checkpoint offline).
"""
import math

import pytest
import torch

from oracle import dit_ref as R

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16
S_IMG, S_TXT, D, H = 8192, 216, 3072, 24
SHAPES = [(1, 64, 64), (1, 64, 64)]


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm()).item()


@pytest.fixture(scope="module")
def big(dev):
    from qwen_image_edit_streamdiffusion_amd import QwenImageTransformer2DModel
    m = QwenImageTransformer2DModel(num_layers=60, device=dev).random_init_(seed=0)
    yield m
    del m
    torch.cuda.empty_cache()


def test_attention_headline_shape_sampled_rows(dev):
    from qwen_image_edit_streamdiffusion_amd import ops
    B, S = 2, S_IMG + S_TXT
    s_pad = ((S + 255) // 256) * 256
    kv_len = [S, S - 5]
    g = torch.Generator(device=dev).manual_seed(7)
    qkv = torch.randn(3, B, H, s_pad, 128, generator=g, device=dev).to(BF16)
    qkv[:, :, :, S:] = 0
    qkv[0] = (qkv[0].float() * (math.log2(math.e) / math.sqrt(128))).to(BF16)  # log2-unit q
    nb = ops.attention_workspace_bytes(B, H, s_pad, S_IMG, S_TXT)
    ws = torch.full((nb // 4,), float("nan"), device=dev)
    oi = torch.empty(B * S_IMG, H * 128, dtype=BF16, device=dev)
    ot = torch.empty(B * S_TXT, H * 128, dtype=BF16, device=dev)
    ops.attention(qkv, kv_len, oi, ot, S_IMG, S_TXT, workspace=ws, log2q=True)
    torch.cuda.synchronize()
    # first / last rows of query blocks, the split tail block (rows >= 8192) and random rows
    rows = sorted(set([0, 1, 255, 256, 4095, 8191, 8192, 8200, 8300, S - 1] +
                      torch.randint(0, S, (54,), generator=torch.Generator().manual_seed(8)).tolist()))
    for b in range(B):
        L = kv_len[b]
        q = qkv[0, b][:, rows].float()                      # [H, R, 128]
        k, v = qkv[1, b, :, :L].float(), qkv[2, b, :, :L].float()
        p = torch.softmax(q @ k.transpose(-1, -2) * math.log(2.0), -1)
        ref = (p @ v).permute(1, 0, 2).reshape(len(rows), H * 128)
        got = torch.stack([oi[b * S_IMG + r] if r < S_IMG else ot[b * S_TXT + r - S_IMG] for r in rows])
        assert torch.isfinite(got.float()).all()
        e = rel(got, ref)
        assert e <= 1e-2, (b, e)


def _fullsize_inputs(dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    hs = torch.randn(2, S_IMG, 64, generator=g, device=dev).to(BF16)
    enc = torch.randn(2, S_TXT, 3584, generator=g, device=dev).to(BF16)
    enc[1, S_TXT - 5:] = 0  # row 1: a 211-token prompt padded to 216 (batched-CFG layout)
    return hs, enc, [S_TXT, S_TXT - 5]


def test_fullsize_forward_deterministic_and_row_independent(dev, big):
    hs, enc, lens = _fullsize_inputs(dev, 11)
    t = R.model_timestep(torch.tensor([1000.0, 20.0])).to(dev)
    a = big(hs, enc, None, t, [SHAPES] * 2, lens, return_dict=False)[0].clone()
    b = big(hs, enc, None, t, [SHAPES] * 2, lens, return_dict=False)[0].clone()
    assert a.shape == (2, S_IMG, 64) and torch.isfinite(a.float()).all()
    assert torch.equal(a, b)
    for r in range(2):
        one = big(hs[r:r + 1], enc[r:r + 1, :lens[r]], None, t[r:r + 1], [SHAPES], lens[r:r + 1],
                  return_dict=False)[0]
        assert torch.equal(one, a[r:r + 1]), (r, rel(one, a[r:r + 1]))


def test_fullsize_stream_batch_equals_serial(dev, big):
    from qwen_image_edit_streamdiffusion_amd import QwenImageEditPlusPipeline, StreamBatchDenoiser
    g = torch.Generator(device=dev).manual_seed(12)
    pe = torch.randn(1, S_TXT, 3584, generator=g, device=dev).to(BF16)
    frames = [torch.randn(1, 4096, 64, generator=g, device=dev).to(BF16) for _ in range(3)]
    noises = [torch.randn(1, 4096, 64, generator=g, device=dev).to(BF16) for _ in range(3)]
    eng = StreamBatchDenoiser(big, num_steps=2, latent_hw=(64, 64), cond_hw=(64, 64))
    eng.set_conditions(pe)
    outs = {}
    for n, f in zip(noises, frames):
        r = eng.push(n, f)
        if r is not None:
            outs[r[0]] = r[1].clone()
    for fid, lat in eng.flush():
        outs[fid] = lat.clone()
    assert sorted(outs) == [0, 1, 2]
    pipe = QwenImageEditPlusPipeline(big)
    for i in range(3):
        ser = pipe(prompt_embeds=pe, image_latents=frames[i], latents=noises[i], true_cfg_scale=1.0,
                   num_inference_steps=2, height=1024, width=1024, output_type="latent").images
        assert torch.isfinite(ser.float()).all()
        assert torch.equal(outs[i], ser), (i, rel(outs[i], ser))


def test_fullsize_vae_deterministic(dev):
    from qwen_image_edit_streamdiffusion_amd.vae import QwenImageVAEDecoder, QwenImageVAEEncoder
    enc = QwenImageVAEEncoder(device=dev).random_init_(seed=2)
    dec = QwenImageVAEDecoder(device=dev).random_init_(seed=1)
    g = torch.Generator(device=dev).manual_seed(13)
    rgb = torch.randint(0, 256, (1, 1024, 1024, 3), generator=g, device=dev, dtype=torch.uint8)
    z0, z1 = enc.encode(rgb).clone(), enc.encode(rgb).clone()
    assert z0.shape == (1, 4096, 64) and torch.isfinite(z0.float()).all()
    assert torch.equal(z0, z1)
    i0, i1 = dec.decode(z0, 128, 128).clone(), dec.decode(z0, 128, 128).clone()
    assert i0.dtype == torch.uint8 and i0.shape == (1, 1024, 1024, 3)
    assert torch.equal(i0, i1)
    assert 0 < i0.float().std().item()  # not a constant image
