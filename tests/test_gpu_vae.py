"""VAE decoder on the GPU: every VAE entry point of libqie vs the CPU oracle
(oracle/vae_ref.py, which keeps the causal 3-D form), then the whole decode.

Tolerances (bf16 storage, fp32 accumulation):
  * conv2d (implicit GEMM) vs fp32 F.conv2d on the same bf16 operands: rel-L2 <= 4e-3, max |diff|
    <= 2 bf16 ulps of max|ref| (as the GEMMs); the residual form adds one more rounding: 4 ulps
  * RMS_norm (+ SiLU), latents-in: rel-L2 <= 4e-3, 2 ulps (same rounding points as the oracle)
  * softmax rows: rel-L2 <= 4e-3; transpose: exact; fp32 matmul: rel-L2 <= 1e-5
  * whole decode (small config: base_dim 32, 32x32 latents -> 256x256): rel-L2 <= 3e-2 on the
    [-1, 1] image (every conv/norm re-rounds to bf16), uint8 RGB: mean |diff| <= 1.5 levels
"""
import math

import pytest
import torch
import torch.nn.functional as F

from oracle import vae_ref as V

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16


def _ops():
    from qwen_image_edit_streamdiffusion_amd import ops
    return ops


def rnd(shape, dev, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).to(BF16).to(dev)


def close(actual, ref, rel_l2=4e-3, ulps=2):
    a, r = actual.float().cpu(), ref.float().cpu()
    assert a.shape == r.shape, (a.shape, r.shape)
    assert torch.isfinite(a).all(), "non-finite output"
    err = (a - r).norm() / max(r.norm().item(), 1e-30)
    mx = (a - r).abs().max().item()
    bound = ulps * 2.0 ** -8 * r.abs().max().item() + 1e-6
    assert err <= rel_l2 and mx <= bound, f"rel_l2={err:.3e} max_abs={mx:.3e} bound={bound:.3e}"


def _nhwc(x):  # [C, H, W] -> [H*W, C]
    return x.permute(1, 2, 0).reshape(-1, x.shape[0]).contiguous()


@pytest.mark.parametrize("H,W,C,N,k,up", [
    (16, 16, 96, 96, 3, False),     # K = 864 -> padded 896
    (32, 8, 16, 384, 3, False),     # conv_in shape: C = 16, K = 144 -> 192
    (8, 16, 384, 192, 3, True),     # Resample: upsample folded into the gather
    (16, 16, 192, 384, 1, False),   # conv_shortcut 1x1
    (24, 20, 96, 4, 3, False),      # conv_out: 3 (+1 pad) channels, ragged tiles
    (128, 256, 64, 512, 3, False),  # many workgroups
    (64, 128, 96, 384, 3, True),    # upsampling gather, 2 workgroups per CU
    (32, 48, 96, 96, 3, "down"),    # encoder Resample: ZeroPad2d((0,1,0,1)) + stride 2
    (256, 512, 64, 128, 3, "down"),  # stride 2, many workgroups
    (256, 256, 64, 192, 3, False),  # 96-wide output tiles
    (256, 512, 32, 96, 3, False),   # N = 96, C = 32 < 64: multi-tap K tiles
    # halo-tiled kernel (>= 256 workgroups): ragged edges, both tile shapes, upsampled halo
    (250, 500, 96, 192, 3, False),  # 8 x 32 tiles x 192 channels, partial tiles at both edges
    (260, 600, 64, 96, 3, False),   # 16 x 32 tiles x 96 channels, partial tiles
    (130, 250, 192, 96, 3, True),   # upsampled halo (18 source columns), N = 96
    (66, 132, 128, 384, 3, True),   # upsampled halo, two 192-channel tiles
])
def test_conv2d(dev, H, W, C, N, k, up):
    from qwen_image_edit_streamdiffusion_amd.vae import conv_weight
    ops = _ops()
    x = rnd((C, H, W), dev, 1.0, 1)
    w4 = rnd((N, C, k, k), dev, 1.0 / math.sqrt(C * k * k), 2)
    b = rnd((N,), dev, 0.1, 3)
    down = up == "down"
    y = ops.conv2d(_nhwc(x), H, W, conv_weight(w4), b, ksize=k, up=up is True, down=down)
    xi = x.float().cpu()[None]
    if down:
        ref = F.conv2d(F.pad(xi, (0, 1, 0, 1)), w4.float().cpu(), b.float().cpu(), stride=2)[0].to(BF16)
    else:
        if up:
            xi = F.interpolate(xi, scale_factor=2.0, mode="nearest-exact")
        ref = F.conv2d(xi, w4.float().cpu(), b.float().cpu(), padding=k // 2)[0].to(BF16)
    close(y, _nhwc(ref))


def test_conv2d_residual_halo(dev):
    """The ResidualBlock epilogue (in place onto the shortcut) on the halo-tiled kernel's shapes."""
    from qwen_image_edit_streamdiffusion_amd.vae import conv_weight
    ops = _ops()
    for H, W, C, N in ((512, 256, 96, 96), (128, 512, 192, 192)):
        x = rnd((C, H, W), dev, 1.0, 8)
        w4 = rnd((N, C, 3, 3), dev, 1.0 / math.sqrt(9 * C), 9)
        b = rnd((N,), dev, 0.1, 10)
        h = rnd((N, H, W), dev, 1.0, 11)
        conv = F.conv2d(x.float().cpu()[None], w4.float().cpu(), b.float().cpu(), padding=1)[0]
        ref = (conv.to(BF16).float() + h.float().cpu()).to(BF16)
        out = _nhwc(h)
        ops.conv2d(_nhwc(x), H, W, conv_weight(w4), b, out=out, residual=True)
        close(out, _nhwc(ref), ulps=4)


@pytest.mark.parametrize("H,W,C,N,up", [
    (512, 256, 96, 96, False),   # halo kernel, N = 96: norm fused into the epilogue
    (256, 256, 192, 96, True),   # fused, upsampled halo
    (64, 64, 96, 96, False),     # too few tiles: conv_kernel, then the norm kernel
    (128, 256, 96, 192, False),  # N = 192 (channels over two waves): two launches
])
def test_conv2d_rmsnorm(dev, H, W, C, N, up):
    """conv1 + norm2 (+ SiLU) of the ResidualBlock in one call == the conv then qie_vae_rms_norm_bf16
    (the fused sum of squares runs in another order: within 1 bf16 ulp), and both vs the fp32
    reference chain."""
    from qwen_image_edit_streamdiffusion_amd.vae import conv_weight
    ops = _ops()
    x = rnd((C, H, W), dev, 1.0, 31)
    w4 = rnd((N, C, 3, 3), dev, 1.0 / math.sqrt(9 * C), 32)
    b = rnd((N,), dev, 0.1, 33)
    gamma = (1 + rnd((N,), dev, 0.1, 34).float()).to(BF16)
    fused = ops.conv2d_rmsnorm(_nhwc(x), H, W, conv_weight(w4), b, gamma, True, up=up)
    two = ops.conv2d(_nhwc(x), H, W, conv_weight(w4), b, up=up)
    ops.vae_rms_norm(two, gamma, True, out=two)
    close(fused, two, ulps=2)
    xi = x.float().cpu()[None]
    if up:
        xi = F.interpolate(xi, scale_factor=2.0, mode="nearest-exact")
    conv = F.conv2d(xi, w4.float().cpu(), b.float().cpu(), padding=1)[0].to(BF16).float()
    r = V._R(True)
    ref = V.silu(V.rms_norm(conv[None], gamma.float().cpu().view(N, 1, 1), r), r)[0]
    close(fused, _nhwc(ref.to(BF16)), rel_l2=8e-3, ulps=8)


def test_conv2d_residual_and_causal3d(dev):
    """A causal 3x3x3 conv on one frame (oracle: F.pad 2 zero frames + conv3d) == the 2-D conv with
    the last temporal slice, and the residual epilogue adds onto the shortcut in place."""
    from qwen_image_edit_streamdiffusion_amd.vae import conv_weight
    ops = _ops()
    H, W, C = 16, 24, 64
    x = rnd((C, H, W), dev, 1.0, 4)
    w5 = rnd((C, C, 3, 3, 3), dev, 1.0 / math.sqrt(27 * C), 5)
    b = rnd((C,), dev, 0.1, 6)
    h = rnd((C, H, W), dev, 1.0, 7)
    r = V._R(True)
    conv = V.causal_conv3d(x.float().cpu()[None, :, None], w5.cpu(), b.cpu(), 1, r)[0, :, 0]
    ref = r(conv + h.float().cpu())
    out = _nhwc(h)
    ops.conv2d(_nhwc(x), H, W, conv_weight(w5), b, out=out, residual=True)
    close(out, _nhwc(ref), ulps=4)


@pytest.mark.parametrize("C,silu", [(96, True), (384, False), (192, True), (16, True)])
def test_vae_rms_norm(dev, C, silu):
    ops = _ops()
    x = rnd((C, 8, 16), dev, 2.0, 8)
    g = (1 + rnd((C,), dev, 0.1, 9).float()).to(BF16)
    y = ops.vae_rms_norm(_nhwc(x), g, silu)
    r = V._R(True)
    ref = V.rms_norm(x.float().cpu()[None], g.cpu().view(C, 1, 1), r)
    if silu:
        ref = V.silu(ref, r)
    close(y, _nhwc(ref[0]))
    z = _nhwc(x)
    ops.vae_rms_norm(z, g, silu, out=z)  # in place
    assert torch.equal(z, y)


@pytest.mark.parametrize("P", [16384, 1000, 4104])
def test_vae_attention_flash(dev, P):
    """qie_vae_attention_bf16 (one head, C = 384) vs fp32 SDPA on the same bf16 q / k / v (torch on
    the device): rel-L2 <= 4e-3, max |diff| <= 4 bf16 ulps of max|ref| (P rounded to bf16 before
    P.V, as in the materialised form). 16384: two key ranges; 1000 / 4104: ragged, four ranges."""
    ops = _ops()
    C = 384
    qkv = rnd((P, 3 * C), dev, 1.0, 21)
    kp = -(-P // 64) * 64
    vt = torch.zeros(C, kp, dtype=BF16, device=dev)
    ops.transpose(qkv[:, 2 * C:], out=vt[:, :P])
    ws = torch.empty(-(-ops.vae_attention_workspace_bytes(P, C) // 4), dtype=torch.float32, device=dev)
    out = torch.empty(P, C, dtype=BF16, device=dev)
    ops.vae_attention(qkv, vt, out, ws)
    q, k, v = (qkv[:, i * C:(i + 1) * C].float() for i in range(3))
    ref = torch.softmax((q @ k.T) / math.sqrt(C), dim=-1) @ v
    close(out, ref.to(BF16), ulps=4)


def test_softmax_transpose_matmul(dev):
    ops = _ops()
    P, C = 2048, 384
    qkv = rnd((P, 3 * C), dev, 1.0, 10)
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    s = ops.matmul_f32out(q, k)
    sref = q.float().cpu() @ k.float().cpu().T
    assert ((s.cpu() - sref).norm() / sref.norm()).item() < 1e-5
    p = ops.softmax_rows(s, 1.0 / math.sqrt(C))
    close(p, torch.softmax(sref / math.sqrt(C), -1))
    vt = ops.transpose(v)
    assert torch.equal(vt.cpu(), v.cpu().T)
    # ragged row length into a K-padded output: zeros past column N
    s2 = s[:100, :1000].contiguous()
    out = torch.full((100, 1024), float("nan"), device=dev).to(BF16)
    ops.softmax_rows(s2, 0.05, out=out)
    close(out[:, :1000], torch.softmax(sref[:100, :1000] * 0.05, -1))
    assert (out[:, 1000:] == 0).all()


def test_vae_latents_in(dev):
    from qwen_image_edit_streamdiffusion_amd.vae import QwenImageVAEDecoder, VAEConfig
    ops = _ops()
    cfg = VAEConfig(base_dim=32)
    dec = QwenImageVAEDecoder(cfg, dev).random_init_(3)
    h, w = 16, 24
    packed = rnd((2, h * w // 4, 64), dev, 1.0, 11)
    y = ops.vae_latents_in(packed[1:].contiguous(), h, w, dec.w["sinv"], dec.w["mean"],
                           dec.w["post_quant_conv.weight"], dec.w["post_quant_conv.bias"])
    p = V.random_params(V.VAEConfig(base_dim=32), 3)
    r = V._R(True)
    z = V.unpack_latents(packed[1:].float().cpu(), h, w)
    mean_t = torch.tensor(V.LATENTS_MEAN).view(1, -1, 1, 1, 1).to(BF16).float()
    sinv = r(1.0 / torch.tensor(V.LATENTS_STD).view(1, -1, 1, 1, 1).to(BF16).float())
    z = r(r(z / sinv) + mean_t)
    ref = V.causal_conv3d(z, p["post_quant_conv.weight"], p["post_quant_conv.bias"], 0, r)[0, :, 0]
    close(y, _nhwc(ref))


def _small_decode(dev, seed=12):
    from qwen_image_edit_streamdiffusion_amd.vae import QwenImageVAEDecoder, VAEConfig
    cfg = VAEConfig(base_dim=32)
    dec = QwenImageVAEDecoder(cfg, dev).random_init_(5)
    h = w = 32  # mid-block attention over 1024 tokens; image 256 x 256
    packed = rnd((1, h * w // 4, 64), dev, 1.0, seed)
    p = V.random_params(V.VAEConfig(base_dim=32), 5)
    return dec, packed, p, h, w


def test_vae_decode_vs_oracle(dev):
    dec, packed, p, h, w = _small_decode(dev)
    img = dec.decode(packed, h, w, output="pt")[0]
    ref = V.decode(p, packed.cpu(), h, w, V.VAEConfig(base_dim=32), emulate_bf16=True)[0]
    assert img.shape == ref.shape == (3, 8 * h, 8 * w)
    err = ((img.float().cpu() - ref).norm() / ref.norm()).item()
    assert err <= 3e-2, err
    u8 = dec.decode(packed, h, w)[0]
    ru8 = V.to_uint8(ref[None])[0]
    assert u8.shape == ru8.shape and u8.dtype == torch.uint8
    assert (u8.cpu().float() - ru8.float()).abs().mean().item() <= 1.5


def test_vae_decode_ragged_latent(dev):
    """18 x 22 latents: mid-block attention over 396 tokens (P.V K padded to 448), ragged tiles."""
    from qwen_image_edit_streamdiffusion_amd.vae import QwenImageVAEDecoder, VAEConfig
    dec = QwenImageVAEDecoder(VAEConfig(base_dim=16), dev).random_init_(6)
    h, w = 18, 22
    packed = rnd((1, h * w // 4, 64), dev, 1.0, 15)
    img = dec.decode(packed, h, w, output="pt")[0]
    p = V.random_params(V.VAEConfig(base_dim=16), 6)
    ref = V.decode(p, packed.cpu(), h, w, V.VAEConfig(base_dim=16), emulate_bf16=True)[0]
    err = ((img.float().cpu() - ref).norm() / ref.norm()).item()
    assert err <= 3e-2, err


def test_vae_decode_deterministic_and_batch_independent(dev):
    dec, packed, _, h, w = _small_decode(dev, 13)
    two = torch.cat([packed, rnd(packed.shape, dev, 1.0, 14)]).contiguous()
    a = dec.decode(two, h, w)
    b = dec.decode(packed, h, w)
    assert torch.equal(a[:1], b)
    assert torch.equal(dec.decode(packed, h, w), b)


def test_pipeline_decodes_with_hip_vae(dev):
    """QwenImageEditPlusPipeline with pipe.vae set: output_type pil / np / pt / uint8 all come from
    the HIP decode of the same final latents (output_type="latent")."""
    from oracle import dit_ref as R
    from qwen_image_edit_streamdiffusion_amd import QwenImageEditPlusPipeline, QwenImageTransformer2DModel
    from qwen_image_edit_streamdiffusion_amd.vae import QwenImageVAEDecoder, VAEConfig
    cfg = R.tiny_config()
    m = QwenImageTransformer2DModel(num_layers=cfg.num_layers, num_attention_heads=cfg.num_attention_heads,
                                    joint_attention_dim=cfg.joint_attention_dim, device=dev)
    m.load_diffusers_state_dict(R.random_params(cfg, seed=0))
    pipe = QwenImageEditPlusPipeline(m)
    pipe.vae = QwenImageVAEDecoder(VAEConfig(base_dim=16), dev).random_init_(7)
    g = torch.Generator().manual_seed(8)
    pe = torch.randn(1, 20, cfg.joint_attention_dim, generator=g).to(BF16).to(dev)
    cond = torch.randn(1, 64, 64, generator=g).to(BF16).to(dev)
    kw = dict(prompt_embeds=pe, image_latents=cond, num_inference_steps=2, height=128, width=128)
    lat = pipe(generator=torch.Generator().manual_seed(42), output_type="latent", **kw).images
    u8 = pipe(generator=torch.Generator().manual_seed(42), output_type="uint8", **kw).images
    assert u8.shape == (1, 128, 128, 3) and u8.dtype == torch.uint8
    assert torch.equal(u8, pipe.vae.decode(lat, 16, 16))
    pil = pipe(generator=torch.Generator().manual_seed(42), **kw).images
    assert len(pil) == 1 and pil[0].size == (128, 128)
    import numpy as np
    assert np.array_equal(np.asarray(pil[0]), u8[0].cpu().numpy())
    pt = pipe(generator=torch.Generator().manual_seed(42), output_type="pt", **kw).images
    assert pt.shape == (1, 3, 128, 128) and torch.allclose(pt * 255, u8.permute(0, 3, 1, 2).float())


def test_vae_rgb_in_latents_out(dev):
    ops = _ops()
    g = torch.Generator().manual_seed(20)
    rgb = torch.randint(0, 256, (24 * 40, 3), generator=g, dtype=torch.uint8)
    x = ops.vae_rgb_in(rgb.to(dev))
    ref = (2.0 * (rgb.float() / 255.0) - 1.0).to(BF16)
    assert torch.equal(x[:, :3].cpu(), ref) and (x[:, 3:] == 0).all()
    z = rnd((2 * 16 * 24, 40), dev, 2.0, 21)  # quant_conv output, row stride 40 (>= 32)
    mean = torch.tensor(V.LATENTS_MEAN).to(BF16)
    std = torch.tensor(V.LATENTS_STD).to(BF16)
    packed = ops.vae_latents_out(z, 2, 16, 24, mean.to(dev), std.to(dev))
    mu = z[:, :16].cpu().float().view(2, 16, 24, 16).permute(0, 3, 1, 2)[:, :, None]
    r = V._R(True)
    want = V.pack_latents(r(r(mu - mean.float().view(1, -1, 1, 1, 1)) / std.float().view(1, -1, 1, 1, 1)))
    assert torch.equal(packed.cpu().float(), want)


def _small_encode(dev, seed=22):
    from qwen_image_edit_streamdiffusion_amd.vae import QwenImageVAEEncoder, VAEConfig
    enc = QwenImageVAEEncoder(VAEConfig(base_dim=16), dev).random_init_(9)
    g = torch.Generator().manual_seed(seed)
    rgb = torch.randint(0, 256, (1, 256, 256, 3), generator=g, dtype=torch.uint8)
    p = V.random_encoder_params(V.VAEConfig(base_dim=16), 9)
    return enc, rgb, p


def test_vae_encode_vs_oracle(dev):
    """Encoder (base_dim 16, 256x256 -> 32x32 latents, mid-block attention over 1024 tokens) vs
    the oracle's causal-3-D restatement: rel-L2 <= 3e-2 on the normalised packed latents."""
    enc, rgb, p = _small_encode(dev)
    z = enc.encode(rgb.to(dev))
    ref = V.encode(p, rgb, V.VAEConfig(base_dim=16), emulate_bf16=True)
    assert z.shape == ref.shape == (1, 256, 64)
    err = ((z.float().cpu() - ref).norm() / ref.norm()).item()
    assert err <= 3e-2, err


def test_pipeline_encodes_and_decodes_with_hip_vae(dev):
    """pipe(image=PIL) with the HIP encoder == pipe(image_latents=encoder(image)); the image is
    resized to the VAE size of its aspect ratio first."""
    from PIL import Image
    from oracle import dit_ref as R
    from qwen_image_edit_streamdiffusion_amd import QwenImageEditPlusPipeline, QwenImageTransformer2DModel
    from qwen_image_edit_streamdiffusion_amd.pipeline import images_to_rgb
    from qwen_image_edit_streamdiffusion_amd.vae import QwenImageVAEDecoder, QwenImageVAEEncoder, VAEConfig
    cfg = R.tiny_config()
    m = QwenImageTransformer2DModel(num_layers=cfg.num_layers, num_attention_heads=cfg.num_attention_heads,
                                    joint_attention_dim=cfg.joint_attention_dim, device=dev)
    m.load_diffusers_state_dict(R.random_params(cfg, seed=0))
    pipe = QwenImageEditPlusPipeline(m)
    pipe.vae = QwenImageVAEDecoder(VAEConfig(base_dim=16), dev).random_init_(7)
    pipe.vae_encoder = QwenImageVAEEncoder(VAEConfig(base_dim=16), dev).random_init_(8)
    g = torch.Generator().manual_seed(23)
    im = Image.fromarray(torch.randint(0, 256, (300, 300, 3), generator=g, dtype=torch.uint8).numpy())
    pe = torch.randn(1, 20, cfg.joint_attention_dim, generator=g).to(BF16).to(dev)
    rgb = images_to_rgb(im, dev)
    assert rgb.shape == (1, 1024, 1024, 3)
    kw = dict(prompt_embeds=pe, num_inference_steps=2, height=128, width=128, output_type="uint8")
    a = pipe(image=im, generator=torch.Generator().manual_seed(42), **kw).images
    lat = pipe.vae_encoder.encode(rgb)
    b = pipe(image_latents=lat, cond_shape=(64, 64), generator=torch.Generator().manual_seed(42), **kw).images
    assert a.shape == (1, 128, 128, 3) and torch.equal(a, b)
