"""Model / pipeline parity on the GPU (through the C ABI) against the CPU oracle.

Tolerances: the HIP forward rounds to bf16 at the same points as the
reference (oracle emulate_bf16=True) but accumulates in a different order, so
per-element bf16 ties flip and the differences compound through the layers:
  * tiny 2-layer model, full forward:     rel-L2 <= 2e-2
  * full-width (D=3072, H=24) one block:  rel-L2 <= 2e-2
  * batched CFG vs sequential CFG:        bitwise equal (same per-row math)
  * stream batch vs serial denoise:       bitwise equal
  * int8 (W8A8) vs bf16 model:            rel-L2 <= 8e-2 (quantisation error)
"""
import pytest
import torch

from oracle import dit_ref as R

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm()).item()


def make_model(cfg, params, dev):
    from qwen_image_edit_streamdiffusion_amd import QwenImageTransformer2DModel
    m = QwenImageTransformer2DModel(num_layers=cfg.num_layers, num_attention_heads=cfg.num_attention_heads,
                                    joint_attention_dim=cfg.joint_attention_dim, device=dev)
    m.load_diffusers_state_dict(params)
    return m


@pytest.fixture(scope="module")
def tiny(dev):
    cfg = R.tiny_config()
    params = R.random_params(cfg, seed=0)
    return cfg, params, make_model(cfg, params, dev)


def _inputs(B, shapes, S_txt, jd, seed=0):
    g = torch.Generator().manual_seed(seed)
    S_img = sum(f * h * w for f, h, w in shapes)
    hs = torch.randn(B, S_img, 64, generator=g).to(BF16)
    enc = torch.randn(B, S_txt, jd, generator=g).to(BF16)
    return hs, enc


def test_tiny_forward_vs_oracle(dev, tiny):
    cfg, params, m = tiny
    shapes = [(1, 8, 8), (1, 8, 8)]
    hs, enc = _inputs(2, shapes, 16, cfg.joint_attention_dim)
    lens = [16, 11]
    enc[1, 11:] = 0
    t = R.model_timestep(torch.tensor([1000.0, 20.0]))
    out = m(hs.to(dev), enc.to(dev), None, t.to(dev), [shapes] * 2, lens, return_dict=False)[0]
    ref = R.transformer_forward(params, cfg, hs, enc, t, shapes, lens)
    e = rel(out, ref)
    assert e <= 2e-2, e
    # rows must not leak into each other: row 0 alone gives the same result
    out0 = m(hs[:1].to(dev), enc[:1].to(dev), None, t[:1].to(dev), [shapes], lens[:1],
             return_dict=False)[0]
    assert torch.equal(out0, out[:1])


def test_batched_modulation_bitwise(dev, tiny):
    """One GEMV launch for every block's modulation == one launch per block and stream, bit for
    bit (each output column is the same wave's arithmetic either way); the per-block w_mod_*
    buffers are views of the packed [L * 12D, D] matrix the batched launch reads."""
    cfg, params, m = tiny
    blk = m.transformer_blocks[1]
    assert blk.w_mod_txt.data_ptr() == m._mod_w[blk.mod_off + 6 * m.config.inner_dim:].data_ptr()
    shapes = [(1, 8, 8), (1, 8, 8)]
    hs, enc = _inputs(2, shapes, 16, cfg.joint_attention_dim, seed=5)
    t = R.model_timestep(torch.tensor([1000.0, 500.0]))
    outs = []
    for batched in (True, False):
        m.batched_modulation = batched
        outs.append(m(hs.to(dev), enc.to(dev), None, t.to(dev), [shapes] * 2, [16, 16],
                      return_dict=False)[0].clone())
    m.batched_modulation = True
    assert torch.equal(outs[0], outs[1])


def test_full_width_block_vs_oracle(dev):
    cfg = R.DiTConfig(num_layers=1)
    params = R.random_params(cfg, seed=1)
    m = make_model(cfg, params, dev)
    shapes = [(1, 16, 16), (1, 16, 16)]
    hs, enc = _inputs(1, shapes, 64, cfg.joint_attention_dim, seed=2)
    t = R.model_timestep(torch.tensor([766.7094]))
    out = m(hs.to(dev), enc.to(dev), None, t.to(dev), [shapes], [64], return_dict=False)[0]
    ref = R.transformer_forward(params, cfg, hs, enc, t, shapes, [64])
    e = rel(out, ref)
    assert e <= 2e-2, e


def test_text_split_configs_vs_oracle(dev):
    """Text-stream linears split over K per linear (``text_splits`` dict, bench --text-splits):
    fp32 partials + reduce change only the summation order, so every configuration stays within
    the full-width bound of the oracle and close to the unsplit forward (rel-L2 <= 1e-2); the
    fused text QKV + norm + RoPE launch is used only when the text QKV is unsplit."""
    cfg = R.DiTConfig(num_layers=1)
    params = R.random_params(cfg, seed=3)
    m = make_model(cfg, params, dev)
    shapes = [(1, 16, 16), (1, 16, 16)]
    hs, enc = _inputs(2, shapes, 64, cfg.joint_attention_dim, seed=4)
    enc[1, 40:] = 0
    lens = [64, 40]
    t = R.model_timestep(torch.tensor([1000.0, 20.0]))
    ref = R.transformer_forward(params, cfg, hs, enc, t, shapes, lens)
    outs = {}
    for name, ts in (("unsplit", 1), ("down+out", {"down": 0, "out": 0}), ("qkv", {"qkv": 0}), ("all", None)):
        m.text_splits = ts
        outs[name] = m(hs.to(dev), enc.to(dev), None, t.to(dev), [shapes] * 2, lens, return_dict=False)[0].clone()
        assert rel(outs[name], ref) <= 2e-2, (name, rel(outs[name], ref))
    m.text_splits = 1
    for name in ("down+out", "qkv", "all"):
        assert rel(outs[name], outs["unsplit"]) <= 1e-2, name


def _pipe(m):
    from qwen_image_edit_streamdiffusion_amd import QwenImageEditPlusPipeline
    return QwenImageEditPlusPipeline(m)


def test_batched_cfg_equals_sequential(dev, tiny):
    cfg, params, m = tiny
    pipe = _pipe(m)
    g = torch.Generator().manual_seed(3)
    pe = torch.randn(1, 20, cfg.joint_attention_dim, generator=g).to(BF16).to(dev)
    ne = torch.randn(1, 13, cfg.joint_attention_dim, generator=g).to(BF16).to(dev)
    cond = torch.randn(1, 64, 64, generator=g).to(BF16).to(dev)
    kw = dict(prompt_embeds=pe, negative_prompt_embeds=ne, image_latents=cond, true_cfg_scale=4.0,
              num_inference_steps=2, height=128, width=128, output_type="latent")
    a = pipe(generator=torch.Generator().manual_seed(42), batched_cfg=True, **kw).images
    b = pipe(generator=torch.Generator().manual_seed(42), batched_cfg=False, **kw).images
    assert torch.equal(a, b), rel(a, b)


def test_pipeline_vs_oracle_denoise(dev, tiny):
    cfg, params, m = tiny
    pipe = _pipe(m)
    g = torch.Generator().manual_seed(4)
    pe = torch.randn(1, 20, cfg.joint_attention_dim, generator=g).to(BF16)
    ne = torch.randn(1, 13, cfg.joint_attention_dim, generator=g).to(BF16)
    cond = torch.randn(1, 64, 64, generator=g).to(BF16)
    noise = R.pack_latents(torch.randn((1, 1, 16, 16, 16), generator=torch.Generator().manual_seed(42)).to(BF16))
    out = pipe(prompt_embeds=pe.to(dev), negative_prompt_embeds=ne.to(dev), image_latents=cond.to(dev),
               latents=noise.to(dev), true_cfg_scale=4.0, num_inference_steps=2, height=128, width=128,
               output_type="latent").images
    ref = R.denoise(params, cfg, noise, cond, pe, [(1, 8, 8), (1, 8, 8)], 2, neg_embeds=ne)
    e = rel(out, ref)
    assert e <= 3e-2, e


@pytest.mark.parametrize("cfg_scale", [1.0, 4.0])
def test_stream_batch_equals_serial(dev, tiny, cfg_scale):
    cfg, params, m = tiny
    from qwen_image_edit_streamdiffusion_amd import StreamBatchDenoiser
    pipe = _pipe(m)
    g = torch.Generator().manual_seed(5)
    pe = torch.randn(1, 20, cfg.joint_attention_dim, generator=g).to(BF16).to(dev)
    ne = torch.randn(1, 13, cfg.joint_attention_dim, generator=g).to(BF16).to(dev)
    frames = [torch.randn(1, 64, 64, generator=g).to(BF16).to(dev) for _ in range(4)]
    noises = [torch.randn(1, 64, 64, generator=g).to(BF16).to(dev) for _ in range(4)]
    eng = StreamBatchDenoiser(m, num_steps=2, true_cfg_scale=cfg_scale, latent_hw=(8, 8), cond_hw=(8, 8))
    eng.set_conditions(pe, None, ne if cfg_scale > 1 else None)
    outs = {}
    for n, f in zip(noises, frames):
        r = eng.push(n, f)
        if r is not None:
            outs[r[0]] = r[1]
    for fid, lat in eng.flush():
        outs[fid] = lat
    assert sorted(outs) == [0, 1, 2, 3]
    for i in range(4):
        ser = pipe(prompt_embeds=pe, negative_prompt_embeds=ne if cfg_scale > 1 else None,
                   image_latents=frames[i], latents=noises[i], true_cfg_scale=cfg_scale,
                   num_inference_steps=2, height=128, width=128, output_type="latent").images
        assert torch.equal(outs[i], ser), (i, rel(outs[i], ser))


def test_int8_model_error_bound(dev, tiny):
    cfg, params, _ = tiny
    m8 = make_model(cfg, params, dev).quantize_int8()
    m16 = make_model(cfg, params, dev)
    shapes = [(1, 8, 8), (1, 8, 8)]
    hs, enc = _inputs(1, shapes, 16, cfg.joint_attention_dim, seed=6)
    t = R.model_timestep(torch.tensor([1000.0]))
    a = m8(hs.to(dev), enc.to(dev), None, t.to(dev), [shapes], [16], return_dict=False)[0]
    b = m16(hs.to(dev), enc.to(dev), None, t.to(dev), [shapes], [16], return_dict=False)[0]
    e = rel(a, b)
    assert e <= 8e-2, e


def test_lora_fuse_matches_dense_delta(dev, tiny):
    cfg, params, _ = tiny
    m = make_model(cfg, params, dev)
    from qwen_image_edit_streamdiffusion_amd import weights as W
    g = torch.Generator().manual_seed(7)
    D = cfg.inner_dim
    A = torch.randn(8, D, generator=g) * 0.01
    Bm = torch.randn(D, 8, generator=g) * 0.01
    sd = {"transformer.transformer_blocks.0.attn.to_k.lora_A.weight": A,
          "transformer.transformer_blocks.0.attn.to_k.lora_B.weight": Bm}
    assert W.fuse_lora(m, sd) == 1
    w = m._param_slot("transformer_blocks.0.attn.to_k.weight").float().cpu()
    exp = (params["transformer_blocks.0.attn.to_k.weight"].float() + Bm @ A).to(BF16).float()
    assert torch.equal(w, exp)


def test_int8_image_roundtrip_bitwise(dev, tiny, tmp_path):
    """A pre-quantised on-disk image reloads into a model that allocates no
    bf16 copy of the quantised linears and computes bitwise the same forward."""
    cfg, params, _ = tiny
    from qwen_image_edit_streamdiffusion_amd import weights as W
    from qwen_image_edit_streamdiffusion_amd import QwenImageEditPlusPipeline
    m8 = make_model(cfg, params, dev).quantize_int8()
    W.save_int8(m8, str(tmp_path / "transformer_int8"), blocks_per_shard=1)
    m8b = W.load_int8(str(tmp_path), device=dev)
    assert m8b.int8 and m8b.int8_only
    assert m8b.transformer_blocks[0].w_up_img.numel() == 0
    shapes = [(1, 8, 8), (1, 8, 8)]
    hs, enc = _inputs(2, shapes, 16, cfg.joint_attention_dim, seed=8)
    t = R.model_timestep(torch.tensor([1000.0, 20.0]))
    a = m8(hs.to(dev), enc.to(dev), None, t.to(dev), [shapes] * 2, [16, 16], return_dict=False)[0]
    b = m8b(hs.to(dev), enc.to(dev), None, t.to(dev), [shapes] * 2, [16, 16], return_dict=False)[0]
    assert torch.equal(a, b)
    pipe = QwenImageEditPlusPipeline.from_pretrained(str(tmp_path), device=dev)
    assert pipe.transformer.int8_only


def test_forward_three_image_segments_vs_oracle(dev, tiny):
    """Edit-Plus with two condition images: img_shapes carries three (frame, h, w) entries, each a
    RoPE frame index of its own (noise latents, picture 1, picture 2 of another size)."""
    cfg, params, m = tiny
    g = torch.Generator().manual_seed(41)
    shapes = [(1, 8, 8), (1, 8, 8), (1, 4, 8)]
    S = sum(f * h * w for f, h, w in shapes)
    hs = torch.randn(1, S, 64, generator=g).to(torch.bfloat16)
    enc = torch.randn(1, 12, cfg.joint_attention_dim, generator=g).to(torch.bfloat16)
    t = R.model_timestep(torch.tensor([500.0]))
    out = m(hs.to(dev), enc.to(dev), None, t.to(dev), [shapes], [12], return_dict=False)[0]
    ref = R.transformer_forward(params, cfg, hs, enc, t, shapes, [12])
    assert ((out.float().cpu() - ref).norm() / ref.norm()).item() <= 2e-2


def test_pipeline_two_condition_images(dev, tiny):
    """pipe(image=[PIL, PIL]) VAE-encodes each picture at its own aspect ratio and concatenates
    them == pipe(image_latents=cat(...), cond_shape=[...])."""
    from PIL import Image
    from qwen_image_edit_streamdiffusion_amd import QwenImageEditPlusPipeline
    from qwen_image_edit_streamdiffusion_amd.pipeline import images_to_rgb
    from qwen_image_edit_streamdiffusion_amd.vae import QwenImageVAEDecoder, QwenImageVAEEncoder, VAEConfig
    cfg, params, m = tiny
    pipe = QwenImageEditPlusPipeline(m)
    pipe.vae = QwenImageVAEDecoder(VAEConfig(base_dim=16), dev).random_init_(7)
    pipe.vae_encoder = QwenImageVAEEncoder(VAEConfig(base_dim=16), dev).random_init_(8)
    g = torch.Generator().manual_seed(43)
    ims = [Image.fromarray(torch.randint(0, 256, (h, w, 3), generator=g, dtype=torch.uint8).numpy())
           for h, w in ((300, 300), (200, 400))]
    pe = torch.randn(1, 20, cfg.joint_attention_dim, generator=g).to(torch.bfloat16).to(dev)
    kw = dict(prompt_embeds=pe, num_inference_steps=2, height=128, width=128, output_type="uint8")
    a = pipe(image=ims, generator=torch.Generator().manual_seed(42), **kw).images
    rgbs = [images_to_rgb(im, dev) for im in ims]
    assert rgbs[0].shape[1:3] == (1024, 1024) and rgbs[1].shape[1] < rgbs[1].shape[2]  # own aspect ratios
    lat = torch.cat([pipe.vae_encoder.encode(r) for r in rgbs], 1)
    shapes = [(r.shape[1] // 16, r.shape[2] // 16) for r in rgbs]
    b = pipe(image_latents=lat, cond_shape=shapes, generator=torch.Generator().manual_seed(42), **kw).images
    assert a.shape == (1, 128, 128, 3) and torch.equal(a, b)
    with pytest.raises(ValueError):
        pipe(image_latents=lat, cond_shape=shapes[:1], generator=torch.Generator().manual_seed(42), **kw)


def test_modulation_cache_bitwise_and_invalidated(dev, tiny):
    """The cached modulation vectors (keyed on scheduler.model_timesteps' host values) give the
    same forward bit for bit, alternate between two keys like the stream engine, and are dropped
    when the weights change."""
    from qwen_image_edit_streamdiffusion_amd import weights as W
    from qwen_image_edit_streamdiffusion_amd.scheduler import model_timesteps
    cfg, params, _ = tiny
    m = make_model(cfg, params, dev)
    shapes = [(1, 8, 8), (1, 8, 8)]
    hs, enc = _inputs(2, shapes, 16, cfg.joint_attention_dim, seed=3)
    hs, enc = hs.to(dev), enc.to(dev)
    ta, tb = model_timesteps([1000.0, 20.0], dev), model_timesteps([20.0, 1000.0], dev)

    def run(t):
        return m(hs, enc, None, t, [shapes] * 2, [16, 16], return_dict=False)[0].clone()

    m.cache_modulation = False
    ref_a, ref_b = run(ta), run(tb)
    m.cache_modulation = True
    outs = [run(ta), run(tb), run(ta), run(tb)]  # miss, miss, hit, hit
    assert len(m._mod_cache) == 2
    for o, r in zip(outs, [ref_a, ref_b, ref_a, ref_b]):
        assert torch.equal(o, r)
    # an untagged tensor (no host copy) is never cached
    m(hs, enc, None, ta.clone(), [shapes] * 2, [16, 16], return_dict=False)
    assert len(m._mod_cache) == 2
    # weights change -> cache dropped, new result
    D = cfg.inner_dim
    g = torch.Generator().manual_seed(9)
    sd = {"transformer_blocks.0.img_mod.1.lora_A.weight": torch.randn(4, D, generator=g) * 0.1,
          "transformer_blocks.0.img_mod.1.lora_B.weight": torch.randn(6 * D, 4, generator=g) * 0.1}
    W.fuse_lora(m, sd)
    assert len(m._mod_cache) == 0
    m.cache_modulation = False
    ref_new = run(ta)
    m.cache_modulation = True
    assert torch.equal(run(ta), ref_new) and torch.equal(run(ta), ref_new)
    assert not torch.equal(ref_new, ref_a)
    # an in-place write outside the loaders (no clear_modulation_cache call) must miss the cache:
    # the weights' version counters are part of the key
    with torch.no_grad():
        m._param_slot("transformer_blocks.1.txt_mod.1.bias").add_(0.25)
        m.norm_out_w.mul_(1.5)
    m.cache_modulation = False
    ref_inplace = run(ta)
    m.cache_modulation = True
    assert torch.equal(run(ta), ref_inplace) and torch.equal(run(ta), ref_inplace)
    assert not torch.equal(ref_inplace, ref_new)


def test_cfg_pair_engine_layouts_equal_batched_cfg(dev, tiny):
    """parallel.CFGPairStreamDenoiser on the HIP path, single process: a pair of one (both branches
    local, the exchange still taken) and two engines wired through begin() / finish() both equal
    the batched-CFG stream engine bit for bit."""
    cfg, params, m = tiny
    from qwen_image_edit_streamdiffusion_amd import StreamBatchDenoiser
    from qwen_image_edit_streamdiffusion_amd.parallel import CFGPairStreamDenoiser
    g = torch.Generator().manual_seed(51)
    pe = torch.randn(1, 20, cfg.joint_attention_dim, generator=g).to(BF16).to(dev)
    ne = torch.randn(1, 13, cfg.joint_attention_dim, generator=g).to(BF16).to(dev)
    frames = [(torch.randn(1, 64, 64, generator=g).to(BF16).to(dev),
               torch.randn(1, 64, 64, generator=g).to(BF16).to(dev)) for _ in range(4)]
    kw = dict(num_steps=2, true_cfg_scale=4.0, latent_hw=(8, 8), cond_hw=(8, 8))

    def drive(eng):
        outs = {}
        for n, c in frames:
            r = eng.push(n, c)
            if r is not None:
                outs[r[0]] = r[1].clone()
        outs.update({k: v.clone() for k, v in eng.flush()})
        return outs

    base = StreamBatchDenoiser(m, **kw)
    base.set_conditions(pe, None, ne)
    ref = drive(base)
    one = CFGPairStreamDenoiser(m, role=0, group_size=1, exchange=lambda v: [v.clone()], **kw)
    one.set_conditions(pe, None, ne)
    assert one.rows == 4
    got = drive(one)
    assert sorted(got) == [0, 1, 2, 3] and all(torch.equal(got[i], ref[i]) for i in range(4))
    eng = [CFGPairStreamDenoiser(m, role=r, exchange=lambda v: None, **kw) for r in (0, 1)]
    for e in eng:
        e.set_conditions(pe, None, ne)
    both = {0: {}, 1: {}}

    def push_pair(n, c):
        parts = [e.begin(n, c).clone() for e in eng]
        for r in (0, 1):
            res = eng[r].finish(parts)
            if res is not None:
                both[r][res[0]] = res[1].clone()

    for n, c in frames:
        push_pair(n, c)
    while any(s >= 0 for s in eng[0].stage):
        push_pair(None, None)
    for r in (0, 1):
        assert all(torch.equal(both[r][i], ref[i]) for i in range(4)), r
    with pytest.raises(ValueError):
        CFGPairStreamDenoiser(m, role=0, group_size=1, exchange=lambda v: [v], **dict(kw, true_cfg_scale=1.0))


def test_stream_per_frame_prompt_equals_serial(dev, tiny):
    """Every frame with its own prompt embedding (the reference's realtime call re-encodes the
    prompt with each camera frame, qwen_realtime.py:247-255): the stream engine's per-slot text
    rows give each frame exactly the serial pipeline's result for ITS embedding -- lengths differ
    per frame, so rows of one forward carry different valid text lengths."""
    cfg, params, m = tiny
    from qwen_image_edit_streamdiffusion_amd import StreamBatchDenoiser
    pipe = _pipe(m)
    g = torch.Generator().manual_seed(52)
    lens = [20, 17, 20, 11]
    pes = [torch.randn(1, n, cfg.joint_attention_dim, generator=g).to(BF16).to(dev) for n in lens]
    ne = torch.randn(1, 13, cfg.joint_attention_dim, generator=g).to(BF16).to(dev)
    frames = [torch.randn(1, 64, 64, generator=g).to(BF16).to(dev) for _ in range(4)]
    noises = [torch.randn(1, 64, 64, generator=g).to(BF16).to(dev) for _ in range(4)]
    for cfg_scale in (1.0, 4.0):
        eng = StreamBatchDenoiser(m, num_steps=2, true_cfg_scale=cfg_scale, latent_hw=(8, 8), cond_hw=(8, 8))
        eng.set_conditions(pes[0], None, ne if cfg_scale > 1 else None)
        outs = {}
        for i in range(4):
            r = eng.push(noises[i], frames[i], prompt_embeds=pes[i])
            if r is not None:
                outs[r[0]] = r[1].clone()
        outs.update({k: v.clone() for k, v in eng.flush()})
        for i in range(4):
            ser = pipe(prompt_embeds=pes[i], negative_prompt_embeds=ne if cfg_scale > 1 else None,
                       image_latents=frames[i], latents=noises[i], true_cfg_scale=cfg_scale,
                       num_inference_steps=2, height=128, width=128, output_type="latent").images
            assert torch.equal(outs[i], ser), (cfg_scale, i, rel(outs[i], ser))
    with pytest.raises(ValueError):  # longer than the text rows set_conditions() sized
        eng.push(noises[0], frames[0], prompt_embeds=torch.zeros(1, 21, cfg.joint_attention_dim, dtype=BF16, device=dev))


def test_realtime_latent_cache_through_stream_engine(dev, tiny):
    """qwen_realtime.py:201-224 prepare_latent (never called by the reference's own loop): fresh
    noise on keyframes (every ``keyframe_interval`` frames, and while no frame has completed),
    otherwise the last completed latent + noise_strength * noise. Through QwenRealtimePipeline and
    the stream engine: the latents each frame started from follow that rule with the pipeline's
    generator stream, and every finished frame equals the serial 2-step pipeline run from the same
    start latents, bitwise."""
    cfg, params, m = tiny
    from qwen_image_edit_streamdiffusion_amd import QwenRealtimePipeline, StreamConfig
    sc = StreamConfig(num_inference_steps=2, true_cfg_scale=1.0, noise_strength=0.05, keyframe_interval=3,
                      output_size=(128, 128), cond_size=(128, 128), use_prev_latent=True)
    rt = QwenRealtimePipeline(sc)
    rt.load_model(transformer=m)
    g = torch.Generator().manual_seed(53)
    pe = torch.randn(1, 20, cfg.joint_attention_dim, generator=g).to(BF16).to(dev)
    rt.precompute_conditions("a prompt", prompt_embeds=pe)
    conds = [torch.randn(1, 64, 64, generator=g).to(BF16).to(dev) for _ in range(7)]
    starts, keyflags, prevs = [], [], []
    orig = rt.prepare_latent

    def spy(cond):
        prevs.append(None if rt.prev_latent is None else rt.prev_latent.clone())
        x = orig(cond)
        starts.append(x.clone())
        keyflags.append(rt.is_keyframe)
        return x

    rt.prepare_latent = spy
    done = []
    for c in conds:
        out = rt.process_frame(c)
        if out is not None:
            done.append(out.clone())
    done += [lat.clone() for _, lat in rt.engine.flush()]
    assert len(done) == 7
    # the rule, replayed with the same generator stream (seed 42 on the device, load_model)
    gen = torch.Generator(device=dev).manual_seed(42)
    assert keyflags == [True, True, False, True, False, False, True]  # no finished frame yet at frame 1
    for i in range(7):
        noise = torch.randn((1, 64, 64), generator=gen, device=dev, dtype=BF16)
        if keyflags[i]:
            exp = noise
        else:
            assert prevs[i] is not None and torch.equal(prevs[i], done[i - 2])  # depth 2: frame i-2 is the last finished
            exp = (prevs[i].float() + 0.05 * noise.float()).to(BF16)
        assert torch.equal(starts[i], exp), i
    pipe = _pipe(m)
    for i in range(7):
        ser = pipe(prompt_embeds=pe, image_latents=conds[i], latents=starts[i], true_cfg_scale=1.0,
                   num_inference_steps=2, height=128, width=128, output_type="latent").images
        assert torch.equal(done[i], ser), (i, rel(done[i], ser))
