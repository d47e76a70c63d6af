"""CPU checks of the product's host logic against the oracle: scheduler math,
RoPE tables, pipeline dimension rules, diffusers state_dict packing, LoRA fuse,
host-side argument validation, and the stream-batch slot bookkeeping (with the
device ops replaced by CPU stand-ins, test-only)."""
import numpy as np
import os

import pytest
import torch

from oracle import dit_ref as R
from qwen_image_edit_streamdiffusion_amd import ops, pipeline, rope, scheduler, stream
from qwen_image_edit_streamdiffusion_amd import weights as W
from qwen_image_edit_streamdiffusion_amd.transformer import QwenImageTransformer2DModel

BF16 = torch.bfloat16


@pytest.mark.parametrize("n", [2, 3, 4, 8, 28])
@pytest.mark.parametrize("seq", [256, 1024, 4096, 8192])
def test_scheduler_matches_oracle(n, seq):
    s = scheduler.FlowMatchEulerDiscreteScheduler()
    s.set_timesteps(n, image_seq_len=seq)
    ref, ts = R.sigma_schedule(n, seq)
    assert torch.equal(s.sigmas, ref)
    assert torch.equal(s.timesteps, ts)
    for i in range(n):
        assert s.dt(i) == float((ref[i + 1] - ref[i]).item())


def test_scheduler_rejects_single_step_terminal_stretch():
    with pytest.raises(ValueError):
        scheduler.FlowMatchEulerDiscreteScheduler().set_timesteps(1, image_seq_len=4096)


def test_model_timesteps_match_oracle():
    ts = [1000.0, 766.7094, 455.6137, 20.0]
    a = scheduler.model_timesteps(ts, "cpu")
    assert torch.equal(a, R.model_timestep(torch.tensor(ts)))


@pytest.mark.parametrize("shapes,txt", [([(1, 64, 64), (1, 64, 64)], 216), ([(1, 8, 12), (1, 16, 16)], 7),
                                        ([(1, 32, 32)], 0)])
def test_rope_tables_match_oracle(shapes, txt):
    ia, ta = rope.rope_angles(shapes, txt)
    ip, tp = R.rope_phases(shapes, txt)
    assert torch.equal(ia, ip) and torch.equal(ta, tp)


def test_calculate_dimensions():
    assert pipeline.calculate_dimensions(1024 * 1024, 1.0) == (1024, 1024)
    w, h = pipeline.calculate_dimensions(1024 * 1024, 4 / 3)
    assert w % 32 == 0 and h % 32 == 0 and abs(w / h - 4 / 3) < 0.05
    assert pipeline.calculate_dimensions(384 * 384, 1.0) == (384, 384)


def _tiny_cpu_model(params=None):
    cfg = R.tiny_config()
    m = QwenImageTransformer2DModel(num_layers=cfg.num_layers, num_attention_heads=cfg.num_attention_heads,
                                    joint_attention_dim=cfg.joint_attention_dim, device="cpu")
    if params is not None:
        m.load_diffusers_state_dict(params)
    return cfg, m


def test_state_dict_packing_roundtrip():
    cfg = R.tiny_config()
    params = R.random_params(cfg, seed=5)
    _, m = _tiny_cpu_model(params)
    D = cfg.inner_dim
    blk = m.transformer_blocks[1]
    assert torch.equal(blk.w_qkv_img[D:2 * D], params["transformer_blocks.1.attn.to_k.weight"])
    assert torch.equal(blk.b_qkv_txt[2 * D:], params["transformer_blocks.1.attn.add_v_proj.bias"])
    assert torch.equal(blk.w_down_txt, params["transformer_blocks.1.txt_mlp.net.2.weight"])
    assert torch.equal(blk.norm_added_k, params["transformer_blocks.1.attn.norm_added_k.weight"])
    out = dict(m.diffusers_state_dict())
    assert set(out) == set(params)
    for k, v in params.items():
        assert torch.equal(out[k], v), k
    assert m.config.num_layers == 2 and m.config["attention_head_dim"] == 128


def test_state_dict_strictness():
    cfg = R.tiny_config()
    params = R.random_params(cfg, seed=5)
    _, m = _tiny_cpu_model()
    bad = dict(params)
    bad["transformer_blocks.0.attn.bogus.weight"] = torch.zeros(1)
    with pytest.raises(KeyError):
        m.load_diffusers_state_dict(bad)
    missing = dict(params)
    missing.pop("proj_out.bias")
    with pytest.raises(KeyError):
        m.load_diffusers_state_dict(missing)


def test_random_init_seeded_and_norm_weights_near_one():
    _, a = _tiny_cpu_model()
    _, b = _tiny_cpu_model()
    a.random_init_(seed=7)
    b.random_init_(seed=7)
    for (k, x), (_, y) in zip(a.diffusers_state_dict(), b.diffusers_state_dict()):
        assert torch.equal(x, y), k
    nq = a.transformer_blocks[0].norm_q.float()
    assert abs(nq.mean().item() - 1.0) < 0.02
    assert abs(a.transformer_blocks[0].w_up_img.float().std().item() - 0.02) < 0.002


def test_lora_fuse_on_packed_slices():
    cfg = R.tiny_config()
    params = R.random_params(cfg, seed=5)
    _, m = _tiny_cpu_model(params)
    D = cfg.inner_dim
    g = torch.Generator().manual_seed(1)
    A, B = torch.randn(4, D, generator=g) * 0.1, torch.randn(D, 4, generator=g) * 0.1
    sd = {"transformer_blocks.1.attn.add_q_proj.lora_down.weight": A,
          "transformer_blocks.1.attn.add_q_proj.lora_up.weight": B,
          "transformer_blocks.1.attn.add_q_proj.alpha": torch.tensor(2.0)}
    assert W.fuse_lora(m, sd, scale=1.0) == 1
    exp = (params["transformer_blocks.1.attn.add_q_proj.weight"].float() + 0.5 * (B @ A)).to(BF16)
    assert torch.equal(m.transformer_blocks[1].w_qkv_txt[:D], exp)
    # the neighbouring k slice is untouched
    assert torch.equal(m.transformer_blocks[1].w_qkv_txt[D:2 * D],
                       params["transformer_blocks.1.attn.add_k_proj.weight"])


_LORA_FORMS = {
    # peft / diffusers (transformer. prefix, optional .default adapter name)
    "peft": ("transformer.{s}.lora_A.weight", "transformer.{s}.lora_B.weight", None),
    "peft_default": ("{s}.lora_A.default.weight", "{s}.lora_B.default.weight", None),
    # lightx2v / ComfyUI: diffusion_model. prefix on either naming
    "comfy_AB": ("diffusion_model.{s}.lora_A.weight", "diffusion_model.{s}.lora_B.weight", None),
    "comfy_updown": ("diffusion_model.{s}.lora_down.weight", "diffusion_model.{s}.lora_up.weight",
                     "diffusion_model.{s}.alpha"),
    # kohya: lora_unet_ + the stem with every "." as "_"
    "kohya": ("lora_unet_{u}.lora_down.weight", "lora_unet_{u}.lora_up.weight", "lora_unet_{u}.alpha"),
}


@pytest.mark.parametrize("form", sorted(_LORA_FORMS))
@pytest.mark.parametrize("stem", ["transformer_blocks.0.attn.to_out.0", "transformer_blocks.1.img_mlp.net.0.proj",
                                  "transformer_blocks.1.attn.add_k_proj", "transformer_blocks.0.txt_mod.1"])
def test_lora_key_forms_fuse(form, stem):
    cfg = R.tiny_config()
    params = R.random_params(cfg, seed=5)
    _, m = _tiny_cpu_model(params)
    w0 = params[stem + ".weight"]
    g = torch.Generator().manual_seed(2)
    A = torch.randn(4, w0.shape[1], generator=g) * 0.1
    B = torch.randn(w0.shape[0], 4, generator=g) * 0.1
    ka, kb, kal = _LORA_FORMS[form]
    sub = dict(s=stem, u=stem.replace(".", "_"))
    sd = {ka.format(**sub): A, kb.format(**sub): B}
    s = 1.0
    if kal:
        sd[kal.format(**sub)] = torch.tensor(8.0)
        s = 2.0
    assert W.fuse_lora(m, sd) == 1
    exp = (w0.float() + s * (B @ A)).to(BF16)
    assert torch.equal(m._param_slot(stem + ".weight"), exp)


def test_lora_rejects_unmapped_keys():
    cfg = R.tiny_config()
    _, m = _tiny_cpu_model(R.random_params(cfg, seed=5))
    D = cfg.inner_dim
    A, B = torch.zeros(4, D), torch.zeros(D, 4)
    good = {"transformer_blocks.0.attn.to_q.lora_A.weight": A, "transformer_blocks.0.attn.to_q.lora_B.weight": B}
    # nothing maps: always an error, strict or not
    bad = {"single_blocks.0.linear.lora_A.weight": A, "single_blocks.0.linear.lora_B.weight": B}
    for strict in (True, False):
        with pytest.raises(W.LoraKeyError):
            W.fuse_lora(m, bad, strict=strict)
    with pytest.raises(W.LoraKeyError):
        W.fuse_lora(m, {}, strict=False)
    # a half-adapter or a stray key: error when strict, skipped otherwise
    for extra in ({"transformer_blocks.0.attn.to_k.lora_A.weight": A}, {"some.other.tensor": A},
                  bad):
        with pytest.raises(W.LoraKeyError):
            W.fuse_lora(m, {**good, **extra})
        assert W.fuse_lora(m, {**good, **extra}, strict=False) == 1
    # shapes that do not fit the weight: always an error
    with pytest.raises(W.LoraKeyError):
        W.fuse_lora(m, {"transformer_blocks.0.attn.to_q.lora_A.weight": torch.zeros(4, D + 1),
                        "transformer_blocks.0.attn.to_q.lora_B.weight": B}, strict=False)


def test_ops_reject_host_tensors():
    x = torch.zeros(32, 64, dtype=BF16)
    with pytest.raises(ValueError):
        ops.linear(x, torch.zeros(64, 64, dtype=BF16), torch.zeros(64, dtype=BF16))
    with pytest.raises(ValueError):
        ops.silu(x)


def test_flops_match_oracle():
    from qwen_image_edit_streamdiffusion_amd.transformer import TransformerConfig
    full = QwenImageTransformer2DModel.__new__(QwenImageTransformer2DModel)  # no 41 GB allocation
    full.config = TransformerConfig()
    assert QwenImageTransformer2DModel.flops_per_forward(full, 8192, 216) == pytest.approx(
        R.flops_per_forward(8192, 216))


# ----------------------------------------------------------------------------- stream bookkeeping
class _FakeTF:
    """Deterministic per-row stand-in for the DiT: v = 0.5*x + t (row-local)."""
    device = torch.device("cpu")

    def __call__(self, inp, enc, mask, t, shapes, lens, return_dict=False):
        return (0.5 * inp.float() + t.float()[:, None, None]).to(BF16),


@pytest.fixture
def cpu_ops(monkeypatch):
    def copy_batched(src, dst):
        dst.copy_(src)
        return dst

    def euler_step(x, v, dt, out):
        for b in range(x.shape[0]):
            out[b] = R.euler_step(x[b], v[b], 0.0, dt[b])
        return out

    def cfg_combine(c, u, s, out=None):
        r = R.cfg_combine(c, u, s)
        if out is not None:
            out.copy_(r)
            return out
        return r

    monkeypatch.setattr(stream.ops, "copy_batched", copy_batched)
    monkeypatch.setattr(stream.ops, "euler_step", euler_step)
    monkeypatch.setattr(stream.ops, "cfg_combine", cfg_combine)


def _serial(tf, noise, cond, steps, cfg_scale, pe, ne):
    eng = stream.StreamBatchDenoiser(tf, num_steps=steps, true_cfg_scale=cfg_scale, latent_hw=(2, 2),
                                     cond_hw=(2, 2))
    eng.set_conditions(pe, None, ne)
    eng.push(noise, cond)
    return eng.flush()[0][1]


@pytest.mark.parametrize("steps,cfg_scale", [(2, 1.0), (3, 1.0), (2, 4.0)])
def test_stream_slots_fill_steady_flush(cpu_ops, steps, cfg_scale):
    tf = _FakeTF()
    pe = torch.randn(1, 5, 8).to(BF16)
    ne = torch.randn(1, 3, 8).to(BF16) if cfg_scale > 1 else None
    eng = stream.StreamBatchDenoiser(tf, num_steps=steps, true_cfg_scale=cfg_scale, latent_hw=(2, 2),
                                     cond_hw=(2, 2))
    eng.set_conditions(pe, None, ne)
    g = torch.Generator().manual_seed(0)
    frames = [(torch.randn(1, 4, 64, generator=g).to(BF16), torch.randn(1, 4, 64, generator=g).to(BF16))
              for _ in range(6)]
    got = []
    for i, (n, c) in enumerate(frames):
        r = eng.push(n, c)
        if i < steps - 1:
            assert r is None  # pipeline filling
        else:
            assert r is not None and r[0] == i - steps + 1  # FIFO, one frame per push
            got.append(r)
    got += eng.flush()
    assert [f for f, _ in got] == list(range(6))
    for fid, lat in got:
        ref = _serial(tf, frames[fid][0], frames[fid][1], steps, cfg_scale, pe, ne)
        assert torch.equal(lat, ref), fid


def test_realtime_frame_resize_non_square():
    """A 640x480 webcam frame goes to (width, height) with LANCZOS first
    (qwen_realtime.py:239-243), then to the engine's cond size -- never 1184x896."""
    from PIL import Image
    cfg = stream.StreamConfig()
    rt = stream.QwenRealtimePipeline(cfg)
    rt.transformer = type("T", (), {"device": torch.device("cpu")})()
    rng = np.random.default_rng(0)
    frame = Image.fromarray(rng.integers(0, 255, (480, 640, 3), dtype=np.uint8))
    t = rt.frame_to_rgb(frame)
    ch, cw = cfg.cond_size
    assert t.dtype == torch.uint8 and tuple(t.shape) == (1, ch, cw, 3)
    exp = frame.resize((cfg.width, cfg.height), Image.LANCZOS).resize((cw, ch), Image.LANCZOS)
    assert np.array_equal(t[0].numpy(), np.asarray(exp))
    # numpy frames (OpenCV-style RGB arrays) take the same path
    assert torch.equal(rt.frame_to_rgb(np.asarray(frame)), t)
    # uint8 tensors must already be at the cond size
    assert torch.equal(rt.frame_to_rgb(t[0]), t)
    with pytest.raises(ValueError):
        rt.frame_to_rgb(torch.zeros(480, 640, 3, dtype=torch.uint8))


def test_prompt_cache_keys_on_reference_image():
    from PIL import Image
    c = stream.CachedConditions()
    c.prompt, c.prompt_embeds = "p", torch.zeros(1)
    assert c.is_valid("p") and not c.is_valid("q")
    a, b = Image.new("RGB", (8, 8), "red"), Image.new("RGB", (8, 8), "blue")
    assert not c.is_valid("p", a)
    c.reference_key = c.image_key(a)
    assert c.is_valid("p", Image.new("RGB", (8, 8), "red")) and not c.is_valid("p", b)
    # tensor images of any dtype (numpy has no bfloat16): keyed on shape, dtype and raw bytes
    tb = torch.arange(48, dtype=torch.float32).view(4, 4, 3).to(torch.bfloat16)
    k = c.image_key(tb)
    assert k == c.image_key(tb.clone()) and k != c.image_key(tb + 1) and k != c.image_key(tb.float())
    assert c.image_key(tb.view(2, 8, 3)) != k


def test_importing_the_package_leaves_the_environment_alone():
    """The HIP hardware-queue setting belongs to the launchers (bench.py, parallel.raise_hip_hw_queues),
    not to `import`: a fresh interpreter's environment is the same before and after the import."""
    import subprocess
    import sys
    code = ("import os; a = dict(os.environ); import qwen_image_edit_streamdiffusion_amd; "
            "import qwen_image_edit_streamdiffusion_amd.parallel as p; assert dict(os.environ) == a; "
            "assert p.raise_hip_hw_queues(8) and os.environ['GPU_MAX_HW_QUEUES'] == '8'")
    env = dict(os.environ, GPU_MAX_HW_QUEUES="4")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


def test_text_split_rule_and_per_linear_config():
    """Text-stream split-K counts (bench --text-splits): one count for all linears, a per-linear
    dict (names missing from it unsplit), or 0 / None = ops.splitk_splits, which depends on
    (N, K) only (so batched CFG == sequential) and always divides the K tiles."""
    m = QwenImageTransformer2DModel.__new__(QwenImageTransformer2DModel)
    D, F = 3072, 12288
    shapes = {"qkv": (3 * D, D), "out": (D, D), "up": (F, D), "down": (D, F)}
    for name, (N, K) in shapes.items():
        s = ops.splitk_splits(N, K)
        assert s >= 1 and (K * 2 // 128) % s == 0
        assert 2 * -(-N // 256) * s <= 256 or s == 1
        m.text_splits = 1
        assert m._txt_splits(name, N, K) == 1
        m.text_splits = None
        assert m._txt_splits(name, N, K) == s
        m.text_splits = {"down": 0, "up": 3}
        assert m._txt_splits(name, N, K) == {"down": s, "up": 3}.get(name, 1)
    assert [ops.splitk_splits(*shapes[n]) for n in ("qkv", "out", "up", "down")] == [3, 4, 2, 8]
