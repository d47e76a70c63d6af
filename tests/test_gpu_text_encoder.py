"""Prompt encoder language model on the GPU: the Qwen2.5-VL kernels of vl.hip
and the whole QwenVLTextModel vs transformers' Qwen2_5_VLTextModel (oracle/vl_ref.py; random
weights of reduced width, bf16-representable, fp32 eager oracle).

Tolerances:
  * embed_rows, rope_half (bf16 tables): exact vs torch restatements with the same bf16 rounding
    points; silu_mul, rope_half (fp32 tables), erf GELU: <= 1 bf16 ulp on < 1% of entries
  * causal softmax rows: rel-L2 <= 4e-3, masked entries exactly 0
  * whole text model (2 layers, S = 77 / 128, padded to multiples of 64): rel-L2 <= 2e-2 on the
    last hidden state (every projection re-rounds to bf16; the oracle stays fp32)
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16
DEV = "cuda"


def _ops():
    from qwen_image_edit_streamdiffusion_amd import ops
    return ops


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm()).item()


def test_embed_rows_exact():
    ops = _ops()
    g = torch.Generator().manual_seed(0)
    table = torch.randn(1000, 256, generator=g).to(BF16)
    ids = torch.randint(0, 1000, (77,), generator=g, dtype=torch.int32)
    out = ops.embed_rows(table.to(DEV), ids.to(DEV))
    assert torch.equal(out.cpu(), table[ids.long()])


def test_silu_mul_exact():
    ops = _ops()
    g = torch.Generator().manual_seed(1)
    gu = (3 * torch.randn(65, 2 * 512, generator=g)).to(BF16)
    out = ops.silu_mul(gu.to(DEV))
    gate, up = gu[:, :512].float(), gu[:, 512:].float()
    want = (torch.nn.functional.silu(gate).to(BF16).float() * up).to(BF16)
    diff = (out.cpu().float() - want.float()).abs()
    # expf vs torch's silu can differ in the last fp32 bit: allow one bf16 ulp on a handful of entries
    assert (diff <= want.float().abs() * 2 ** -7 + 1e-30).all() and (diff > 0).float().mean() < 1e-2


def test_rope_half_matches_rotate_half():
    ops = _ops()
    from qwen_image_edit_streamdiffusion_amd.text_encoder import TextEncoderConfig, mrope_tables
    cfg = TextEncoderConfig(hidden_size=512, num_attention_heads=4, num_key_value_heads=2)
    S, Dh = 70, 128
    g = torch.Generator().manual_seed(2)
    x = torch.randn(S, 9 * Dh, generator=g).to(BF16)  # 4 q + 2 k + 2 v heads and one spare
    pos = torch.stack([torch.arange(S), torch.arange(S) // 3, torch.arange(S) % 7])
    cos, sin = mrope_tables(cfg, pos)
    xd = x.to(DEV)
    ops.rope_half(xd, 0, 6, Dh, cos.to(DEV), sin.to(DEV))
    q = x[:, :6 * Dh].view(S, 6, Dh)
    rot = torch.cat([-q[..., 64:], q[..., :64]], -1)
    want = ((q * cos[:, None]).to(BF16) + (rot * sin[:, None]).to(BF16)).view(S, -1)
    assert torch.equal(xd.cpu()[:, :6 * Dh], want)
    assert torch.equal(xd.cpu()[:, 6 * Dh:], x[:, 6 * Dh:])


def test_causal_softmax_rows():
    ops = _ops()
    g = torch.Generator().manual_seed(3)
    R = 96
    s = 4 * torch.randn(R, R, generator=g)
    p = torch.empty(R, 128, dtype=BF16, device=DEV)
    ops.softmax_rows(s.to(DEV), 0.125, out=p, causal=True)
    mask = torch.ones(R, R).triu(1).bool()
    want = torch.softmax((0.125 * s).masked_fill(mask, float("-inf")), -1)
    got = p.cpu().float()
    assert _rel(got[:, :R], want) <= 4e-3
    assert (got[:, :R][mask] == 0).all() and (got[:, R:] == 0).all()


@pytest.mark.parametrize("S", [77, 128])
def test_text_model_vs_transformers(S):
    from oracle import vl_ref as VL
    from qwen_image_edit_streamdiffusion_amd.text_encoder import QwenVLTextModel, TextEncoderConfig
    m, sd = VL.tiny_text_model(0)
    cfg = TextEncoderConfig(vocab_size=1000, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                            num_attention_heads=2, num_key_value_heads=1)
    te = QwenVLTextModel(cfg, DEV).load_state_dict(sd)
    ids = torch.randint(0, 1000, (S,), generator=torch.Generator().manual_seed(S))
    want = VL.text_forward(m, input_ids=ids)
    got = te(ids)
    assert got.shape == (S, 256) and got.dtype == BF16
    assert _rel(got, want) <= 2e-2


def test_text_model_3d_positions_and_embeds():
    """The condition-image path: inputs_embeds rows (vision embeddings spliced in) with distinct
    temporal / height / width positions on a block of tokens, as get_rope_index builds them."""
    from oracle import vl_ref as VL
    from qwen_image_edit_streamdiffusion_amd.text_encoder import QwenVLTextModel, TextEncoderConfig
    m, sd = VL.tiny_text_model(4)
    cfg = TextEncoderConfig(vocab_size=1000, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                            num_attention_heads=2, num_key_value_heads=1)
    te = QwenVLTextModel(cfg, DEV).load_state_dict({"model.language_model." + k: v for k, v in sd.items()})
    S, g = 90, torch.Generator().manual_seed(5)
    emb = (0.5 * torch.randn(S, 256, generator=g)).to(BF16)
    pos = torch.arange(S).view(1, S).repeat(3, 1)
    grid = torch.arange(36)  # a 6x6 image block at tokens 10..45: t fixed, h / w on the grid
    pos[0, 10:46] = 10
    pos[1, 10:46] = 10 + grid // 6
    pos[2, 10:46] = 10 + grid % 6
    pos[:, 46:] = torch.arange(S - 46) + 16
    want = VL.text_forward(m, inputs_embeds=emb, position_ids=pos)
    got = te(inputs_embeds=emb.to(DEV), position_ids=pos)
    assert _rel(got, want) <= 2e-2


def _vision_cfg():
    from qwen_image_edit_streamdiffusion_amd.vision import VisionConfig
    return VisionConfig(depth=4, hidden_size=320, intermediate_size=200, num_heads=4, out_hidden_size=256,
                        fullatt_block_indexes=(1, 3))


def test_rope_half_fp32_tables_slots():
    """The vision form: fp32 tables, one rounding, 80-wide heads in 128-wide slots."""
    ops = _ops()
    g = torch.Generator().manual_seed(6)
    S, Dh, SL = 50, 80, 128
    x = torch.randn(S, 4 * SL, generator=g).to(BF16)
    ang = torch.randn(S, Dh // 2, generator=g)
    cos, sin = torch.cat([ang.cos(), ang.cos()], -1), torch.cat([ang.sin(), ang.sin()], -1)
    xd = x.to(DEV)
    ops.rope_half(xd, 0, 3, Dh, cos.to(DEV), sin.to(DEV), head_stride=SL)
    q = x.view(S, 4, SL)[:, :3, :Dh].float()
    rot = torch.cat([-q[..., 40:], q[..., :40]], -1)
    want = (q * cos[:, None] + rot * sin[:, None]).to(BF16)
    got = xd.cpu().view(S, 4, SL)
    d = (got[:, :3, :Dh].float() - want.float()).abs()
    frac = (d > 0).float().mean().item()
    # fp32 products / sum then one rounding; v_mul/v_add vs the CPU's vectorised ops may differ in
    # the last fp32 bit, which moves a rounding tie by one bf16 ulp on a few entries
    assert (d <= want.float().abs() * 2 ** -7 + 1e-30).all() and frac < 1e-2, (frac, d.max().item())
    assert torch.equal(got[:, :3, Dh:], x.view(S, 4, SL)[:, :3, Dh:]) and torch.equal(got[:, 3], x.view(S, 4, SL)[:, 3])


def test_ranged_softmax_and_gelu_erf():
    ops = _ops()
    g = torch.Generator().manual_seed(7)
    R = 70
    s = 3 * torch.randn(R, 72, generator=g)
    cu = [0, 12, 20, 44, 45, 70]  # ragged segments, one of length 1, one unaligned start
    rng = torch.zeros(R, 2, dtype=torch.int32)
    for a, b in zip(cu[:-1], cu[1:]):
        rng[a:b, 0], rng[a:b, 1] = a, b
    p = torch.full((R, 128), float("nan"), device=DEV).to(BF16)
    ops.softmax_rows(s.to(DEV), 0.2, out=p, ranges=rng.to(DEV))
    mask = torch.ones(R, 72, dtype=torch.bool)
    for a, b in zip(cu[:-1], cu[1:]):
        mask[a:b, a:b] = False
    want = torch.softmax((0.2 * s).masked_fill(mask, float("-inf")), -1)
    got = p.cpu().float()
    assert _rel(got[:, :72], want) <= 4e-3 and (got[:, :72][mask] == 0).all() and (got[:, 72:] == 0).all()
    # head-batched: three heads' score blocks share the per-row ranges (period R)
    s3 = 3 * torch.randn(3 * R, 72, generator=g)
    p3 = torch.empty(3 * R, 72, dtype=BF16, device=DEV)
    ops.softmax_rows(s3.to(DEV), 0.2, out=p3, ranges=rng.to(DEV))
    want3 = torch.softmax((0.2 * s3).masked_fill(mask.repeat(3, 1), float("-inf")), -1)
    assert _rel(p3, want3) <= 4e-3
    x = (4 * torch.randn(33, 256, generator=g)).to(BF16)
    y = ops.gelu_erf_(x.to(DEV).clone()).cpu()
    want = torch.nn.functional.gelu(x.float()).to(BF16)
    assert ((y.float() - want.float()).abs() <= want.float().abs() * 2 ** -7 + 1e-6).all()


@pytest.mark.parametrize("grid", [[(1, 20, 28)], [(1, 16, 16), (1, 8, 12)]])
def test_vision_tower_vs_transformers(grid):
    """Patch embed, window permutation, ragged windows, full-attention blocks per image, 2x2 merger."""
    from oracle import vl_ref as VL
    from qwen_image_edit_streamdiffusion_amd.vision import QwenVLVisionTower
    m, sd = VL.tiny_vl_model(1)
    tower = QwenVLVisionTower(_vision_cfg(), DEV).load_state_dict(sd)
    S = sum(t * h * w for t, h, w in grid)
    pv = torch.randn(S, 1176, generator=torch.Generator().manual_seed(S))
    want = VL.vision_forward(m, pv, torch.tensor(grid))
    got = tower(pv, grid)
    assert got.shape == want.shape
    assert _rel(got, want) <= 2e-2


def test_vl_encoder_prompt_with_image_vs_transformers():
    """Whole Qwen2_5_VLModel: image rows scattered over <|image_pad|>, 3-D positions, hidden_states[-1]."""
    from oracle import vl_ref as VL
    from qwen_image_edit_streamdiffusion_amd.text_encoder import QwenVLEncoder, TextEncoderConfig
    m, sd = VL.tiny_vl_model(2)
    enc = QwenVLEncoder(TextEncoderConfig(vocab_size=1000, hidden_size=256, intermediate_size=512,
                                          num_hidden_layers=2, num_attention_heads=2, num_key_value_heads=1),
                        _vision_cfg(), DEV, image_token_id=990).load_state_dict(sd)
    g = torch.Generator().manual_seed(8)
    grid = torch.tensor([[1, 20, 28]])
    pv = torch.randn(560, 1176, generator=g)
    ids = torch.cat([torch.randint(0, 900, (70,), generator=g), torch.tensor([992]), torch.full((140,), 990),
                     torch.tensor([993]), torch.randint(0, 900, (25,), generator=g)])
    want, _ = VL.vl_forward(m, ids, pv, grid)
    got = enc(ids, pv, grid)
    assert got.shape == want.shape and _rel(got, want) <= 2e-2
    # text-only prompt through the same encoder (the negative / empty-image case)
    want_t, _ = VL.vl_forward(m, ids[:70])
    assert _rel(enc(ids[:70]), want_t) <= 2e-2


@pytest.mark.parametrize("group", [1, 7])
def test_matmul_heads_batched(group):
    """Head-batched products on strided column slices (GQA: the w operand advances per group)."""
    ops = _ops()
    g = torch.Generator().manual_seed(9)
    S, Dh, H = 192, 128, 14  # S is the P.V reduction length: a multiple of 64 (the models pad)
    Hk = H // group
    qkv = torch.randn(S, (H + 2 * Hk) * Dh, generator=g).to(BF16).to(DEV)
    s = torch.empty(H * S, S, dtype=torch.float32, device=DEV)
    ops.matmul_heads(qkv[:, :Dh], Dh, qkv[:, H * Dh:(H + 1) * Dh], Dh, s[:S], S * S, H, group=group)
    q = qkv[:, :H * Dh].float().cpu().view(S, H, Dh)
    k = qkv[:, H * Dh:(H + Hk) * Dh].float().cpu().view(S, Hk, Dh)
    want = torch.einsum("shd,thd->hst", q, k.repeat_interleave(group, 1)).reshape(H * S, S)
    assert _rel(s, want) <= 1e-5
    p = torch.randn(H * S, S, generator=g).to(BF16).to(DEV)
    vt = torch.randn(Hk * Dh, S, generator=g).to(BF16).to(DEV)
    out = torch.empty(S, H * Dh, dtype=BF16, device=DEV)
    bias = torch.zeros(Dh, dtype=BF16, device=DEV)
    ops.matmul_heads(p[:S], S * S, vt[:Dh], Dh * S, out[:, :Dh], Dh, H, group=group, bias=bias)
    pv = torch.einsum("hst,hdt->shd", p.float().cpu().view(H, S, S),
                      vt.float().cpu().view(Hk, Dh, S).repeat_interleave(group, 0)).reshape(S, H * Dh)
    assert _rel(out, pv) <= 4e-3
    with pytest.raises(ValueError):  # the last head would run past the buffer
        ops.matmul_heads(qkv[:, :Dh], Dh, qkv[:, H * Dh:(H + 1) * Dh], Dh, s[:S], S * S, H + 1, group=group)


def test_encoder_linears_splitk():
    """The encoders' split-K projections (plain and residual) vs fp32 torch on the same operands."""
    from qwen_image_edit_streamdiffusion_amd.text_encoder import EncoderLinears, encoder_splits
    g = torch.Generator().manual_seed(10)
    M, N, K = 320, 512, 2048
    assert encoder_splits(M, N, K) > 1
    x = torch.randn(M, K, generator=g).to(BF16)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(BF16)
    b = (0.1 * torch.randn(N, generator=g)).to(BF16)
    lin = EncoderLinears(torch.device(DEV))
    out = lin.linear(x.to(DEV), w.to(DEV), b.to(DEV), torch.empty(M, N, dtype=BF16, device=DEV))
    want = x.float() @ w.float().T + b.float()
    assert _rel(out, want) <= 4e-3
    r = torch.randn(M, N, generator=g).to(BF16)
    rd = r.to(DEV)
    lin.residual(x.to(DEV), w.to(DEV), b.to(DEV), torch.ones(1, N, dtype=BF16, device=DEV), rd)
    assert _rel(rd, r.float() + want) <= 4e-3


def test_pipeline_prompt_hook_end_to_end():
    """pipe(image=PIL, prompt=str) through QwenImageEditPromptEncoder (tiny Qwen2.5-VL on the HIP
    path behind a stub processor) == pipe(prompt_embeds=hook(prompt, image)); the hook drops the
    first 64 tokens of the encoder's hidden states."""
    from PIL import Image
    from oracle import dit_ref as R
    from oracle import vl_ref as VL
    from qwen_image_edit_streamdiffusion_amd import QwenImageEditPlusPipeline, QwenImageTransformer2DModel
    from qwen_image_edit_streamdiffusion_amd.text_encoder import (QwenImageEditPromptEncoder, QwenVLEncoder,
                                                                  TextEncoderConfig)
    from qwen_image_edit_streamdiffusion_amd.vision import VisionConfig
    from qwen_image_edit_streamdiffusion_amd.vae import QwenImageVAEDecoder, QwenImageVAEEncoder, VAEConfig
    cfg = R.tiny_config()
    _, sd = VL.tiny_vl_model(5, text_hidden=cfg.joint_attention_dim, text_heads=1)
    enc = QwenVLEncoder(TextEncoderConfig(vocab_size=1000, hidden_size=cfg.joint_attention_dim, intermediate_size=512,
                                          num_hidden_layers=2, num_attention_heads=1, num_key_value_heads=1),
                        VisionConfig(depth=4, hidden_size=320, intermediate_size=200, num_heads=4,
                                     out_hidden_size=cfg.joint_attention_dim, fullatt_block_indexes=(1, 3)),
                        DEV, image_token_id=990).load_state_dict(sd)
    g = torch.Generator().manual_seed(31)
    ids = torch.cat([torch.randint(0, 900, (70,), generator=g), torch.tensor([992]), torch.full((16,), 990),
                     torch.tensor([993]), torch.randint(0, 900, (12,), generator=g)])
    pv = torch.randn(64, 1176, generator=g)
    seen = []

    class Proc:  # the processor's contract: input_ids, pixel_values, image_grid_thw
        def __call__(self, text, images=None, return_tensors=None):
            seen.append((text, images))
            return {"input_ids": ids.view(1, -1), "attention_mask": torch.ones(1, ids.numel(), dtype=torch.long),
                    "pixel_values": pv, "image_grid_thw": torch.tensor([[1, 8, 8]])}

    hook = QwenImageEditPromptEncoder(enc, Proc())
    e, msk = hook("make it red", Image.new("RGB", (640, 480)))
    want = enc(ids, pv, torch.tensor([[1, 8, 8]]))[64:]
    assert e.shape == (1, ids.numel() - 64, cfg.joint_attention_dim) and torch.equal(e[0], want)
    assert seen[0][1][0].size == (448, 320)  # condition image resized to the 384^2 area
    m = QwenImageTransformer2DModel(num_layers=cfg.num_layers, num_attention_heads=cfg.num_attention_heads,
                                    joint_attention_dim=cfg.joint_attention_dim, device=DEV)
    m.load_diffusers_state_dict(R.random_params(cfg, seed=0))
    pipe = QwenImageEditPlusPipeline(m, prompt_encoder=hook)
    pipe.vae = QwenImageVAEDecoder(VAEConfig(base_dim=16), DEV).random_init_(7)
    pipe.vae_encoder = QwenImageVAEEncoder(VAEConfig(base_dim=16), DEV).random_init_(8)
    im = Image.fromarray(torch.randint(0, 256, (256, 256, 3), generator=g, dtype=torch.uint8).numpy())
    kw = dict(num_inference_steps=2, height=128, width=128, output_type="uint8")
    a = pipe(image=im, prompt="make it red", generator=torch.Generator().manual_seed(42), **kw).images
    b = pipe(image=im, prompt_embeds=e, prompt_embeds_mask=msk, generator=torch.Generator().manual_seed(42), **kw).images
    assert a.shape == (1, 128, 128, 3) and torch.equal(a, b)


def test_vl_encoder_vision_cache():
    """Same condition image, new prompt: the vision tower runs once (VLM cache) and the result
    equals the uncached encoder's."""
    from oracle import vl_ref as VL
    from qwen_image_edit_streamdiffusion_amd.text_encoder import QwenVLEncoder, TextEncoderConfig
    _, sd = VL.tiny_vl_model(2)
    tc = TextEncoderConfig(vocab_size=1000, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                           num_attention_heads=2, num_key_value_heads=1)
    enc = QwenVLEncoder(tc, _vision_cfg(), DEV, image_token_id=990).load_state_dict(sd)
    ref = QwenVLEncoder(tc, _vision_cfg(), DEV, image_token_id=990, vision_cache_size=0).load_state_dict(sd)
    runs = []
    tower = enc.vision.forward
    enc.vision.forward = lambda *a, **k: runs.append(1) or tower(*a, **k)
    g = torch.Generator().manual_seed(12)
    grid = torch.tensor([[1, 8, 8]])
    pv = torch.randn(64, 1176, generator=g)
    for n in (30, 41):
        ids = torch.cat([torch.randint(0, 900, (n,), generator=g), torch.full((16,), 990), torch.arange(5)])
        got = enc(ids, pv, grid)
        assert torch.equal(got, ref(ids, pv, grid))
    assert len(enc.vision_cache) == 1 and len(runs) == 1


def test_vl_encoder_full_width_one_layer():
    """Qwen2.5-VL-7B widths (text 3584 / 28 heads / 4 kv heads / SwiGLU 18944; vision 1280 / 16 heads
    of 80 / SwiGLU 3420 / merger 5120 -> 3584) with one text layer and two vision blocks (one window,
    one full), on a 392^2 condition image (28 x 28 patches) inside a 300-token prompt: the real GQA
    group of 7, the real head-slot padding and the real window raggedness vs transformers."""
    from oracle import vl_ref as VL
    from qwen_image_edit_streamdiffusion_amd.text_encoder import QwenVLEncoder, TextEncoderConfig
    from qwen_image_edit_streamdiffusion_amd.vision import VisionConfig
    m, sd = VL.tiny_vl_model(9, text_hidden=3584, vis_hidden=1280, vis_heads=16, vis_intermediate=3420, depth=2,
                             fullatt=(1,), text_heads=28, text_kv_heads=4, text_layers=1, text_intermediate=18944)
    enc = QwenVLEncoder(TextEncoderConfig(vocab_size=1000, hidden_size=3584, intermediate_size=18944,
                                          num_hidden_layers=1, num_attention_heads=28, num_key_value_heads=4),
                        VisionConfig(depth=2, fullatt_block_indexes=(1,)), DEV, image_token_id=990).load_state_dict(sd)
    g = torch.Generator().manual_seed(13)
    grid = torch.tensor([[1, 28, 28]])
    pv = torch.randn(784, 1176, generator=g)
    ids = torch.cat([torch.randint(0, 900, (70,), generator=g), torch.tensor([992]), torch.full((196,), 990),
                     torch.tensor([993]), torch.randint(0, 900, (32,), generator=g)])
    want, _ = VL.vl_forward(m, ids, pv, grid)
    got = enc(ids, pv, grid)
    assert got.shape == want.shape == (300, 3584)
    assert _rel(got, want) <= 2e-2
