"""CPU checks of the oracle itself: closed-form known answers, invariants and
the committed golden fixtures (tests/golden/make_golden.py).

Parity vs the reference is unpinned (no reference vectors exist, diffusers is
absent); these pin the oracle by closed forms and invariants.
"""
import math
import os

import numpy as np
import pytest
import torch

from oracle import dit_ref as R
from oracle import int8_ref as Q8

BF16 = torch.bfloat16
GOLD = os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.npz")


def from_bits(a):
    return torch.from_numpy(a).view(BF16)


# ----------------------------------------------------------------------------- scheduler
def test_calculate_shift_closed_form():
    mu = R.calculate_shift(4096, R.SchedulerConfig())
    assert mu == pytest.approx(0.5 + 0.4 * (4096 - 256) / (8192 - 256), abs=1e-12)


@pytest.mark.parametrize("n,expected", [
    (2, [1.0, 0.02, 0.0]),
    (4, [1.0, 0.76671, 0.45561, 0.02, 0.0]),
])
def test_sigma_schedule_known_values(n, expected):
    s, t = R.sigma_schedule(n, 4096)
    assert np.allclose(s.numpy(), expected, atol=2e-5)
    assert torch.allclose(t, s[:-1] * 1000)


def test_sigma_schedule_hand_formula():
    # independent float64 restatement of time_shift + stretch
    mu = 0.5 + 0.4 * (4096 - 256) / 7936
    for n in (2, 3, 5, 8):
        sig = np.linspace(1.0, 1.0 / n, n)
        sh = math.exp(mu) / (math.exp(mu) + (1 / sig - 1))
        om = 1 - sh
        st = 1 - om / (om[-1] / 0.98)
        s, _ = R.sigma_schedule(n, 4096)
        assert np.allclose(s.numpy()[:-1], st, atol=1e-6)
        assert s[-1] == 0 and s[-2].item() == pytest.approx(0.02, abs=1e-6)


def test_model_timestep_bf16_rounding():
    t = R.model_timestep(torch.tensor([1000.0, 20.0]))
    assert t.dtype == BF16
    assert t.float().tolist() == [1.0, 0.02001953125]


def test_euler_step_semantics():
    x = torch.randn(8, 64).to(BF16)
    v = torch.randn(8, 64).to(BF16)
    assert torch.equal(R.euler_step(x, v, 0.5, 0.5), x)  # dt = 0
    y = R.euler_step(x, v, 1.0, 0.02)
    exp = (x.float() + (torch.tensor(-0.98) * v.float()).to(BF16).float()).to(BF16)
    assert torch.equal(y, exp)


def test_cfg_combine_invariants():
    c = torch.randn(4, 10, 64).to(BF16)
    u = torch.randn(4, 10, 64).to(BF16)
    o = R.cfg_combine(c, u, 4.0).float()
    # norm rescale: ||out|| == ||cond|| per token (to bf16 precision)
    assert torch.allclose(o.norm(dim=-1), c.float().norm(dim=-1), rtol=2e-2)
    # scale 1 returns cond direction exactly scaled back to its own norm
    o1 = R.cfg_combine(c, u, 1.0).float()
    assert torch.allclose(o1, c.float(), rtol=2e-2, atol=2e-2)


# ----------------------------------------------------------------------------- embeddings
def test_timestep_sinusoid_closed_form():
    e = R.timestep_sinusoid(torch.tensor([0.0, 1.0]), 256)
    assert torch.equal(e[0, :128], torch.ones(128)) and torch.equal(e[0, 128:], torch.zeros(128))
    k = torch.arange(128, dtype=torch.float64)
    arg = 1000.0 * torch.exp(-math.log(10000.0) * k / 128)
    assert torch.allclose(e[1, :128].double(), torch.cos(arg), atol=5e-4)
    assert torch.allclose(e[1, 128:].double(), torch.sin(arg), atol=5e-4)


def test_rope_layout_closed_form():
    ip, tp = R.rope_phases([(1, 64, 64), (1, 64, 64)], 216)
    assert ip.shape == (8192, 64) and tp.shape == (216, 64)
    inv16 = 10000.0 ** (-np.arange(0, 16, 2) / 16)
    inv56 = 10000.0 ** (-np.arange(0, 56, 2) / 56)
    # image 0, token (h=0, w=0) -> frame 0, h index -32, w index -32
    assert np.allclose(ip[0, :8], 0.0)
    assert np.allclose(ip[0, 8:36], -32 * inv56, rtol=1e-6)
    assert np.allclose(ip[0, 36:], -32 * inv56, rtol=1e-6)
    # image 1 (cond) uses frame index 1
    assert np.allclose(ip[4096, :8], 1 * inv16, rtol=1e-6)
    # token (h=40, w=7) -> h index 40-32=8, w index 7-32=-25
    tok = 40 * 64 + 7
    assert np.allclose(ip[tok, 8:36], 8 * inv56, rtol=1e-6)
    assert np.allclose(ip[tok, 36:], -25 * inv56, rtol=1e-6)
    # text token n -> position 32 + n on all three axes
    assert np.allclose(tp[5, :8], 37 * inv16, rtol=1e-6)
    assert np.allclose(tp[5, 8:36], 37 * inv56, rtol=1e-6)


def test_apply_rope_is_rotation():
    r = R._R(False)
    x = torch.randn(2, 10, 3, 128)
    ph = torch.randn(10, 64)
    y = R.apply_rope(x, ph, r)
    assert torch.allclose(y.norm(dim=-1), x.norm(dim=-1), rtol=1e-5)
    assert torch.allclose(R.apply_rope(x, torch.zeros(10, 64), r), x)


def test_pack_unpack_roundtrip_and_layout():
    x = torch.randn(2, 16, 1, 8, 12)
    p = R.pack_latents(x)
    assert p.shape == (2, 24, 64)
    # token (i=1, j=2), channel c=3, sub-pixel (di=1, dj=0)
    assert p[1, 1 * 6 + 2, 3 * 4 + 2] == x[1, 3, 0, 3, 4]
    assert torch.equal(R.unpack_latents(p, 8, 12), x)
    # diffusers prepare_latents layout (B, 1, C, H, W) packs identically
    assert torch.equal(R.pack_latents(x.permute(0, 2, 1, 3, 4)), p)


# ----------------------------------------------------------------------------- attention / model
def test_attention_masking_equals_truncation():
    r = R._R(False)
    q, k, v = (torch.randn(1, 20, 2, 128) for _ in range(3))
    valid = torch.ones(1, 20, dtype=torch.bool)
    valid[0, 15:] = False
    a = R.joint_attention(q, k, v, valid, r)
    b = R.joint_attention(q, k[:, :15], v[:, :15], None, r)
    assert torch.allclose(a, b, atol=1e-6)


def test_batched_padded_text_equals_unbatched():
    """Key masking makes a padded batch row equal to running it alone
    (the batched-CFG invariant)."""
    cfg = R.tiny_config()
    p = R.random_params(cfg, seed=3)
    g = torch.Generator().manual_seed(0)
    shapes = [(1, 4, 4), (1, 4, 4)]
    hs = torch.randn(2, 32, 64, generator=g).to(BF16)
    enc = torch.randn(2, 12, cfg.joint_attention_dim, generator=g).to(BF16)
    t = R.model_timestep(torch.tensor([1000.0, 1000.0]))
    both = R.transformer_forward(p, cfg, hs, enc, t, shapes, [12, 7], emulate_bf16=False)
    alone = R.transformer_forward(p, cfg, hs[1:], enc[1:, :7], t[1:], shapes, [7], emulate_bf16=False)
    assert torch.allclose(both[1:], alone, atol=1e-5, rtol=1e-4)


def test_flops_formula():
    f = R.flops_per_forward(8192, 216)
    assert f / 1e12 == pytest.approx(166.41, abs=0.05)  # per B=1 forward at 1024^2, S_txt = 216


# ----------------------------------------------------------------------------- int8
def test_quantize_rows_known_answer():
    x = np.array([[127.0, -63.5, 0.5, -0.5, 1.5, 2.5, 0.0, 63.5],
                  [0, 0, 0, 0, 0, 0, 0, 0]], dtype=np.float32)
    q, s = Q8.quantize_rows(x)
    # 127/127 = 1 -> rint: half to even
    assert q[0].tolist() == [127, -64, 0, 0, 2, 2, 0, 64]
    assert s[0] == np.float32(1.0) and s[1] == np.float32(1.0) and (q[1] == 0).all()


def test_int8_gemm_exact_integer():
    g = np.random.default_rng(0)
    a = g.integers(-127, 128, (5, 256)).astype(np.int8)
    w = g.integers(-127, 128, (3, 256)).astype(np.int8)
    acc = Q8.int8_gemm_acc(a, w)
    assert np.array_equal(acc, (a.astype(np.int64) @ w.astype(np.int64).T))


def test_int8_linear_error_vs_fp32():
    g = np.random.default_rng(1)
    x = g.standard_normal((64, 512)).astype(np.float32)
    w = (g.standard_normal((128, 512)) * 0.02).astype(np.float32)
    y = Q8.int8_linear(x, w)
    ref = x @ w.T
    assert np.linalg.norm(y - ref) / np.linalg.norm(ref) < 2e-2


# ----------------------------------------------------------------------------- goldens
@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def test_golden_forward(gold):
    cfg = R.tiny_config()
    params = R.random_params(cfg, seed=0)
    y = R.transformer_forward(params, cfg, from_bits(gold["fwd_hidden_states"]),
                              from_bits(gold["fwd_encoder_hidden_states"]), from_bits(gold["fwd_timestep"]),
                              [(1, 8, 8), (1, 8, 8)], [16, 11])
    assert torch.equal(y.to(BF16), from_bits(gold["fwd_out"]))


def test_golden_small_ops(gold):
    for n in (2, 3, 4, 8):
        s, _ = R.sigma_schedule(n, 4096)
        assert np.array_equal(s.numpy(), gold[f"sigmas_{n}_4096"])
    e = R.timestep_sinusoid(torch.tensor([1.0, 0.02001953125, 0.5]), 256).numpy()
    assert np.allclose(e, gold["timestep_emb"], atol=1e-6)
    ip, tp = R.rope_phases([(1, 4, 6), (1, 4, 4)], 5)
    assert np.array_equal(ip.numpy(), gold["rope_img"]) and np.array_equal(tp.numpy(), gold["rope_txt"])
    q, s = Q8.quantize_rows(gold["q8_x"])
    assert np.array_equal(q, gold["q8_q"]) and np.array_equal(s, gold["q8_s"])
    c = R.cfg_combine(from_bits(gold["cfg_c"]), from_bits(gold["cfg_u"]), 4.0)
    assert torch.equal(c, from_bits(gold["cfg_out"]))
    y = R.euler_step(from_bits(gold["euler_x"]), from_bits(gold["euler_v"]), 1.0, 0.02)
    assert torch.equal(y, from_bits(gold["euler_out"]))
