"""A second, independent statement of the DiT forward, written the way the upstream model is
written -- a tree of stock ``torch.nn`` modules (nn.Linear, nn.LayerNorm, nn.RMSNorm, nn.SiLU,
``F.scaled_dot_product_attention``, ``F.gelu(approximate="tanh")``, complex-number RoPE through
``torch.view_as_complex`` / ``torch.polar``) whose attribute names produce the diffusers
state_dict keys by themselves -- against the functional oracle (oracle/dit_ref.py), in fp32.

What this pins: every primitive of the oracle (softmax scale and axis, LayerNorm / RMSNorm
formula and eps placement, the GELU variant, the rotation convention of the rotary embedding, the
joint [text; image] order, the chunk order of the modulation vectors, scale-before-shift in
norm_out) to PyTorch's own implementation of that primitive, and the oracle's parameter names to a
module tree that ``load_state_dict(strict=True)`` accepts. What it cannot pin: that this tree is
diffusers' tree -- diffusers is not installed here, so that part stays a restatement.
"""
import math

import torch
import torch.nn.functional as F
from torch import nn

from oracle import dit_ref as R


class _GELUProj(nn.Module):  # FeedForward's first entry: Linear + tanh-GELU
    def __init__(self, d, f):
        super().__init__()
        self.proj = nn.Linear(d, f)

    def forward(self, x):
        return F.gelu(self.proj(x), approximate="tanh")


class _FeedForward(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.net = nn.ModuleList([_GELUProj(d, 4 * d), nn.Dropout(0.0), nn.Linear(4 * d, d)])

    def forward(self, x):
        for m in self.net:
            x = m(x)
        return x


class _Attention(nn.Module):
    def __init__(self, d, heads, dh, eps):
        super().__init__()
        self.heads = heads
        self.to_q, self.to_k, self.to_v = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)
        self.add_q_proj, self.add_k_proj, self.add_v_proj = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)
        self.norm_q, self.norm_k = nn.RMSNorm(dh, eps=eps), nn.RMSNorm(dh, eps=eps)
        self.norm_added_q, self.norm_added_k = nn.RMSNorm(dh, eps=eps), nn.RMSNorm(dh, eps=eps)
        self.to_out = nn.ModuleList([nn.Linear(d, d), nn.Dropout(0.0)])
        self.to_add_out = nn.Linear(d, d)

    @staticmethod
    def _rope(x, freqs):  # x [B, S, H, Dh], freqs complex [S, Dh/2]
        xc = torch.view_as_complex(x.float().reshape(*x.shape[:-1], -1, 2))
        return torch.view_as_real(xc * freqs[None, :, None, :]).flatten(3)

    def forward(self, img, txt, img_freqs, txt_freqs, attn_mask=None):
        B, S_txt = txt.shape[:2]
        sp = lambda t: t.unflatten(-1, (self.heads, -1))  # noqa: E731
        iq, ik, iv = sp(self.to_q(img)), sp(self.to_k(img)), sp(self.to_v(img))
        tq, tk, tv = sp(self.add_q_proj(txt)), sp(self.add_k_proj(txt)), sp(self.add_v_proj(txt))
        iq, ik = self._rope(self.norm_q(iq), img_freqs), self._rope(self.norm_k(ik), img_freqs)
        tq, tk = self._rope(self.norm_added_q(tq), txt_freqs), self._rope(self.norm_added_k(tk), txt_freqs)
        q, k, v = (torch.cat([a, b], 1).transpose(1, 2) for a, b in ((tq, iq), (tk, ik), (tv, iv)))
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=attn_mask, dropout_p=0.0, is_causal=False)
        o = o.transpose(1, 2).flatten(2)
        return self.to_out[0](o[:, S_txt:]), self.to_add_out(o[:, :S_txt])


class _Block(nn.Module):
    def __init__(self, d, heads, dh, eps):
        super().__init__()
        self.img_mod = nn.Sequential(nn.SiLU(), nn.Linear(d, 6 * d))
        self.txt_mod = nn.Sequential(nn.SiLU(), nn.Linear(d, 6 * d))
        self.norm = nn.LayerNorm(d, eps=eps, elementwise_affine=False)  # img_norm1/2, txt_norm1/2 (no parameters)
        self.attn = _Attention(d, heads, dh, eps)
        self.img_mlp, self.txt_mlp = _FeedForward(d), _FeedForward(d)

    @staticmethod
    def _modulate(x, mod):
        shift, scale, gate = mod.chunk(3, dim=-1)
        return x * (1 + scale.unsqueeze(1)) + shift.unsqueeze(1), gate.unsqueeze(1)

    def forward(self, img, txt, temb, img_freqs, txt_freqs, attn_mask):
        im1, im2 = self.img_mod(temb).chunk(2, dim=-1)
        tm1, tm2 = self.txt_mod(temb).chunk(2, dim=-1)
        ih, ig1 = self._modulate(self.norm(img), im1)
        th, tg1 = self._modulate(self.norm(txt), tm1)
        ia, ta = self.attn(ih, th, img_freqs, txt_freqs, attn_mask)
        img, txt = img + ig1 * ia, txt + tg1 * ta
        ih, ig2 = self._modulate(self.norm(img), im2)
        th, tg2 = self._modulate(self.norm(txt), tm2)
        return img + ig2 * self.img_mlp(ih), txt + tg2 * self.txt_mlp(th)


class _TimeEmbed(nn.Module):
    def __init__(self, d, tdim):
        super().__init__()
        self.timestep_embedder = nn.Module()
        self.timestep_embedder.linear_1 = nn.Linear(tdim, d)
        self.timestep_embedder.linear_2 = nn.Linear(d, d)
        self.tdim = tdim

    def forward(self, t):
        half = self.tdim // 2
        freqs = torch.exp(-math.log(10000.0) * torch.arange(half, dtype=torch.float32) / half)
        arg = 1000.0 * t.float()[:, None] * freqs[None, :]
        emb = torch.cat([torch.cos(arg), torch.sin(arg)], dim=-1)  # flip_sin_to_cos: cos first
        te = self.timestep_embedder
        return te.linear_2(F.silu(te.linear_1(emb)))


class TorchDiT(nn.Module):
    def __init__(self, cfg: R.DiTConfig):
        super().__init__()
        d, dh = cfg.inner_dim, cfg.attention_head_dim
        self.cfg = cfg
        self.img_in = nn.Linear(cfg.in_channels, d)
        self.txt_norm = nn.RMSNorm(cfg.joint_attention_dim, eps=cfg.eps)
        self.txt_in = nn.Linear(cfg.joint_attention_dim, d)
        self.time_text_embed = _TimeEmbed(d, cfg.timestep_dim)
        self.transformer_blocks = nn.ModuleList(
            [_Block(d, cfg.num_attention_heads, dh, cfg.eps) for _ in range(cfg.num_layers)])
        self.norm_out = nn.Module()
        self.norm_out.linear = nn.Linear(d, 2 * d)
        self.proj_out = nn.Linear(d, cfg.patch_size ** 2 * cfg.out_channels)

    def _freqs(self, img_shapes, txt_len):
        """Complex rotary factors from integer positions: image i at frame i, rows / columns
        centred around 0 (negative half first), text after the largest half extent."""
        axes = self.cfg.axes_dims_rope

        def cis(pos, dim):
            inv = 1.0 / (10000.0 ** (torch.arange(0, dim, 2, dtype=torch.float32) / dim))
            ang = pos.to(torch.float32)[:, None] * inv[None, :]
            return torch.polar(torch.ones_like(ang), ang)

        rows, off = [], 0
        for i, (f, h, w) in enumerate(img_shapes):
            fi = torch.arange(i, i + f).view(f, 1, 1).expand(f, h, w).reshape(-1)
            hi = (torch.arange(h) - (h - h // 2)).view(1, h, 1).expand(f, h, w).reshape(-1)
            wi = (torch.arange(w) - (w - w // 2)).view(1, 1, w).expand(f, h, w).reshape(-1)
            rows.append(torch.cat([cis(fi, axes[0]), cis(hi, axes[1]), cis(wi, axes[2])], dim=-1))
            off = max(off, h // 2, w // 2)
        tp = torch.arange(off, off + txt_len)
        return torch.cat(rows, 0), torch.cat([cis(tp, a) for a in axes], dim=-1)

    def forward(self, hidden_states, encoder_hidden_states, timestep, img_shapes, txt_seq_lens):
        B, S_txt = encoder_hidden_states.shape[:2]
        img = self.img_in(hidden_states.float())
        txt = self.txt_in(self.txt_norm(encoder_hidden_states.float()))
        temb = self.time_text_embed(timestep)
        img_freqs, txt_freqs = self._freqs(img_shapes, S_txt)
        mask = None
        if any(int(n) != S_txt for n in txt_seq_lens):
            valid = torch.arange(S_txt)[None, :] < torch.tensor([int(n) for n in txt_seq_lens])[:, None]
            valid = torch.cat([valid, torch.ones(B, img.shape[1], dtype=torch.bool)], dim=1)
            mask = valid[:, None, None, :]
        for blk in self.transformer_blocks:
            img, txt = blk(img, txt, temb, img_freqs, txt_freqs, mask)
        scale, shift = self.norm_out.linear(F.silu(temb)).chunk(2, dim=-1)  # scale first
        x = F.layer_norm(img, (img.shape[-1],), eps=self.cfg.eps) * (1 + scale[:, None]) + shift[:, None]
        return self.proj_out(x)


def _model_and_params(cfg, seed):
    params = R.random_params(cfg, seed=seed)
    m = TorchDiT(cfg).float()
    # the names the functional oracle uses are exactly this tree's state_dict keys
    res = m.load_state_dict({k: v.float() for k, v in params.items()}, strict=True)
    assert not res.missing_keys and not res.unexpected_keys
    assert set(m.state_dict()) == set(dict(R.param_shapes(cfg)))
    return m.eval(), params


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


def test_torch_module_tree_matches_functional_oracle_fp32():
    cfg = R.tiny_config()
    m, params = _model_and_params(cfg, seed=5)
    g = torch.Generator().manual_seed(6)
    shapes = [(1, 8, 6), (1, 4, 10)]  # non-square grids, two images: the centred h / w indices differ
    S_img = sum(f * h * w for f, h, w in shapes)
    hs = torch.randn(2, S_img, 64, generator=g).to(torch.bfloat16)
    enc = torch.randn(2, 14, cfg.joint_attention_dim, generator=g).to(torch.bfloat16)
    t = R.model_timestep(torch.tensor([1000.0, 455.6]))
    with torch.no_grad():
        for lens in ([14, 14], [14, 9]):  # unpadded, and a padded row with a key mask
            got = m(hs, enc, t, shapes, lens)
            ref = R.transformer_forward(params, cfg, hs, enc, t, shapes, lens, emulate_bf16=False)
            assert _rel(got, ref) <= 2e-5, (lens, _rel(got, ref))


def test_rope_complex_form_equals_oracle_rotation():
    cfg = R.tiny_config()
    m, _ = _model_and_params(cfg, seed=1)
    shapes = [(1, 6, 4), (1, 2, 8)]
    img_f, txt_f = m._freqs(shapes, 5)
    ip, tp = R.rope_phases(shapes, 5, cfg.axes_dims_rope)
    assert torch.allclose(torch.angle(img_f), torch.atan2(torch.sin(ip), torch.cos(ip)), atol=1e-6)
    assert torch.allclose(torch.angle(txt_f), torch.atan2(torch.sin(tp), torch.cos(tp)), atol=1e-6)
    x = torch.randn(1, ip.shape[0], 2, 128, generator=torch.Generator().manual_seed(2))
    a = _Attention._rope(x, img_f)
    b = R.apply_rope(x, ip, R._R(False))
    assert torch.allclose(a, b, atol=1e-5)


def test_bf16_emulation_stays_close_to_the_fp32_module_tree():
    """The rounding-point emulation (what the kernels are held to) is the fp32 tree plus bf16
    rounding noise, not a different function."""
    cfg = R.tiny_config()
    m, params = _model_and_params(cfg, seed=7)
    g = torch.Generator().manual_seed(8)
    shapes = [(1, 8, 8), (1, 8, 8)]
    hs = torch.randn(1, 128, 64, generator=g).to(torch.bfloat16)
    enc = torch.randn(1, 16, cfg.joint_attention_dim, generator=g).to(torch.bfloat16)
    t = R.model_timestep(torch.tensor([20.0]))
    with torch.no_grad():
        got = m(hs, enc, t, shapes, [16])
    ref = R.transformer_forward(params, cfg, hs, enc, t, shapes, [16], emulate_bf16=True)
    assert _rel(ref, got) <= 1.5e-2
