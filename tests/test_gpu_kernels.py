"""Per-kernel parity: every libqie entry point vs the CPU oracle (or, for the
floating-point contractions, the oracle's fp32 math with the reference's bf16
rounding points).  Runs through the C ABI on the GPU.

Tolerances (bf16 storage, fp32 accumulation; the HIP kernels sum in a
different order than the CPU, so results may differ by the last bf16 bit):
  * GEMM / GEMV / norms:   rel-L2 <= 4e-3 and max |diff| <= 2 bf16 ulps of the
                           tensor's max magnitude (2 * 2^-8 * max|ref|)
  * attention:             rel-L2 <= 1e-2 vs fp32 softmax (P is rounded to bf16
                           before P.V, as in the reference's flash SDPA)
  * Euler step, pack/unpack, int8 quantisation: bit-exact
  * int8 GEMM:             within 1 bf16 ulp of the exact-integer oracle
"""
import math

import numpy as np
import pytest
import torch

from oracle import dit_ref as R
from oracle import int8_ref as Q8

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


RB = R._R(True)
_R_F32 = R._R(False)  # no rounding: the kernel rounds the rotated (and q-scaled) value once


@pytest.mark.parametrize("M,N,K", [(300, 384, 192), (2000, 2304, 128), (4300, 3072, 256),
                                   (4096, 4096, 64), (17, 512, 3072)])
@pytest.mark.parametrize("act", [0, 1])
def test_linear(dev, M, N, K, act):
    ops = _ops()
    x, w, b = rnd((M, K), dev, 1.0, 1), rnd((N, K), dev, 0.05, 2), rnd((N,), dev, 0.1, 3)
    y = ops.linear(x, w, b, act=act)
    ref = R.linear(x.cpu(), w.cpu(), b.cpu(), RB)
    if act:
        ref = R.gelu_tanh(ref, RB)
    close(y, ref)


def test_linear_strided_input(dev):
    ops = _ops()
    big = rnd((512, 384), dev, 1.0, 4)
    x = big[:, 128:]  # row stride 384, K = 256
    w, b = rnd((256, 256), dev, 0.05, 5), rnd((256,), dev, 0.1, 6)
    close(ops.linear(x, w, b), R.linear(x.cpu(), w.cpu(), b.cpu(), RB))


@pytest.mark.parametrize("M,N,K", [(1, 18432, 3072), (2, 18432, 3072), (2, 6144, 3072), (4, 3072, 256), (9, 512, 1024),
                                   (2, 100, 1000), (3, 37, 4168)])
def test_gemv(dev, M, N, K):
    ops = _ops()
    x, w, b = rnd((M, K), dev, 1.0, 7), rnd((N, K), dev, 0.02, 8), rnd((N,), dev, 0.02, 9)
    close(ops.gemv(x, w, b), R.linear(x.cpu(), w.cpu(), b.cpu(), RB))


@pytest.mark.parametrize("B,rpb,N,K", [(2, 300, 512, 256), (2, 4096, 3072, 512), (3, 40, 256, 1024)])
def test_gated_residual(dev, B, rpb, N, K):
    ops = _ops()
    M = B * rpb
    x, w, b = rnd((M, K), dev, 1.0, 10), rnd((N, K), dev, 0.05, 11), rnd((N,), dev, 0.1, 12)
    mods = rnd((B, 6 * N), dev, 0.5, 13)
    gate = mods[:, 2 * N:3 * N]
    resid = rnd((M, N), dev, 1.0, 14)
    ref = R.gated_residual(resid.cpu().float().view(B, rpb, N), gate.cpu(),
                           R.linear(x.cpu(), w.cpu(), b.cpu(), RB).view(B, rpb, N), RB).view(M, N)
    ops.linear_gated_residual(x, w, b, gate, rpb, resid)
    close(resid, ref)


def test_qkv_scatter(dev):
    ops = _ops()
    B, H, Dh, rpb, s_pad, off, K = 2, 2, 128, 200, 512, 300, 256
    x, w, b = rnd((B * rpb, K), dev, 1.0, 15), rnd((3 * H * Dh, K), dev, 0.05, 16), rnd((3 * H * Dh,), dev, 0.1, 17)
    qkv = torch.zeros(3, B, H, s_pad, Dh, dtype=BF16, device=dev)
    ops.linear_qkv(x, w, b, qkv, rpb, off)
    ref = R.linear(x.cpu(), w.cpu(), b.cpu(), RB).view(B, rpb, 3, H, Dh).permute(2, 0, 3, 1, 4)
    close(qkv[:, :, :, off:off + rpb].cpu(), ref)
    assert (qkv[:, :, :, :off] == 0).all() and (qkv[:, :, :, off + rpb:] == 0).all()


@pytest.mark.parametrize("B,rpb,D", [(2, 100, 3072), (1, 33, 256), (3, 7, 1024)])
def test_layernorm_modulate(dev, B, rpb, D):
    ops = _ops()
    x = rnd((B * rpb, D), dev, 2.0, 18)
    mods = rnd((B, 6 * D), dev, 0.5, 19)
    y = ops.layernorm_modulate(x, mods[:, :D], mods[:, D:2 * D], rpb)
    xc = x.cpu().float().view(B, rpb, D)
    ref = R.modulate(R.layer_norm(xc, 1e-6, RB), mods.cpu()[:, :D], mods.cpu()[:, D:2 * D], RB)
    close(y, ref.view(B * rpb, D))


def test_layernorm_modulate_i8_matches_quantized_bf16(dev):
    ops = _ops()
    B, rpb, D = 2, 64, 3072
    x = rnd((B * rpb, D), dev, 2.0, 20)
    mods = rnd((B, 6 * D), dev, 0.5, 21)
    y = ops.layernorm_modulate(x, mods[:, :D], mods[:, D:2 * D], rpb)
    q = torch.empty(B * rpb, D, dtype=torch.int8, device=dev)
    s = torch.empty(B * rpb, dtype=torch.float32, device=dev)
    ops.layernorm_modulate_i8(x, mods[:, :D], mods[:, D:2 * D], rpb, q, s)
    qr, sr = Q8.quantize_rows(y.float().cpu().numpy())
    assert np.array_equal(q.cpu().numpy(), qr)
    assert np.array_equal(s.cpu().numpy(), sr)


@pytest.mark.parametrize("R_,D", [(64, 3584), (5, 128), (300, 1024)])
def test_rmsnorm(dev, R_, D):
    ops = _ops()
    x, w = rnd((R_, D), dev, 3.0, 22), (1 + rnd((D,), dev, 0.02, 23).float()).to(BF16)
    close(ops.rmsnorm(x, w), R.rms_norm(x.cpu(), w.cpu(), 1e-6, RB))


@pytest.mark.parametrize("q_scale", [1.0, 1.4426950408889634 / math.sqrt(128)])
def test_qk_norm_rope(dev, q_scale):
    """q_scale multiplies the rotated q rows before their one rounding; k rows are unscaled."""
    ops = _ops()
    from qwen_image_edit_streamdiffusion_amd.rope import rope_tables
    B, H, s_pad = 2, 3, 512
    shapes, txt = [(1, 8, 8), (1, 8, 16)], 37
    S_img = 64 + 128
    qkv = rnd((3, B, H, s_pad, 128), dev, 2.0, 24)
    orig = qkv.clone()
    ws = [(1 + rnd((128,), dev, 0.1, 25 + i).float()).to(BF16) for i in range(4)]
    ic, is_, tc, ts = rope_tables(shapes, txt, dev)
    ops.qk_norm_rope(qkv, 0, S_img, ws[0], ws[1], ic, is_, q_scale=q_scale)
    ops.qk_norm_rope(qkv, S_img, txt, ws[2], ws[3], tc, ts, q_scale=q_scale)
    ip, tp = R.rope_phases(shapes, txt)
    for which in (0, 1):
        for seg, (a, n, wq, ph) in enumerate([(0, S_img, ws[which], ip), (S_img, txt, ws[2 + which], tp)]):
            x = orig[which, :, :, a:a + n].cpu().permute(0, 2, 1, 3)  # [B, S, H, Dh]
            ref = R.apply_rope(R.rms_norm(x, wq.cpu(), 1e-6, RB), ph, _R_F32).permute(0, 2, 1, 3)
            ref = (ref * (q_scale if which == 0 else 1.0)).to(BF16)
            close(qkv[which, :, :, a:a + n], ref)
    assert torch.equal(qkv[2], orig[2])  # V untouched
    assert torch.equal(qkv[:, :, :, S_img + txt:], orig[:, :, :, S_img + txt:])


def _qkv_nr_case(dev, B, rpb, H, K, off, s_pad, seed, hw):
    from qwen_image_edit_streamdiffusion_amd.rope import rope_tables
    x = rnd((B * rpb, K), dev, 1.0, seed)
    w, b = rnd((3 * H * 128, K), dev, 0.05, seed + 1), rnd((3 * H * 128,), dev, 0.1, seed + 2)
    nq, nk = [(1 + rnd((128,), dev, 0.1, seed + 3 + i).float()).to(BF16) for i in range(2)]
    shapes = [(1,) + hw, (1,) + hw]
    assert 2 * hw[0] * hw[1] == rpb
    ic, is_, _, _ = rope_tables(shapes, 16, dev)
    return x, w, b, nq, nk, ic, is_, shapes


@pytest.mark.parametrize("B,rpb,H,K,off,s_pad,hw", [
    (2, 2048, 8, 256, 0, 2304, (32, 32)),    # 192 big tiles: the fused gemm_pp epilogue
    (1, 4096, 16, 384, 0, 4352, (32, 64)),   # 16 x 24 tiles, K = 3 tiles
    (2, 200, 2, 128, 40, 512, (10, 10)),     # small: GEMM + qie_qk_norm_rope_bf16 fallback
    (3, 1000, 16, 256, 0, 1024, (20, 25)),   # 288 big tiles whose rows cross batch boundaries (table-row wrap)
    (24, 200, 8, 256, 40, 256, (10, 10)),    # 228 big tiles, batches shorter than a tile (table row by modulo)
])
@pytest.mark.parametrize("q_scale", [1.0, 0.12752])
def test_qkv_norm_rope_fused(dev, B, rpb, H, K, off, s_pad, hw, q_scale):
    """QKV projection with QK RMSNorm + RoPE in the epilogue == the two-launch path (within the
    GEMM tolerance: only the fp32 order of the sum of squares differs) and the oracle."""
    ops = _ops()
    x, w, b, nq, nk, ic, is_, shapes = _qkv_nr_case(dev, B, rpb, H, K, off, s_pad, 70, hw)
    fused = torch.zeros(3, B, H, s_pad, 128, dtype=BF16, device=dev)
    ops.linear_qkv_norm_rope(x, w, b, fused, rpb, off, nq, nk, ic, is_, q_scale=q_scale)
    two = torch.zeros_like(fused)
    ops.linear_qkv(x, w, b, two, rpb, off)
    ops.qk_norm_rope(two, off, rpb, nq, nk, ic, is_, q_scale=q_scale)
    sl = slice(off, off + rpb)
    close(fused[:, :, :, sl], two[:, :, :, sl])
    assert torch.equal(fused[2], two[2])  # V: no norm, same GEMM epilogue
    assert (fused[:, :, :, :off] == 0).all() and (fused[:, :, :, off + rpb:] == 0).all()
    lin = R.linear(x.cpu(), w.cpu(), b.cpu(), RB).view(B, rpb, 3, H, 128)
    ip, _ = R.rope_phases(shapes, 16)
    for which, wn in ((0, nq), (1, nk)):
        ref = R.apply_rope(R.rms_norm(lin[:, :, which], wn.cpu(), 1e-6, RB), ip, _R_F32).permute(0, 2, 1, 3)
        ref = (ref * (q_scale if which == 0 else 1.0)).to(BF16)
        close(fused[which, :, :, sl], ref, rel_l2=8e-3, ulps=4)


def test_qkv_norm_rope_fused_headline_persistent(dev):
    """The headline image QKV (B = 2 x 8192 rows, 24 heads, K = 3072): 2304 tiles, so each
    persistent work-group runs ~9 tiles with the norm + RoPE epilogue between them; == the
    two-launch path within the GEMM tolerance, V bitwise."""
    ops = _ops()
    B, rpb, H, K, s_pad = 2, 8192, 24, 3072, 8448
    x, w, b, nq, nk, ic, is_, _ = _qkv_nr_case(dev, B, rpb, H, K, 0, s_pad, 74, (64, 64))
    fused = torch.zeros(3, B, H, s_pad, 128, dtype=BF16, device=dev)
    ops.linear_qkv_norm_rope(x, w, b, fused, rpb, 0, nq, nk, ic, is_, q_scale=0.12752)
    two = torch.zeros_like(fused)
    ops.linear_qkv(x, w, b, two, rpb, 0)
    ops.qk_norm_rope(two, 0, rpb, nq, nk, ic, is_, q_scale=0.12752)
    close(fused[:, :, :, :rpb], two[:, :, :, :rpb])
    assert torch.equal(fused[2], two[2])
    assert (fused[:, :, :, rpb:] == 0).all()


def test_qkv_norm_rope_fused_i8(dev):
    ops = _ops()
    B, rpb, H, K = 2, 2048, 8, 256
    g = torch.Generator().manual_seed(72)
    xq = torch.randint(-127, 128, (B * rpb, K), generator=g, dtype=torch.int8).to(dev)
    sx = (torch.rand(B * rpb, generator=g) * 0.01 + 1e-3).to(dev)
    wq8 = torch.randint(-127, 128, (3 * H * 128, K), generator=g, dtype=torch.int8).to(dev)
    sw = (torch.rand(3 * H * 128, generator=g) * 1e-3 + 1e-4).to(dev)
    _, _, b, nq, nk, ic, is_, _ = _qkv_nr_case(dev, B, rpb, H, K, 0, 2304, 73, (32, 32))
    fused = torch.zeros(3, B, H, 2304, 128, dtype=BF16, device=dev)
    ops.linear_qkv_norm_rope_i8(xq, sx, wq8, sw, b, fused, rpb, 0, nq, nk, ic, is_, q_scale=0.12752)
    two = torch.zeros_like(fused)
    ops.linear_qkv_i8(xq, sx, wq8, sw, b, two, rpb, 0)
    ops.qk_norm_rope(two, 0, rpb, nq, nk, ic, is_, q_scale=0.12752)
    close(fused[:, :, :, :rpb], two[:, :, :, :rpb])
    assert torch.equal(fused[2], two[2])


def _attn_ref(qkv, kv_len, s_img, txt_rows, log2q=False):
    """fp32 SDPA; log2q: the q plane holds q * scale * log2(e), i.e. logits in log2 units."""
    _, B, H, s_pad, Dh = qkv.shape
    S = s_img + txt_rows
    q, k, v = (qkv[i].float().cpu() for i in range(3))
    sc = math.log(2.0) if log2q else 1.0 / math.sqrt(Dh)
    outs = []
    for b in range(B):
        L = kv_len[b]
        s = q[b, :, :S] @ k[b, :, :L].transpose(-1, -2) * sc
        o = torch.softmax(s, -1) @ v[b, :, :L]  # [H, S, Dh]
        outs.append(o.permute(1, 0, 2).reshape(S, H * Dh))
    o = torch.stack(outs)
    return o[:, :s_img].reshape(B * s_img, H * Dh), o[:, s_img:].reshape(B * txt_rows, H * Dh)


@pytest.mark.parametrize("B,H,s_img,txt_rows,kv_len,scale", [
    (1, 2, 512, 40, [552], 1.0),
    (2, 2, 512, 40, [552, 530], 1.0),
    (2, 3, 1024, 216, [1240, 1235], 3.0),
    (1, 1, 256, 0, [256], 1.0),
])
def test_attention(dev, B, H, s_img, txt_rows, kv_len, scale):
    ops = _ops()
    s_pad = ((s_img + txt_rows + 255) // 256) * 256
    qkv = rnd((3, B, H, s_pad, 128), dev, scale, 30)
    qkv[:, :, :, s_img + txt_rows:] = 0
    oi = torch.empty(B * s_img, H * 128, dtype=BF16, device=dev)
    ot = torch.empty(max(B * txt_rows, 1), H * 128, dtype=BF16, device=dev)
    ops.attention(qkv, kv_len, oi, ot[: B * txt_rows] if txt_rows else None, s_img, txt_rows)
    ri, rt = _attn_ref(qkv, kv_len, s_img, txt_rows)
    close(oi, ri, rel_l2=1e-2, ulps=8)
    if txt_rows:
        close(ot[: B * txt_rows], rt, rel_l2=1e-2, ulps=8)


@pytest.mark.parametrize("B,H,s_img,txt_rows,kv_len", [
    (1, 2, 512, 40, [552]),            # 3 query blocks, last one split over 9 key tiles
    (2, 3, 1024, 216, [1240, 1100]),   # masked keys in a middle range of row 1
    (1, 1, 256, 20, [100]),            # 2 key tiles < 5 ranges: empty ranges combine to nothing
    (1, 1, 256, 0, [256]),             # one query block: nothing to split
])
def test_attention_split_tail(dev, B, H, s_img, txt_rows, kv_len):
    """qie_attention_fwd_split_bf16: the last query block of each (b, h) as key ranges + combine;
    same tolerance as the unsplit kernel vs the oracle, and close to the unsplit result."""
    ops = _ops()
    s_pad = ((s_img + txt_rows + 255) // 256) * 256
    qkv = rnd((3, B, H, s_pad, 128), dev, 1.0, 33)
    qkv[:, :, :, s_img + txt_rows:] = 0
    nb = ops.attention_workspace_bytes(B, H, s_pad, s_img, txt_rows)
    assert (nb > 0) == (s_pad > 256)
    ws = torch.full((max(nb // 4, 4),), float("nan"), device=dev)  # stale data must not leak
    outs = []
    for w in (ws, None):
        oi = torch.empty(B * s_img, H * 128, dtype=BF16, device=dev)
        ot = torch.empty(max(B * txt_rows, 1), H * 128, dtype=BF16, device=dev)
        ops.attention(qkv, kv_len, oi, ot[: B * txt_rows] if txt_rows else None, s_img, txt_rows, workspace=w)
        outs.append((oi, ot[: B * txt_rows]))
    ri, rt = _attn_ref(qkv, kv_len, s_img, txt_rows)
    close(outs[0][0], ri, rel_l2=1e-2, ulps=8)
    close(outs[0][0], outs[1][0], rel_l2=4e-3, ulps=4)
    if txt_rows:
        close(outs[0][1], rt, rel_l2=1e-2, ulps=8)


def test_attention_split_workspace_too_small(dev):
    from qwen_image_edit_streamdiffusion_amd import _lib
    ops = _ops()
    qkv = rnd((3, 1, 1, 512, 128), dev, 1.0, 34)
    oi = torch.empty(512, 128, dtype=BF16, device=dev)
    ws = torch.empty(16, device=dev)
    with pytest.raises(_lib.QieError):
        ops.attention(qkv, [512], oi, None, 512, 0, workspace=ws)


def test_attention_spike_rescale(dev):
    """Force the online-softmax rescale: one key far above the rest in a late tile."""
    ops = _ops()
    B, H, s_img = 1, 1, 512
    qkv = rnd((3, B, H, s_img, 128), dev, 1.0, 31)
    qkv[1, 0, 0, 450] = qkv[0, 0, 0, 3] * 6  # key 450 aligned with query 3
    oi = torch.empty(s_img, 128, dtype=BF16, device=dev)
    ops.attention(qkv, [s_img], oi, None, s_img, 0)
    ri, _ = _attn_ref(qkv, [s_img], s_img, 0)
    close(oi, ri, rel_l2=1e-2, ulps=8)


LOG2Q = 1.4426950408889634 / math.sqrt(128)


@pytest.mark.parametrize("B,H,s_img,txt_rows,kv_len,qmul,split", [
    (1, 2, 512, 40, [552], 1.0, True),
    (2, 3, 1024, 216, [1240, 1100], 1.0, True),   # masked keys in row 1
    (2, 2, 512, 40, [552, 530], 3.0, False),      # sharp softmax, rescales every few tiles
    (1, 1, 256, 20, [100], 1.0, True),            # empty key ranges
    (1, 1, 256, 0, [256], 1.0, True),             # one query block
])
def test_attention_log2q(dev, B, H, s_img, txt_rows, kv_len, qmul, split):
    """qie_attention_fwd_log2q_bf16 on a q plane pre-multiplied by scale*log2(e) (one bf16
    rounding of the product, as the producers' q_scale writes it) vs fp32 softmax in base 2,
    and vs the plain kernel on the unscaled q."""
    ops = _ops()
    s_pad = ((s_img + txt_rows + 255) // 256) * 256
    qkv = rnd((3, B, H, s_pad, 128), dev, 1.0, 36)
    qkv[0] *= qmul
    qkv[:, :, :, s_img + txt_rows:] = 0
    pre = qkv.clone()
    pre[0] = (qkv[0].float() * LOG2Q).to(BF16)
    nb = ops.attention_workspace_bytes(B, H, s_pad, s_img, txt_rows)
    ws = torch.full((max(nb // 4, 4),), float("nan"), device=dev) if split else None
    oi = torch.empty(B * s_img, H * 128, dtype=BF16, device=dev)
    ot = torch.empty(max(B * txt_rows, 1), H * 128, dtype=BF16, device=dev)
    ops.attention(pre, kv_len, oi, ot[: B * txt_rows] if txt_rows else None, s_img, txt_rows,
                  workspace=ws, log2q=True)
    ri, rt = _attn_ref(pre, kv_len, s_img, txt_rows, log2q=True)
    close(oi, ri, rel_l2=1e-2, ulps=8)
    if txt_rows:
        close(ot[: B * txt_rows], rt, rel_l2=1e-2, ulps=8)
    oi2 = torch.empty_like(oi)
    ot2 = torch.empty_like(ot)
    ops.attention(qkv, kv_len, oi2, ot2[: B * txt_rows] if txt_rows else None, s_img, txt_rows, workspace=ws)
    close(oi, oi2, rel_l2=1.5e-2, ulps=8)


def test_attention_log2q_rescale_edges(dev):
    """Query 0 sees only very negative logits (about -150 in log2 units: a running max clamped
    at 0 would underflow every p to 0), query 3 a late spike, query 200 an early one: the
    tile-t0 rescale must set the running max from the data."""
    ops = _ops()
    B, H, s_img = 1, 1, 512
    qkv = rnd((3, B, H, s_img, 128), dev, 1.0, 37).float()
    u = torch.randn(128, generator=torch.Generator().manual_seed(5)).to(dev)
    qkv[1, 0, 0] += 3 * u                      # common key component
    qkv[0, 0, 0, 0] = -3 * u                   # query 0 anti-aligned with every key
    qkv[1, 0, 0, 450] = qkv[0, 0, 0, 3] * 6    # late spike for query 3
    qkv[1, 0, 0, 5] = qkv[0, 0, 0, 200] * 6    # early spike for query 200
    qkv = qkv.to(BF16)
    pre = qkv.clone()
    pre[0] = (qkv[0].float() * LOG2Q).to(BF16)
    oi = torch.empty(s_img, 128, dtype=BF16, device=dev)
    ops.attention(pre, [s_img], oi, None, s_img, 0, log2q=True)
    ri, _ = _attn_ref(pre, [s_img], s_img, 0, log2q=True)
    assert torch.isfinite(oi.float()).all()
    close(oi, ri, rel_l2=1e-2, ulps=8)


def test_timestep_embed(dev):
    ops = _ops()
    t = torch.tensor([1.0, 0.02001953125, 0.7695, 0.0], dtype=BF16)
    y = ops.timestep_embed(t.to(dev), 256)
    close(y, R.timestep_sinusoid(t, 256).to(BF16), rel_l2=4e-3, ulps=2)


def test_silu(dev):
    ops = _ops()
    x = rnd((3, 3072), dev, 3.0, 32)
    close(ops.silu(x), R.silu(x.cpu(), RB))


def test_cfg_combine(dev):
    ops = _ops()
    B, S, S_img = 2, 256, 512
    out = rnd((2 * B, S_img, 64), dev, 1.0, 33)
    y = ops.cfg_combine(out[:B, :S], out[B:, :S], 4.0)
    ref = R.cfg_combine(out[:B, :S].cpu(), out[B:, :S].cpu(), 4.0)
    close(y, ref, rel_l2=2e-3, ulps=1)


def test_euler_step_bit_exact(dev):
    ops = _ops()
    B, S, S_img = 3, 256, 512
    inp = rnd((B, S_img, 64), dev, 1.0, 34)
    v = rnd((B, S, 64), dev, 1.0, 35)
    dts = [-0.98, -0.3, 0.0]
    x0 = inp[:, :S].clone()
    ops.euler_step(inp[:, :S], v, dts, inp[:, :S])
    for b in range(B):
        ref = R.euler_step(x0[b].cpu(), v[b].cpu(), 0.0, dts[b])
        assert torch.equal(inp[b, :S].cpu(), ref), b


def test_pack_unpack_exact(dev):
    ops = _ops()
    x = rnd((2, 16, 1, 32, 48), dev, 1.0, 36)
    p = ops.pack_latents(x)
    assert torch.equal(p.cpu(), R.pack_latents(x.cpu()))
    u = ops.unpack_latents(p, 32, 48)
    assert torch.equal(u.cpu(), x.cpu())


def test_quantize_rows_exact(dev):
    ops = _ops()
    x = rnd((37, 12288), dev, 1.5, 37)
    x[5] = 0
    q = torch.empty(37, 12288, dtype=torch.int8, device=dev)
    s = torch.empty(37, dtype=torch.float32, device=dev)
    ops.quantize_rows(x, q, s)
    qr, sr = Q8.quantize_rows(x.float().cpu().numpy())
    assert np.array_equal(q.cpu().numpy(), qr)
    assert np.array_equal(s.cpu().numpy(), sr)


@pytest.mark.parametrize("M,N,K,act", [(300, 384, 256, 0), (4300, 3072, 384, 1), (2048, 2048, 3072, 0)])
def test_linear_i8(dev, M, N, K, act):
    ops = _ops()
    g = torch.Generator().manual_seed(40)
    xq = torch.randint(-127, 128, (M, K), generator=g, dtype=torch.int8)
    wq = torch.randint(-127, 128, (N, K), generator=g, dtype=torch.int8)
    sx = torch.rand(M, generator=g) * 0.01 + 1e-3
    sw = torch.rand(N, generator=g) * 0.001 + 1e-4
    b = (torch.randn(N, generator=g) * 0.1).to(BF16)
    y = torch.empty(M, N, dtype=BF16, device=dev)
    ops.linear_i8(xq.to(dev), sx.to(dev), wq.to(dev), sw.to(dev), b.to(dev), y, act=act)
    acc = Q8.int8_gemm_acc(xq.numpy(), wq.numpy())
    ref = torch.from_numpy(Q8.dequant(acc, sx.numpy(), sw.numpy(), b.float().numpy())).to(BF16).float()
    if act:
        ref = R.gelu_tanh(ref, RB)
    close(y, ref, rel_l2=4e-3, ulps=2)


def test_linear_i8_gated_and_qkv(dev):
    ops = _ops()
    g = torch.Generator().manual_seed(41)
    B, rpb, K, H = 2, 260, 256, 2
    N = H * 128
    xq = torch.randint(-127, 128, (B * rpb, K), generator=g, dtype=torch.int8).to(dev)
    sx = (torch.rand(B * rpb, generator=g) * 0.01 + 1e-3).to(dev)
    wq = torch.randint(-127, 128, (3 * N, K), generator=g, dtype=torch.int8).to(dev)
    sw = (torch.rand(3 * N, generator=g) * 1e-3 + 1e-4).to(dev)
    b = (torch.randn(3 * N, generator=g) * 0.1).to(BF16).to(dev)
    ref = torch.from_numpy(Q8.dequant(Q8.int8_gemm_acc(xq.cpu().numpy(), wq.cpu().numpy()),
                                      sx.cpu().numpy(), sw.cpu().numpy(), b.float().cpu().numpy()))
    ref = ref.to(BF16).float()
    qkv = torch.zeros(3, B, H, 512, 128, dtype=BF16, device=dev)
    ops.linear_qkv_i8(xq, sx, wq, sw, b, qkv, rpb, 0)
    close(qkv[:, :, :, :rpb], ref.view(B, rpb, 3, H, 128).permute(2, 0, 3, 1, 4))
    gate = rnd((B, N), dev, 0.5, 42)
    resid = rnd((B * rpb, N), dev, 1.0, 43)
    r0 = resid.cpu().float()
    ops.linear_gated_residual_i8(xq, sx, wq[:N], sw[:N], b[:N], gate, rpb, resid)
    exp = R.gated_residual(r0.view(B, rpb, N), gate.cpu(), ref[:, :N].reshape(B, rpb, N), RB)
    close(resid, exp.view(B * rpb, N))


# ------------------------------------------------------------------ split-K (text-stream) linears
@pytest.mark.parametrize("M,N,K,splits", [(432, 3072, 3072, 4), (216, 3072, 12288, 8), (37, 512, 1024, 2),
                                          (432, 1024, 768, 3), (130, 256, 512, 1), (432, 3072, 3072, 1),
                                          (37, 1024, 768, 1)])
@pytest.mark.parametrize("kind", [0, 1, 2])
def test_linear_splitk_vs_oracle(dev, M, N, K, splits, kind):
    """bf16 split-K: same tolerances as the unsplit GEMM (only the fp32 sum order differs)."""
    ops = _ops()
    x, w, b = rnd((M, K), dev, 1.0, 60), rnd((N, K), dev, 0.05, 61), rnd((N,), dev, 0.1, 62)
    ws = torch.empty(ops.splitk_workspace_bytes(M, N, splits) // 4, device=dev)
    lin = R.linear(x.cpu(), w.cpu(), b.cpu(), RB)
    if kind == ops.EPI_GATED_RESIDUAL:
        B = 2 if M % 2 == 0 else 1
        rpb = M // B
        gate = rnd((B, N), dev, 0.5, 63)
        resid = rnd((M, N), dev, 1.0, 64)
        ref = R.gated_residual(resid.cpu().float().view(B, rpb, N), gate.cpu(), lin.view(B, rpb, N), RB).view(M, N)
        ops.linear_splitk(x, w, b, kind, resid, ws, splits, gate=gate, rows_per_batch=rpb)
        close(resid, ref)
    else:
        y = torch.empty(M, N, dtype=BF16, device=dev)
        ops.linear_splitk(x, w, b, kind, y, ws, splits)
        close(y, R.gelu_tanh(lin, RB) if kind == ops.EPI_GELU else lin)


@pytest.mark.parametrize("splits", [4, 1])
def test_linear_splitk_qkv_matches_unsplit(dev, splits):
    ops = _ops()
    B, H, Dh, rpb, s_pad, off, K = 2, 2, 128, 216, 512, 256, 3072
    x, w, b = rnd((B * rpb, K), dev, 1.0, 65), rnd((3 * H * Dh, K), dev, 0.02, 66), rnd((3 * H * Dh,), dev, 0.1, 67)
    a = torch.zeros(3, B, H, s_pad, Dh, dtype=BF16, device=dev)
    c = torch.zeros_like(a)
    ops.linear_qkv(x, w, b, a, rpb, off)
    ws = torch.empty(ops.splitk_workspace_bytes(B * rpb, 3 * H * Dh, 4) // 4, device=dev)
    ops.linear_splitk(x, w, b, ops.EPI_QKV, c, ws, splits, rows_per_batch=rpb, seq_offset=off)
    close(c[:, :, :, off:off + rpb], a[:, :, :, off:off + rpb])
    assert (c[:, :, :, :off] == 0).all() and (c[:, :, :, off + rpb:] == 0).all()


@pytest.mark.parametrize("splits", [4, 1])
@pytest.mark.parametrize("kind", [0, 1, 2, 3])
def test_linear_splitk_i8_bitwise_equals_unsplit(dev, kind, splits):
    """int8 split-K sums int32 partials: bitwise the unsplit int8 result for every epilogue."""
    ops = _ops()
    g = torch.Generator().manual_seed(68)
    B, rpb, K, H = 2, 216, 3072, 2
    M, N = B * rpb, 3 * H * 128
    xq = torch.randint(-127, 128, (M, K), generator=g, dtype=torch.int8).to(dev)
    wq = torch.randint(-127, 128, (N, K), generator=g, dtype=torch.int8).to(dev)
    sx = (torch.rand(M, generator=g) * 0.01 + 1e-3).to(dev)
    sw = (torch.rand(N, generator=g) * 1e-3 + 1e-4).to(dev)
    b = (torch.randn(N, generator=g) * 0.1).to(BF16).to(dev)
    ws = torch.empty(ops.splitk_workspace_bytes(M, N, 4) // 4, device=dev)
    if kind == ops.EPI_QKV:
        a = torch.zeros(3, B, H, 512, 128, dtype=BF16, device=dev)
        c = torch.zeros_like(a)
        ops.linear_qkv_i8(xq, sx, wq, sw, b, a, rpb, 0)
        ops.linear_splitk_i8(xq, sx, wq, sw, b, kind, c, ws, splits, rows_per_batch=rpb)
    elif kind == ops.EPI_GATED_RESIDUAL:
        gate = rnd((B, N), dev, 0.5, 69)
        a = rnd((M, N), dev, 1.0, 70)
        c = a.clone()
        ops.linear_gated_residual_i8(xq, sx, wq, sw, b, gate, rpb, a)
        ops.linear_splitk_i8(xq, sx, wq, sw, b, kind, c, ws, splits, gate=gate, rows_per_batch=rpb)
    else:
        a = torch.empty(M, N, dtype=BF16, device=dev)
        c = torch.empty_like(a)
        ops.linear_i8(xq, sx, wq, sw, b, a, act=kind)
        ops.linear_splitk_i8(xq, sx, wq, sw, b, kind, c, ws, splits)
    assert torch.equal(a, c)


def _gpu_ref_linear(x, w, b):
    """fp32 torch reference on the device (bf16 inputs, fp32 accumulate, one bf16 rounding)."""
    return (x.float() @ w.float().t() + b.float()).to(BF16)


@pytest.mark.parametrize("M,N,K,act", [
    (4400, 9216, 3072, 0),   # 18 x 36 = 648 tiles: every work-group of the persistent GEMM runs 2-3 tiles
    (6000, 3072, 3136, 1),   # 288 tiles, nk = 49 (odd: the LDS slot parity flips from tile to tile), GELU
    (6016, 4352, 192, 0),    # nk = 3 (the shortest K the big kernels take), ragged M and N tiles
])
def test_linear_persistent_multi_tile(dev, M, N, K, act):
    """The persistent big-shape GEMM (gemm_w4p: one work-group per CU walking several output tiles,
    the K-tile pipeline crossing tile boundaries) against an fp32 torch reference on the device."""
    ops = _ops()
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g, device=dev).to(BF16)
    w = (torch.randn(N, K, generator=g, device=dev) * 0.02).to(BF16)
    b = (torch.randn(N, generator=g, device=dev) * 0.1).to(BF16)
    y = ops.linear(x, w, b, act=act)
    ref = _gpu_ref_linear(x, w, b)
    if act:
        ref = torch.nn.functional.gelu(ref.float(), approximate="tanh").to(BF16)
    close(y, ref)


def test_gated_residual_persistent_multi_tile(dev):
    ops = _ops()
    B, rpb, N, K = 2, 3000, 3072, 1088  # 24 x 12 = 288 tiles, nk = 17
    M = B * rpb
    g = torch.Generator(device=dev).manual_seed(77)
    x = torch.randn(M, K, generator=g, device=dev).to(BF16)
    w = (torch.randn(N, K, generator=g, device=dev) * 0.02).to(BF16)
    b = (torch.randn(N, generator=g, device=dev) * 0.1).to(BF16)
    gate = (torch.randn(B, N, generator=g, device=dev) * 0.5).to(BF16)
    resid = torch.randn(M, N, generator=g, device=dev).to(BF16)
    h = _gpu_ref_linear(x, w, b).float().view(B, rpb, N)
    ref = (resid.float().view(B, rpb, N) + (gate.float()[:, None, :] * h).to(BF16).float()).to(BF16).view(M, N)
    ops.linear_gated_residual(x, w, b, gate, rpb, resid)
    close(resid, ref)


def test_linear_i8_persistent_multi_tile(dev):
    ops = _ops()
    M, N, K = 6000, 3072, 3200  # 288 tiles, nk = 25 (int8 K tiles of 128)
    g = torch.Generator().manual_seed(41)
    xq = torch.randint(-127, 128, (M, K), generator=g, dtype=torch.int8)
    wq = torch.randint(-127, 128, (N, K), generator=g, dtype=torch.int8)
    sx = torch.rand(M, generator=g) * 0.01 + 1e-3
    sw = torch.rand(N, generator=g) * 0.001 + 1e-4
    b = (torch.randn(N, generator=g) * 0.1).to(BF16)
    y = torch.empty(M, N, dtype=BF16, device=dev)
    ops.linear_i8(xq.to(dev), sx.to(dev), wq.to(dev), sw.to(dev), b.to(dev), y)
    # exact integer accumulation on the device (fp64 holds these int32 sums exactly)
    acc = xq.to(dev).double() @ wq.to(dev).double().t()
    ref = (acc * sx.to(dev).double()[:, None] * sw.to(dev).double()[None, :] + b.to(dev).double()).to(BF16)
    close(y, ref, rel_l2=4e-3, ulps=2)
