"""Prompt encoder language model on the GPU: the Qwen2.5-VL kernels of vl.hip
and the whole QwenVLTextModel vs transformers' Qwen2_5_VLTextModel (oracle/vl_ref.py; random
weights of reduced width, bf16-representable, fp32 eager oracle).

Tolerances:
  * embed_rows, silu_mul, rope_half: exact vs torch restatements with the same bf16 rounding points
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
