"""Pre-quantised int8 on-disk image on the CPU: save/load round trip,
strict key/shape/dtype checks, and the int8_only guard. The quantisation here is the oracle's
(tests only); the GPU round trip through the HIP quantiser is in test_gpu_model.py."""
import pytest
import torch

from oracle import int8_ref
from qwen_image_edit_streamdiffusion_amd import weights as W
from qwen_image_edit_streamdiffusion_amd.transformer import QwenImageTransformer2DModel


def _tiny_int8(seed=0):
    m = QwenImageTransformer2DModel(num_layers=2, num_attention_heads=2, joint_attention_dim=64,
                                    device="cpu")
    g = torch.Generator().manual_seed(seed)
    for n in m.diffusers_names():
        m._param_slot(n).normal_(0, 0.02, generator=g)
    for blk in m.transformer_blocks:
        blk.q8 = {}
        for n in m._I8_LINEARS:
            q, s = int8_ref.quantize_rows(getattr(blk, f"w_{n}").float().numpy())
            blk.q8[n] = (torch.from_numpy(q), torch.from_numpy(s))
    m.int8 = True
    return m


def test_roundtrip_exact(tmp_path):
    m = _tiny_int8()
    files = W.save_int8(m, str(tmp_path), blocks_per_shard=1)
    assert len(files) == 2
    m2 = W.load_int8(str(tmp_path), device="cpu")
    a, b = m.int8_state_dict(), m2.int8_state_dict()
    assert set(a) == set(b)
    for k in a:
        assert a[k].dtype == b[k].dtype and torch.equal(a[k], b[k]), k
    # the eight quantised linears carry no bf16 copy
    for blk in m2.transformer_blocks:
        for n in m2._I8_LINEARS:
            assert getattr(blk, f"w_{n}").numel() == 0
    assert m2.config == m.config


def test_int8_only_refuses_requantise(tmp_path):
    W.save_int8(_tiny_int8(), str(tmp_path))
    m2 = W.load_int8(str(tmp_path), device="cpu")
    with pytest.raises(RuntimeError):
        m2.quantize_int8()
    with pytest.raises(RuntimeError):
        m2.load_diffusers_state_dict({}, strict=False)


def test_rejects_corrupt_images(tmp_path):
    from safetensors.torch import save_file
    m = _tiny_int8()
    sd = {k: v.contiguous() for k, v in m.int8_state_dict().items()}
    import dataclasses
    import json
    meta = {"format": W.INT8_FORMAT, "config": json.dumps(dataclasses.asdict(m.config))}
    # missing key
    bad = dict(sd)
    bad.pop("transformer_blocks.1.up_txt.scale")
    save_file(bad, str(tmp_path / "qie_int8-00001-of-00001.safetensors"), metadata=meta)
    with pytest.raises(KeyError):
        W.load_int8(str(tmp_path), device="cpu")
    # wrong dtype of a quantised weight
    bad = dict(sd)
    bad["transformer_blocks.0.qkv_img.q8"] = bad["transformer_blocks.0.qkv_img.q8"].to(torch.int16)
    save_file(bad, str(tmp_path / "qie_int8-00001-of-00001.safetensors"), metadata=meta)
    with pytest.raises(ValueError):
        W.load_int8(str(tmp_path), device="cpu")
    # wrong format tag
    save_file(sd, str(tmp_path / "qie_int8-00001-of-00001.safetensors"),
              metadata={"format": "something-else", "config": meta["config"]})
    with pytest.raises(ValueError):
        W.load_int8(str(tmp_path), device="cpu")
