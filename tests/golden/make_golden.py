#!/usr/bin/env python3
"""Generate tests/golden/oracle_golden.npz -- REGRESSION fixtures of the CPU oracle.

Parity against the reference is UNPINNED (oracle/__init__.py): the reference
ships no vectors and its arithmetic lives in the absent diffusers package, so
these vectors come from this repo's own oracle (oracle/dit_ref.py,
oracle/int8_ref.py) on seeded inputs.  They freeze the oracle's behaviour so a
later edit to the checker cannot silently move the target the HIP kernels are
tested against.  Regenerate only on a deliberate, reviewed oracle change:

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import dit_ref as R  # noqa: E402
from oracle import int8_ref as Q8  # noqa: E402


def bits(t: torch.Tensor) -> np.ndarray:
    return t.to(torch.bfloat16).view(torch.int16).numpy()


def main():
    out = {}
    cfg = R.tiny_config()
    params = R.random_params(cfg, seed=0)
    g = torch.Generator().manual_seed(123)
    shapes = [(1, 8, 8), (1, 8, 8)]
    hs = torch.randn(2, 128, 64, generator=g).to(torch.bfloat16)
    enc = torch.randn(2, 16, cfg.joint_attention_dim, generator=g).to(torch.bfloat16)
    enc[1, 11:] = 0
    t = R.model_timestep(torch.tensor([1000.0, 20.0]))
    y = R.transformer_forward(params, cfg, hs, enc, t, shapes, [16, 11])
    out["fwd_hidden_states"] = bits(hs)
    out["fwd_encoder_hidden_states"] = bits(enc)
    out["fwd_timestep"] = bits(t)
    out["fwd_out"] = bits(y)
    for n in (2, 3, 4, 8):
        s, ts = R.sigma_schedule(n, 4096)
        out[f"sigmas_{n}_4096"] = s.numpy()
    out["timestep_emb"] = R.timestep_sinusoid(torch.tensor([1.0, 0.02001953125, 0.5]), 256).numpy()
    ip, tp = R.rope_phases([(1, 4, 6), (1, 4, 4)], 5)
    out["rope_img"], out["rope_txt"] = ip.numpy(), tp.numpy()
    x = (torch.randn(7, 256, generator=g) * 3).to(torch.bfloat16).float().numpy()
    x[3] = 0
    q, s = Q8.quantize_rows(x)
    out["q8_x"], out["q8_q"], out["q8_s"] = x, q, s
    c = torch.randn(3, 16, 64, generator=g).to(torch.bfloat16)
    u = torch.randn(3, 16, 64, generator=g).to(torch.bfloat16)
    out["cfg_c"], out["cfg_u"], out["cfg_out"] = bits(c), bits(u), bits(R.cfg_combine(c, u, 4.0))
    xs = torch.randn(16, 64, generator=g).to(torch.bfloat16)
    v = torch.randn(16, 64, generator=g).to(torch.bfloat16)
    out["euler_x"], out["euler_v"] = bits(xs), bits(v)
    out["euler_out"] = bits(R.euler_step(xs, v, 1.0, 0.02))
    np.savez_compressed(os.path.join(HERE, "oracle_golden.npz"), **out)
    print("wrote", os.path.join(HERE, "oracle_golden.npz"))


if __name__ == "__main__":
    main()
