"""The stream engines' arithmetic on the CPU oracle (test infrastructure): lets the slot logic of
StreamBatchDenoiser and the exchange logic of parallel.CFGPairStreamDenoiser run without a GPU
(gloo, world size 2). Every batch row goes through the oracle on its own, with its text cut to
its valid length, so a row's result cannot depend on what else is in the batch -- the property
the HIP kernels have by construction -- and equals the oracle's sequential denoise bit for bit."""
from typing import List

import torch

from oracle import dit_ref as R

BF16 = torch.bfloat16


class OracleStreamCompute:
    def __init__(self, params, cfg):
        self.params, self.cfg = params, cfg
        self.device = torch.device("cpu")
        self.forwards = 0

    def empty(self, *shape):
        return torch.empty(*shape, dtype=BF16)

    def zeros(self, *shape):
        return torch.zeros(*shape, dtype=BF16)

    def timesteps(self, per_row: List[float]):
        return R.model_timestep(torch.tensor([float(t) for t in per_row]))

    def forward(self, inp, enc, t_rows, img_shapes, txt_lens):
        rows = []
        for r in range(inp.shape[0]):
            n = int(txt_lens[r])
            rows.append(R.transformer_forward(self.params, self.cfg, inp[r:r + 1], enc[r:r + 1, :n],
                                              t_rows[r:r + 1], img_shapes[r], [n]).to(BF16))
        self.forwards += 1
        return torch.cat(rows, 0)

    def cfg_combine(self, cond, uncond, scale, out):
        out.copy_(R.cfg_combine(cond, uncond, scale))
        return out

    def euler_step(self, x, v, dts, out):
        for r, dt in enumerate(dts):  # oracle step with sigma = 0, sigma_next = dt (same fp32 difference)
            out[r] = R.euler_step(x[r], v[r], 0.0, float(dt))

    def copy(self, src, dst):
        dst.copy_(src)
