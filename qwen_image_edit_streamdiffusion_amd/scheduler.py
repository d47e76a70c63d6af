"""FlowMatchEulerDiscreteScheduler for the Qwen-Image pipelines [U].

Host side: the sigma schedule (set_timesteps with dynamic exponential shift and
terminal stretch) in fp32 numpy exactly as diffusers computes
it; device side: ``step`` runs the fused Euler kernel (qie_euler_step_bf16),
which reproduces diffusers' rounding: the 0-d fp32 ``dt`` times the bf16 model
output gives a bf16 product, added to the fp32-cast sample, cast back to bf16.

Defaults are the Qwen-Image scheduler config (base_shift 0.5, max_shift 0.9,
seq 256..8192, shift_terminal 0.02).  The reference never replaces the
scheduler (qwen_realtime.py:128-130 only prints its name), also not when the
Lightning LoRA is loaded (server.py:76-79).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from . import ops


@dataclass
class FlowMatchConfig:
    num_train_timesteps: int = 1000
    base_image_seq_len: int = 256
    max_image_seq_len: int = 8192
    base_shift: float = 0.5
    max_shift: float = 0.9
    shift_terminal: Optional[float] = 0.02
    use_dynamic_shifting: bool = True
    shift: float = 1.0


def calculate_shift(image_seq_len: int, base_seq_len: int = 256, max_seq_len: int = 8192,
                    base_shift: float = 0.5, max_shift: float = 0.9) -> float:
    m = (max_shift - base_shift) / (max_seq_len - base_seq_len)
    b = base_shift - m * base_seq_len
    return image_seq_len * m + b


class FlowMatchEulerDiscreteScheduler:
    order = 1

    def __init__(self, config: Optional[FlowMatchConfig] = None):
        self.config = config or FlowMatchConfig()
        self.sigmas: Optional[torch.Tensor] = None
        self.timesteps: Optional[torch.Tensor] = None
        self._step_index: Optional[int] = None

    # ------------------------------------------------------------------ schedule
    def compute_sigmas(self, num_inference_steps: int, mu: Optional[float] = None,
                       sigmas: Optional[Sequence[float]] = None) -> np.ndarray:
        c = self.config
        if sigmas is None:
            sigmas = np.linspace(1.0, 1.0 / num_inference_steps, num_inference_steps)
        s = np.array(sigmas).astype(np.float32)
        if c.use_dynamic_shifting:
            if mu is None:
                raise ValueError("mu is required with use_dynamic_shifting")
            s = (math.exp(mu) / (math.exp(mu) + (1.0 / s - 1.0) ** 1.0)).astype(np.float32)
        else:
            s = (c.shift * s / (1 + (c.shift - 1) * s)).astype(np.float32)
        if c.shift_terminal:
            if len(s) < 2:
                raise ValueError("a single-step schedule with shift_terminal stretches 0/0 "
                                 "(NaN sigma); use >= 2 steps or shift_terminal=None")
            one_minus = 1.0 - s
            scale = one_minus[-1] / (1.0 - c.shift_terminal)
            s = (1.0 - one_minus / scale).astype(np.float32)
        return s

    def set_timesteps(self, num_inference_steps: int = None, device=None,
                      sigmas: Optional[Sequence[float]] = None, mu: Optional[float] = None,
                      image_seq_len: Optional[int] = None):
        if mu is None and image_seq_len is not None:
            c = self.config
            mu = calculate_shift(image_seq_len, c.base_image_seq_len, c.max_image_seq_len,
                                 c.base_shift, c.max_shift)
        s = self.compute_sigmas(num_inference_steps if sigmas is None else len(sigmas), mu, sigmas)
        st = torch.from_numpy(s).to(torch.float32)
        self.timesteps = (st * self.config.num_train_timesteps).to(device or "cpu")
        self.sigmas = torch.cat([st, torch.zeros(1)])  # kept on the host (diffusers: .to("cpu"))
        self._step_index = None
        return self.timesteps

    # ------------------------------------------------------------------ stepping
    def dt(self, i: int) -> float:
        """fp32 (sigma_{i+1} - sigma_i), as the 0-d tensor subtraction computes it."""
        return float((self.sigmas[i + 1] - self.sigmas[i]).item())

    @property
    def step_index(self):
        return self._step_index

    def index_for_timestep(self, timestep) -> int:
        t = float(timestep)
        idx = int(np.argmin(np.abs(self.timesteps.cpu().numpy() - t)))
        return idx

    def step(self, model_output: torch.Tensor, timestep, sample: torch.Tensor,
             out: Optional[torch.Tensor] = None, return_dict: bool = False):
        """x_{i+1} = bf16(x_i + bf16(dt * v)) on the device (qie_euler_step_bf16)."""
        if self._step_index is None:
            self._step_index = self.index_for_timestep(timestep)
        dt = self.dt(self._step_index)
        if out is None:
            out = torch.empty_like(sample)
        B = sample.shape[0]
        ops.euler_step(sample, model_output, [dt] * B, out)
        self._step_index += 1
        return (out,) if not return_dict else {"prev_sample": out}


def model_timesteps(timesteps_1000: Sequence[float], device) -> torch.Tensor:
    """Pipeline convention [U]: ``t.expand(B).to(bf16)`` then ``/ 1000`` in bf16."""
    t = torch.tensor([float(x) for x in timesteps_1000], dtype=torch.float32)
    tb = (t.to(torch.bfloat16) / 1000).to(torch.bfloat16)
    r = tb.to(device)
    # host copy of the values (bf16 bits): the transformer keys its modulation cache on it without
    # reading the device tensor back; _version guards against later in-place changes
    r._qie_host = tuple(int(v) for v in tb.view(torch.int16).tolist())
    r._qie_version = r._version
    return r
