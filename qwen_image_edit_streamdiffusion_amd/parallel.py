"""Multi-GPU axes of the hot path (SURVEY.md §8 e): one process per GPU.

* Frame shard (stream axis): frames are independent, so each rank (or each
  CFG pair) runs its own stream-batch engine on its own frames -- no collective
  on the data path except delivery: rank 0 ``broadcast``s the prompt
  embeddings once per prompt (~1.5 MB) and ``gather``s every finished latent
  (512 KiB per frame) for the serving front end.
* CFG parallel (the absent ``parallel_cfg_*.py`` of README.md:127-131, "GPU6:
  cond, GPU7: uncond"): ranks 2k and 2k+1 run the cond and the uncond branch
  of the SAME latents; per denoise step ONE ``all_gather`` of the 512 KiB
  noise prediction inside the pair, then both ranks apply the CFG combine and
  the Euler step redundantly (identical state, no broadcast back).

Backend "nccl" is RCCL over xGMI on ROCm.  Messages are <= 1.5 MB against a
~190 ms forward, so they are latency-bound; no ring all-reduce, no TP/SP.
The compute is injected (``forward``/``combine``/``step`` callables) so the
exchange logic runs unchanged on CPU + gloo in tests; the defaults are the
HIP transformer and libqie kernels.
"""
from __future__ import annotations

import os
import warnings
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist


def init_distributed(backend: Optional[str] = None):
    """Read RANK/WORLD_SIZE/LOCAL_RANK (torch.distributed.run), init the process
    group if world > 1, return (rank, world, local_rank, device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and torch.cuda.is_initialized() and int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
        warnings.warn("HIP initialised with fewer than 8 hardware queues: RCCL's streams will share "
                      "them with the transformer's text-stream overlap, which then serialises (~9 % "
                      "per step); export GPU_MAX_HW_QUEUES=8 before the first HIP call")
    use_cuda = torch.cuda.is_available() and backend != "gloo"
    device = torch.device("cuda", local) if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(device)
    if world > 1 and not dist.is_initialized():
        be = backend or ("nccl" if use_cuda else "gloo")
        if be == "nccl":
            dist.init_process_group(be, device_id=device)
        else:
            dist.init_process_group(be)
    return rank, world, local, device


def broadcast_prompt(embeds: Optional[torch.Tensor], shape: Sequence[int], dtype, device,
                     src: int = 0, group=None) -> torch.Tensor:
    """Fill the prompt-embed cache on every rank from ``src`` (once per prompt)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return embeds
    if dist.get_rank() == src:
        t = embeds.contiguous()
    else:
        t = torch.empty(*shape, dtype=dtype, device=device)
    dist.broadcast(t, src, group=group)
    return t


def gather_to_root(x: torch.Tensor, root: int = 0, group=None) -> Optional[List[torch.Tensor]]:
    """Deliver one finished latent per rank to ``root`` (list on root, None elsewhere)."""
    if not dist.is_initialized():
        return [x]
    world = dist.get_world_size(group)
    if dist.get_rank() == root:
        bufs = [torch.empty_like(x) for _ in range(world)]
        dist.gather(x.contiguous(), bufs, dst=root, group=group)
        return bufs
    dist.gather(x.contiguous(), None, dst=root, group=group)
    return None


def frame_owner(frame_idx: int, n_shards: int) -> int:
    """Round-robin frame -> shard assignment (a shard is a rank, or a CFG pair)."""
    return frame_idx % n_shards


def make_pair_groups(world: int):
    """All ranks create every pair group in the same order (torch requirement);
    returns (my_pair_group, my_role) with role 0 = cond, 1 = uncond."""
    if world % 2:
        raise ValueError("CFG parallel needs an even number of ranks")
    rank = dist.get_rank()
    mine = None
    for k in range(world // 2):
        g = dist.new_group(ranks=[2 * k, 2 * k + 1])
        if rank // 2 == k:
            mine = g
    return mine, rank % 2


@dataclass
class CFGParallelDenoiser:
    """Denoise one frame per pair; this rank computes one CFG branch.

    forward(x_model_input, step_index) -> noise prediction [B, S_noise, C] of
    THIS rank's branch (its own prompt/negative embeddings captured inside);
    combine(cond, uncond, scale) -> guided prediction; step(x, v, i) -> next x.
    """

    forward: Callable[[torch.Tensor, int], torch.Tensor]
    combine: Callable[[torch.Tensor, torch.Tensor, float], torch.Tensor]
    step: Callable[[torch.Tensor, torch.Tensor, int], torch.Tensor]
    scale: float
    group: object = None

    def denoise(self, x: torch.Tensor, num_steps: int) -> torch.Tensor:
        for i in range(num_steps):
            v_local = self.forward(x, i).contiguous()
            parts = [torch.empty_like(v_local) for _ in range(2)]
            dist.all_gather(parts, v_local, group=self.group)  # [cond, uncond] by pair order
            v = self.combine(parts[0], parts[1], self.scale)
            x = self.step(x, v, i)
        return x


# ---------------------------------------------------------------------------- HIP defaults
def hip_branch_forward(transformer, embeds: torch.Tensor, cond_latents: torch.Tensor,
                       timesteps: Sequence[float], img_shapes):
    """forward(x, i) for one CFG branch on the HIP transformer (B=1 rows)."""
    from . import ops
    from .scheduler import model_timesteps
    S_noise = None
    buf = {}

    def fwd(x: torch.Tensor, i: int) -> torch.Tensor:
        nonlocal S_noise
        S_noise = x.shape[1]
        inp = buf.get("inp")
        if inp is None:
            inp = torch.empty(x.shape[0], S_noise + cond_latents.shape[1], x.shape[2],
                              dtype=x.dtype, device=x.device)
            ops.copy_batched(cond_latents.expand(x.shape[0], -1, -1).contiguous(), inp[:, S_noise:])
            buf["inp"] = inp
        ops.copy_batched(x, inp[:, :S_noise])
        t = model_timesteps([timesteps[i]] * x.shape[0], x.device)
        out = transformer(inp, embeds, None, t, img_shapes, [embeds.shape[1]] * x.shape[0],
                          return_dict=False)[0]
        return out[:, :S_noise]

    return fwd


def hip_combine(cond: torch.Tensor, uncond: torch.Tensor, scale: float) -> torch.Tensor:
    from . import ops
    return ops.cfg_combine(cond.contiguous(), uncond.contiguous(), scale)


def hip_step(dts: Sequence[float]):
    from . import ops

    def step(x: torch.Tensor, v: torch.Tensor, i: int) -> torch.Tensor:
        out = torch.empty_like(x)
        return ops.euler_step(x, v, [dts[i]] * x.shape[0], out)

    return step
