"""Multi-GPU axes of the hot path: one process per GPU.

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
The engines take their arithmetic as an object (``stream.HipStreamCompute`` by
default), so the exchange logic runs unchanged on CPU + gloo in tests.
"""
from __future__ import annotations

import os
import warnings
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .stream import StreamBatchDenoiser


def raise_hip_hw_queues(n: int = 8) -> bool:
    """Explicit opt-in for launchers of multi-rank runs (bench.py does the same inline): raise
    GPU_MAX_HW_QUEUES to ``n`` for this process and its children. Once RCCL adds its streams, HIP's
    default 4 hardware queues make the transformer's two streams share a queue and its text-stream
    overlap serialises (~9 % per step). Only effective before the first HIP call; returns False
    (and changes nothing) when HIP is already initialised. Importing the package never does this."""
    if torch.cuda.is_initialized():
        return False
    if int(os.environ.get("GPU_MAX_HW_QUEUES") or 0) < n:
        os.environ["GPU_MAX_HW_QUEUES"] = str(n)
    return True


def init_distributed(backend: Optional[str] = None):
    """Read RANK/WORLD_SIZE/LOCAL_RANK (torch.distributed.run), init the process
    group if world > 1, return (rank, world, local_rank, device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and torch.cuda.is_initialized() and int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
        warnings.warn("HIP initialised with fewer than 8 hardware queues: RCCL's streams will share "
                      "them with the transformer's text-stream overlap, which then serialises (~9 % "
                      "per step); export GPU_MAX_HW_QUEUES=8 (or call parallel.raise_hip_hw_queues()) "
                      "before the first HIP call")
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
    returns (my_pair_group, my_role, group_size) with role 0 = cond, 1 = uncond. World size 1 is a
    pair of one (that rank computes both branches, group_size 1)."""
    if world > 1 and world % 2:
        raise ValueError("CFG parallel needs an even number of ranks (or a single one)")
    rank = dist.get_rank()
    if world == 1:
        return dist.new_group(ranks=[0]), 0, 1
    mine = None
    for k in range(world // 2):
        g = dist.new_group(ranks=[2 * k, 2 * k + 1])
        if rank // 2 == k:
            mine = g
    return mine, rank % 2, 2


def make_head_group(world: int, pair_size: int):
    """The delivery group of a pairs x frame-shard run: the cond rank of every pair (ranks 0,
    pair_size, 2 * pair_size, ...). Every rank must call this (torch requirement), members or not.
    Returns (group, head_ranks)."""
    heads = list(range(0, world, pair_size))
    return dist.new_group(ranks=heads), heads


def deliver_to_root(x: torch.Tensor, bufs: Optional[List[torch.Tensor]], is_head: bool = True, group=None) -> None:
    """One finished frame per head rank to rank 0 (``bufs``: one tensor per head on rank 0, None
    elsewhere). Ranks that are not heads (the uncond rank of a pair holds the same latents as its
    partner) do not take part."""
    if not is_head or not dist.is_initialized():
        return
    dist.gather(x, bufs if dist.get_rank() == 0 else None, dst=0, group=group)


class CFGPairStreamDenoiser(StreamBatchDenoiser):
    """The stream-batch engine with its two CFG branches on the two ranks of a pair.

    Rank 2k (role 0) carries the cond rows of the ``depth`` in-flight frames, rank 2k + 1 (role 1)
    the uncond rows of the SAME frames: both ranks push the same noise and condition latents.
    Per pushed frame each rank runs one forward of ``depth`` rows, then ONE ``all_gather`` inside
    the pair moves the noise predictions (depth x 512 KiB at 1024^2), and both ranks apply the
    true-CFG combine and the per-row Euler step to identical inputs -- identical latents on both
    ranks afterwards, nothing is sent back. A branch's rows see the shapes they have in the
    batched-CFG engine (text padded to the longer prompt), and every kernel computes batch rows
    independently, so the result equals StreamBatchDenoiser's batched CFG bit for bit.

    ``group`` of one rank (a pair of one: world size 1, or a left-over rank): that rank computes
    both branches and the collective still runs, over the one-rank group.
    ``exchange``: replaces the collective (single-process tests wire two engines together with
    begin() / finish())."""

    def __init__(self, transformer, num_steps: int = 2, true_cfg_scale: float = 4.0,
                 latent_hw: Tuple[int, int] = (64, 64), cond_hw: Tuple[int, int] = (64, 64),
                 scheduler=None, compute=None, role: int = 0, group=None, group_size: Optional[int] = None,
                 exchange: Optional[Callable[[torch.Tensor], List[torch.Tensor]]] = None):
        super().__init__(transformer, num_steps, true_cfg_scale, latent_hw, cond_hw, scheduler, compute)
        if true_cfg_scale <= 1.0:
            raise ValueError("CFG pairs need true_cfg_scale > 1 (cond-only runs have one branch)")
        if group_size is None:
            group_size = 2 if exchange is not None else dist.get_world_size(group)
        if group_size not in (1, 2) or role not in (0, 1) or (group_size == 1 and role != 0):
            raise ValueError("a CFG pair has one or two ranks, roles 0 (cond) and 1 (uncond)")
        self.role, self.group, self.group_size, self.exchange = role, group, group_size, exchange

    def _local_branches(self) -> List[int]:
        if not self.cfg:
            raise ValueError("CFG pairs need negative_prompt_embeds in set_conditions()")
        return [0, 1] if self.group_size == 1 else [self.role]

    def _exchange(self, v_local: torch.Tensor) -> List[torch.Tensor]:
        v_local = v_local.contiguous()
        if self.exchange is not None:
            parts = self.exchange(v_local)
        else:
            parts = [torch.empty_like(v_local) for _ in range(self.group_size)]
            dist.all_gather(parts, v_local, group=self.group)  # pair order: [cond rank, uncond rank]
        if self.group_size == 1:  # both branches in the one part: [cond rows; uncond rows]
            D = self.depth
            return [parts[0][:D], parts[0][D:]]
        return list(parts)
