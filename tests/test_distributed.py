"""Multi-process (gloo, world_size 2, CPU) checks of the parallel module's
exchange logic: prompt broadcast, frame gather to rank 0, and CFG-parallel
pairs (cond on rank 0, uncond on rank 1) reproducing sequential true-CFG
exactly.  The compute is the oracle (CPU); on GPUs the same code runs over
RCCL with the HIP callables."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

BF16 = torch.bfloat16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from qwen_image_edit_streamdiffusion_amd import parallel
    r, w, _, dev = parallel.init_distributed(backend="gloo")
    assert (r, w, dev.type) == (rank, world, "cpu")
    return parallel


def _worker_shard(rank, world, port, q):
    try:
        parallel = _init(rank, world, port)
        pe = torch.arange(12, dtype=torch.float32).view(1, 3, 4).to(BF16) if rank == 0 else None
        got = parallel.broadcast_prompt(pe, (1, 3, 4), BF16, torch.device("cpu"))
        assert torch.equal(got, torch.arange(12, dtype=torch.float32).view(1, 3, 4).to(BF16))
        outs = []
        for f in range(6):  # frames round-robin: rank r owns frames r, r+2, ...
            if parallel.frame_owner(f, world) == rank:
                lat = torch.full((1, 4, 8), float(f), dtype=BF16)
                g = parallel.gather_to_root(lat)
                if rank == 0:
                    outs.append([int(t[0, 0, 0].item()) for t in g])
        if rank == 0:
            q.put(("ok", outs))
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        q.put(("err", repr(e)))
        raise


def _worker_cfg(rank, world, port, q):
    try:
        parallel = _init(rank, world, port)
        from oracle import dit_ref as R
        cfg = R.tiny_config()
        params = R.random_params(cfg, seed=0)
        g = torch.Generator().manual_seed(11)
        pe = torch.randn(1, 12, cfg.joint_attention_dim, generator=g).to(BF16)
        ne = torch.randn(1, 7, cfg.joint_attention_dim, generator=g).to(BF16)
        cond = torch.randn(1, 16, 64, generator=g).to(BF16)
        noise = torch.randn(1, 16, 64, generator=g).to(BF16)
        shapes = [(1, 4, 4), (1, 4, 4)]
        sig, ts = R.sigma_schedule(2, 16)
        emb = pe if rank % 2 == 0 else ne
        group, role = parallel.make_pair_groups(world)
        assert role == rank % 2

        def fwd(x, i):
            t = R.model_timestep(ts[i].expand(1))
            out = R.transformer_forward(params, cfg, torch.cat([x, cond], 1), emb, t, shapes, [emb.shape[1]])
            return out[:, :16].to(BF16)

        den = parallel.CFGParallelDenoiser(
            forward=fwd, combine=R.cfg_combine,
            step=lambda x, v, i: R.euler_step(x, v, float(sig[i]), float(sig[i + 1])),
            scale=4.0, group=group)
        x = den.denoise(noise, 2)
        ref = R.denoise(params, cfg, noise, cond, pe, shapes, 2, neg_embeds=ne, true_cfg_scale=4.0)
        q.put(("ok", rank, bool(torch.equal(x, ref))))
        dist.destroy_process_group()
    except Exception as e:
        q.put(("err", repr(e)))
        raise


def _run(worker, world=2, n_msgs=1, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=timeout) for _ in range(n_msgs)]
    for p in procs:
        p.join(timeout)
        assert p.exitcode == 0
    return msgs


def test_prompt_broadcast_and_frame_gather():
    (st, outs), = _run(_worker_shard)
    assert st == "ok", outs
    assert outs == [[0, 1], [2, 3], [4, 5]]


def test_cfg_parallel_pair_matches_sequential_cfg():
    msgs = _run(_worker_cfg, n_msgs=2)
    for m in msgs:
        assert m[0] == "ok", m
        assert m[2], f"rank {m[1]} diverged from sequential true-CFG"
