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


def _cfg_case():
    from oracle import dit_ref as R
    cfg = R.tiny_config()
    params = R.random_params(cfg, seed=0)
    g = torch.Generator().manual_seed(11)
    pe = torch.randn(1, 12, cfg.joint_attention_dim, generator=g).to(BF16)
    ne = torch.randn(1, 7, cfg.joint_attention_dim, generator=g).to(BF16)
    frames = [(torch.randn(1, 16, 64, generator=g).to(BF16), torch.randn(1, 16, 64, generator=g).to(BF16))
              for _ in range(3)]  # (noise, cond latents)
    return R, cfg, params, pe, ne, frames


def _worker_cfg(rank, world, port, q):
    """parallel.CFGPairStreamDenoiser over gloo: rank 0 = cond rows, rank 1 = uncond rows of the
    same in-flight frames; every finished frame must equal the oracle's sequential true-CFG
    denoise of that frame, bitwise, on both ranks."""
    try:
        parallel = _init(rank, world, port)
        from oracle_compute import OracleStreamCompute
        R, cfg, params, pe, ne, frames = _cfg_case()
        group, role, size = parallel.make_pair_groups(world)
        assert (role, size) == (rank % 2, 2)
        cx = OracleStreamCompute(params, cfg)
        eng = parallel.CFGPairStreamDenoiser(None, num_steps=2, true_cfg_scale=4.0, latent_hw=(4, 4),
                                             cond_hw=(4, 4), compute=cx, role=role, group=group)
        eng.set_conditions(pe, None, ne)
        assert eng.branches == [role] and eng.rows == 2
        outs = {}
        for noise, cond in frames:
            r = eng.push(noise, cond)
            if r is not None:
                outs[r[0]] = r[1]
        outs.update(dict(eng.flush()))
        ok = sorted(outs) == [0, 1, 2]
        shapes = [(1, 4, 4), (1, 4, 4)]
        for i, (noise, cond) in enumerate(frames):
            ref = R.denoise(params, cfg, noise, cond, pe, shapes, 2, neg_embeds=ne, true_cfg_scale=4.0)
            ok = ok and bool(torch.equal(outs[i], ref))
        q.put(("ok", rank, ok, cx.forwards))
        dist.destroy_process_group()
    except Exception as e:
        q.put(("err", repr(e)))
        raise


def _worker_pairs_x_shards(rank, world, port, q):
    """bench.py's `stream2-cfg-pairs` collective sequence on 4 ranks = 2 pairs: pair groups, the
    delivery group of the cond ranks, per-frame all_gather inside each pair, gather of every
    finished frame to rank 0 over the delivery group, then the barrier and the max / sum
    reductions over all ranks. Each pair runs its own frames; rank 0 must receive, per step, the
    finished frame of both pairs, each equal to the oracle's sequential true-CFG result."""
    try:
        parallel = _init(rank, world, port)
        from oracle_compute import OracleStreamCompute
        R, cfg, params, pe, ne, _ = _cfg_case()
        group, role, size = parallel.make_pair_groups(world)
        dgroup, heads = parallel.make_head_group(world, size)
        assert heads == [0, 2] and size == 2 and role == rank % 2
        pe_b = parallel.broadcast_prompt(pe if rank == 0 else None, tuple(pe.shape), BF16, torch.device("cpu"))
        assert torch.equal(pe_b, pe)
        shard = rank // size
        g = torch.Generator().manual_seed(100 + shard)  # both ranks of a pair draw the same frames
        frames = [(torch.randn(1, 16, 64, generator=g).to(BF16), torch.randn(1, 16, 64, generator=g).to(BF16))
                  for _ in range(3)]
        eng = parallel.CFGPairStreamDenoiser(None, num_steps=2, true_cfg_scale=4.0, latent_hw=(4, 4),
                                             cond_hw=(4, 4), compute=OracleStreamCompute(params, cfg),
                                             role=role, group=group, group_size=size)
        eng.set_conditions(pe_b, None, ne)
        head = role == 0
        got = []
        done = 0
        for noise, cond in frames + [(None, None)]:
            r = eng.push(noise, cond)
            if r is None:
                continue
            done += 1 if head else 0
            bufs = [torch.empty(1, 16, 64, dtype=BF16) for _ in heads] if rank == 0 else None
            parallel.deliver_to_root(r[1].contiguous(), bufs, head, dgroup)
            if rank == 0:
                got.append(bufs)
        dist.barrier()
        tt = torch.tensor([float(rank)], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dn = torch.tensor([float(done)], dtype=torch.float64)
        dist.all_reduce(dn, op=dist.ReduceOp.SUM)
        ok = tt.item() == world - 1 and dn.item() == 3 * len(heads)
        if rank == 0:
            shapes = [(1, 4, 4), (1, 4, 4)]
            for hi in range(len(heads)):
                gh = torch.Generator().manual_seed(100 + hi)
                fr = [(torch.randn(1, 16, 64, generator=gh).to(BF16), torch.randn(1, 16, 64, generator=gh).to(BF16))
                      for _ in range(3)]
                for i, (noise, cond) in enumerate(fr):
                    ref = R.denoise(params, cfg, noise, cond, pe, shapes, 2, neg_embeds=ne, true_cfg_scale=4.0)
                    ok = ok and bool(torch.equal(got[i][hi], ref))
            q.put(("ok", ok))
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


def test_cfg_pair_stream_engine_matches_sequential_cfg():
    msgs = _run(_worker_cfg, n_msgs=2)
    for m in msgs:
        assert m[0] == "ok", m
        assert m[2], f"rank {m[1]} diverged from sequential true-CFG"
        assert m[3] == 4  # 3 frames at depth 2: fill + 2 steady + 1 drain forwards per rank


def test_cfg_pair_engine_single_process_layouts():
    """The same engine without a process group: two engines wired together through begin() /
    finish() (the exchange as a local list), the pair of one, and the batched-CFG stream engine all
    give the oracle's sequential true-CFG result, bitwise."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle_compute import OracleStreamCompute
    from qwen_image_edit_streamdiffusion_amd.parallel import CFGPairStreamDenoiser
    from qwen_image_edit_streamdiffusion_amd.stream import StreamBatchDenoiser
    R, cfg, params, pe, ne, frames = _cfg_case()
    shapes = [(1, 4, 4), (1, 4, 4)]
    refs = [R.denoise(params, cfg, n, c, pe, shapes, 2, neg_embeds=ne, true_cfg_scale=4.0) for n, c in frames]
    kw = dict(num_steps=2, true_cfg_scale=4.0, latent_hw=(4, 4), cond_hw=(4, 4))

    def drive(push, flush):
        outs = {}
        for n, c in frames:
            r = push(n, c)
            if r is not None:
                outs[r[0]] = r[1]
        outs.update(dict(flush()))
        return outs

    # two engines, one per role, exchanging through a list
    e = [CFGPairStreamDenoiser(None, compute=OracleStreamCompute(params, cfg), role=r,
                               exchange=lambda v: None, **kw) for r in (0, 1)]
    for x in e:
        x.set_conditions(pe, None, ne)
    both = {0: {}, 1: {}}

    def push_pair(n, c):
        v = [x.begin(n, c) for x in e]
        if v[0] is None:
            return None
        parts = [t.contiguous() for t in v]
        res = [x.finish(parts) for x in e]
        for r in (0, 1):
            if res[r] is not None:
                both[r][res[r][0]] = res[r][1]
        return None

    for n, c in frames:
        push_pair(n, c)
    while any(s >= 0 for s in e[0].stage):
        push_pair(None, None)
    for r in (0, 1):
        assert sorted(both[r]) == [0, 1, 2]
        for i in range(3):
            assert torch.equal(both[r][i], refs[i]), (r, i)
    # a pair of one: both branches local, the exchange still called (returns the local part)
    one = CFGPairStreamDenoiser(None, compute=OracleStreamCompute(params, cfg), role=0, group_size=1,
                                exchange=lambda v: [v], **kw)
    one.set_conditions(pe, None, ne)
    assert one.branches == [0, 1] and one.rows == 4
    outs = drive(one.push, one.flush)
    assert all(torch.equal(outs[i], refs[i]) for i in range(3))
    # the batched-CFG stream engine on the same arithmetic
    base = StreamBatchDenoiser(None, compute=OracleStreamCompute(params, cfg), **kw)
    base.set_conditions(pe, None, ne)
    outs = drive(base.push, base.flush)
    assert all(torch.equal(outs[i], refs[i]) for i in range(3))


def test_cfg_pairs_times_frame_shard_collective_sequence():
    (st, ok), = _run(_worker_pairs_x_shards, world=4)
    assert st == "ok" and ok
