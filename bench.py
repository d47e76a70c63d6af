#!/usr/bin/env python3
"""Headline benchmark: images/sec at 1024x1024, 2-step Lightning edit, on 1..8 MI355X.

Workload (BASELINE.json configs[2], the one its metric is quoted on):
Qwen-Image-Edit-2509 DiT (60 blocks, D=3072, random-init bf16 weights of the
real architecture -- no checkpoints offline), qwen_realtime-style stream batch
of depth 2 (= the 2 Lightning steps), cond-only (the server's default
use_cfg=False path, server.py:49,147-153), prompt-embed cache, 1024^2 output
(4096 noise tokens) + 1024^2 condition image (4096 tokens) + 216 text tokens.
One "step" = one pushed frame = one batched B=2 DiT forward + per-row Euler
step, with the VAE on both ends (HIP): the pushed condition
frame arrives as a uint8 RGB 1024x1024 camera image and is VAE-encoded
(QwenImageEncoder3d + quant_conv + normalise + pack), and the frame that
completes is VAE-decoded to uint8 RGB (unpack + de-normalise + post_quant_conv
+ QwenImageDecoder3d + postprocess).  --vae decode / none drop the encode /
both.  In steady state every step completes one image, so images/sec =
completed frames / time.  Synthetic inputs (randn / randint with fixed seeds)
are resident in HBM before the timed region.  The text encoder is not on this
path: the prompt embedding comes from the prompt cache;
--vl-per-frame puts it on the path (the reference's realtime call re-encodes
the prompt with every frame, qwen_realtime.py:247-255).

The same JSON line carries, under "secondary", the like-for-like workloads of
the reference's published numbers, each timed the same way right after the
headline (same process, same model): "stream2-cfg" (true CFG 4.0 as
benchmark_lightning.py:28-29 / qwen_realtime.py:247-255 run it: B = 4 rows per
frame), "stream2-vl-per-frame" (N = 1: the headline with the prompt re-encoded
with every frame), "stream2-int8" (configs[3]) and, on an even number of ranks
> 1, "stream2-cfg-pairs" (configs[4]: cond / uncond on the two ranks of a
pair, pairs x frame shard).

Multi-GPU (torch.distributed.run, one process per GPU, RCCL): each rank runs
its own stream engine on its own frames (frame shard, weak scaling); rank 0
broadcasts the prompt embeddings once and gathers every finished image
(uint8 RGB, 3 MiB / frame; the 512 KiB latent with --vae none) inside the
timed loop.  value = frames of all ranks / max rank time.  --cfg-parallel
(workload stream2-cfg): ranks 2k / 2k+1 carry the cond / uncond rows of the
same frames and exchange the noise predictions with one all_gather per frame
(parallel.CFGPairStreamDenoiser); the pairs shard the frames.

Also emitted: roofline of the dominant kernel (HIP events around each launch
on its stream inside the timed region), and a CPU baseline: the oracle's fp32
restatement on the host cores, bounded sample (see cpu_baseline()).
"""
from __future__ import annotations

import argparse
import contextlib
import ctypes
import json
import os
import sys
import threading
import time

# HIP hardware queues per process, set before HIP initialises (first torch.cuda call). RCCL's own
# streams (process group, N > 1) otherwise share HIP's default 4 queues with the model's two
# streams, the text-stream overlap (transformer._side_stream) serialises behind the image stream
# and every step costs ~9 % more: 290.8 vs 266.4 ms at N = 1 under --force-dist, 265.7 with 8
# queues (tools/dist_ab.sh, profiles/round2_s5_dist_ab.txt).
if int(os.environ.get("GPU_MAX_HW_QUEUES") or 0) < 8:  # raise an inherited 4, keep a larger value
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BF16 = torch.bfloat16
PEAK_BF16 = 2.5e15     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, spec)
PEAK_I8 = 5.0e15       # i8 MFMA: 2x bf16 per clock
S_NOISE = S_COND = 4096
S_TXT = 216
D_MODEL, F_MLP, N_LAYERS_FULL = 3072, 12288, 60

WORKLOADS = {
    "stream2": "lightning-2step stream-batch depth=2, cond-only, 1024x1024 (configs[2])",
    "stream2-int8": "int8 W8A8 linears, lightning-2step stream-batch depth=2, 1024x1024 (configs[3])",
    "stream2-cfg": "lightning-2step stream-batch depth=2 + true-CFG 4.0 (B=4), 1024x1024",
    "stream2-cfg-pairs": "lightning-2step stream-batch depth=2 + true-CFG 4.0, cond / uncond on the two ranks "
                         "of a pair (one all_gather per frame), pairs x frame shard, 1024x1024 (configs[4])",
    "cfg4": "4-step true-CFG 4.0 batched cond/uncond, 1024x1024 (configs[1])",
}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def _cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(sample_layers: int = 3):
    """The oracle (torch fp32 on the host cores) on BASELINE configs[0], the reference's own
    CPU-runnable case: 256x256 output (256 noise tokens) + the 1024^2-area condition image
    Edit-Plus always encodes (4096 tokens) + 216 text tokens, 2 steps, cond-only, random-init
    weights of the real width. Bounded sample: ``sample_layers`` of the 60 blocks (the blocks are
    identical in cost), scaled x60/sample_layers -> sec/image."""
    from oracle import dit_ref as R
    n = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(n)
    cfg = R.DiTConfig(num_layers=sample_layers)
    params = R.random_params(cfg, seed=0)
    g = torch.Generator().manual_seed(0)
    noise = torch.randn(1, 256, 64, generator=g).to(BF16)
    cond = torch.randn(1, S_COND, 64, generator=g).to(BF16)
    pe = torch.randn(1, S_TXT, cfg.joint_attention_dim, generator=g).to(BF16)
    shapes = [(1, 16, 16), (1, 64, 64)]
    t0 = time.time()
    R.denoise(params, cfg, noise, cond, pe, shapes, 2, emulate_bf16=False)
    dt = time.time() - t0
    scale = N_LAYERS_FULL / sample_layers
    sec_per_image = dt * scale
    flops = 2 * R.flops_per_forward(256 + S_COND, S_TXT, R.DiTConfig(), layers=sample_layers)
    rate = flops / dt  # FLOP/s the host cores reach on this path
    head = 2 * R.flops_per_forward(S_NOISE + S_COND, S_TXT, R.DiTConfig())
    return {"value": 1.0 / sec_per_image, "unit": "images/sec (256x256 output, configs[0])", "cores": n,
            "cpu": _cpu_model(), "kind": "port",
            "sample": (f"oracle fp32 torch-CPU, configs[0]: 256x256 output + 1024^2 condition image, 2 steps, "
                       f"cond-only, B=1, S=4568, DiT denoise loop only (no VAE / prompt encoder); "
                       f"{sample_layers} of 60 blocks timed ({dt:.1f} s), scaled x{scale:.0f} = "
                       f"{sec_per_image:.0f} s/image"),
            "sec_per_image": sec_per_image, "tflops": rate / 1e12,
            "headline_workload_estimate_sec_per_image": head / rate}


@contextlib.contextmanager
def _stdout_to_stderr():
    """Route C-level writes to fd 1 (library banners) to stderr for the duration."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        ctypes.CDLL(None).fflush(None)  # C stdio buffers go out while fd 1 is still stderr
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def attention_flops(rows: int, layers: int = 1) -> float:
    S = S_NOISE + S_COND + S_TXT
    return 4.0 * rows * S * S * D_MODEL * layers


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="stream2", choices=["stream2", "stream2-int8", "stream2-cfg", "cfg4"])
    ap.add_argument("--layers", type=int, default=60, help="debug only; the headline needs 60")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--vae", default="both", choices=["both", "decode", "none"],
                    help="VAE work inside the timed step: encode the uint8 RGB condition frame and decode "
                         "the finished one (both, the default), decode only (condition frames arrive as "
                         "latents), or none (DiT denoise alone)")
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary workloads (stream2-cfg, stream2-int8, stream2-cfg-pairs) that the "
                         "default stream2 run times after the headline")
    ap.add_argument("--secondary-timeout", type=float, default=240.0,
                    help="seconds the secondary workloads may take before the line is printed without them")
    ap.add_argument("--cfg-parallel", action="store_true",
                    help="workload stream2-cfg with the cond / uncond rows on the two ranks of a pair "
                         "(configs[4]); needs an even number of ranks, or one rank with --force-dist")
    ap.add_argument("--vl-per-frame", action="store_true",
                    help="re-encode the prompt with every frame through the HIP Qwen2.5-VL (7B widths, random "
                         "weights, vision cache off) inside the timed step, as qwen_realtime.py:247-255 does")
    ap.add_argument("--host-io", action="store_true",
                    help="PCIe-inclusive rate (never the headline): condition frames start in pinned host "
                         "memory and are copied to HBM inside the timed step, every finished image is "
                         "copied back to pinned host memory (the boundary a server hands over)")
    ap.add_argument("--no-qk-fusion", action="store_true",
                    help="A/B: image QKV GEMM and QK RMSNorm+RoPE as two launches")
    ap.add_argument("--no-log2q", action="store_true",
                    help="A/B: plain q and the softmax scale inside the attention (not log2-unit q)")
    ap.add_argument("--text-splits", default="1",
                    help="A/B: K ranges of the text-stream linears (1 = unsplit, the default; 0 = the "
                         "latency-oriented split rule ops.splitk_splits), or per linear as "
                         "'down=0,up=2' (qkv / out / up / down; unnamed ones unsplit)")
    ap.add_argument("--no-text-overlap", action="store_true",
                    help="A/B: run the text stream on the caller's stream, not on a second HIP stream")
    ap.add_argument("--eager-text-post", action="store_true",
                    help="A/B: the text stream's post-attention linears right after the attention, beside the "
                         "image stream's persistent GEMMs (default: behind them, beside the next block's QKV)")
    ap.add_argument("--no-mod-cache", action="store_true",
                    help="recompute the timestep MLP + modulation vectors every forward (A/B switch)")
    ap.add_argument("--no-batched-mod", action="store_true",
                    help="A/B: one modulation GEMV launch per block and stream, not one for all blocks")
    ap.add_argument("--force-dist", action="store_true",
                    help="debug: run the collective path (process group, broadcast, gather, "
                         "barriers, max-reduce) even at world size 1")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist_on = world > 1 or args.force_dist
    if args.cfg_parallel and (args.workload != "stream2-cfg" or not dist_on or (world > 1 and world % 2)):
        raise SystemExit("--cfg-parallel needs --workload stream2-cfg and an even number of ranks "
                         "(or one rank with --force-dist)")
    if dist_on:
        # RCCL prints a version banner on stdout when the communicator is created; stdout must
        # carry only the one JSON line, so fd 1 points at stderr until the first barrier is done
        with _stdout_to_stderr():
            dist.init_process_group("nccl", device_id=dev)
            dist.barrier()

    from qwen_image_edit_streamdiffusion_amd import (QwenImageTransformer2DModel, StreamBatchDenoiser,
                                                     QwenImageEditPlusPipeline)
    from qwen_image_edit_streamdiffusion_amd import parallel
    from qwen_image_edit_streamdiffusion_amd.vae import QwenImageVAEDecoder, QwenImageVAEEncoder
    t_build = time.time()
    model = QwenImageTransformer2DModel(num_layers=args.layers, device=dev).random_init_(seed=0)
    model.overlap_text_stream = not args.no_text_overlap
    model.fuse_qk_norm_rope = not args.no_qk_fusion
    model.log2q_attention = not args.no_log2q
    model.batched_modulation = not args.no_batched_mod
    model.cache_modulation = not args.no_mod_cache
    model.defer_text_post = not args.eager_text_post
    if "=" in args.text_splits:
        model.text_splits = {k: int(v) for k, v in (kv.split("=") for kv in args.text_splits.split(","))}
    else:
        model.text_splits = int(args.text_splits) or None
    decode = args.vae in ("both", "decode")
    encode = args.vae == "both"
    vae = QwenImageVAEDecoder(device=dev).random_init_(seed=1) if decode else None
    vae_enc = QwenImageVAEEncoder(device=dev).random_init_(seed=2) if encode else None
    torch.cuda.synchronize()
    log(f"[bench] model built in {time.time() - t_build:.1f}s, "
        f"{torch.cuda.memory_allocated() / 1e9:.1f} GB")

    # pair groups (CFG parallel) and the delivery group are created by every rank, in the same
    # order, before any of them is used
    pairs_possible = dist_on and (world == 1 or world % 2 == 0)
    pair_group = pair_role = pair_size = None
    deliver_group = None
    if pairs_possible and (args.cfg_parallel or (args.workload == "stream2" and not args.no_secondary and world > 1)):
        pair_group, pair_role, pair_size = parallel.make_pair_groups(world)
        deliver_group, _ = parallel.make_head_group(world, pair_size)

    # ---- synthetic inputs, resident in HBM before timing
    g = torch.Generator(device=dev).manual_seed(44)
    pe = torch.randn(1, S_TXT, 3584, generator=g, device=dev, dtype=BF16)
    ne = torch.randn(1, 211, 3584, generator=g, device=dev, dtype=BF16)  # shorter negative prompt
    if dist_on:
        dist.broadcast(pe, 0)  # prompt-embed cache filled once, from rank 0
        dist.broadcast(ne, 0)
    nf = 8

    def make_inputs(seed):
        gr = torch.Generator(device=dev).manual_seed(seed)
        conds = [torch.randn(1, S_COND, 64, generator=gr, device=dev, dtype=BF16) for _ in range(nf)]
        noises = [torch.randn(1, S_NOISE, 64, generator=gr, device=dev, dtype=BF16) for _ in range(nf)]
        frames = None
        if encode:  # condition frames as camera images: uint8 RGB 1024x1024, resident in HBM
            frames = [torch.randint(0, 256, (1, 1024, 1024, 3), generator=gr, device=dev, dtype=torch.uint8)
                      for _ in range(nf)]
        return conds, noises, frames

    host_io = args.host_io and encode and decode
    if args.host_io and not host_io:
        raise SystemExit("--host-io needs --vae both (RGB frames in and out)")
    out_host = torch.empty(1, 1024, 1024, 3, dtype=torch.uint8).pin_memory() if host_io else None

    vl_state = {}

    def get_vl():
        """Qwen2.5-VL-7B on the HIP path, random weights; synthetic processor outputs. Built once."""
        if "vl" in vl_state:
            return vl_state["vl"]
        from qwen_image_edit_streamdiffusion_amd.text_encoder import (QwenVLEncoder, TextEncoderConfig,
                                                                      random_state_dict, text_state_dict_shapes)
        from qwen_image_edit_streamdiffusion_amd.vision import VisionConfig, vision_state_dict_shapes
        tc, vc = TextEncoderConfig(), VisionConfig()
        sd = {"model.language_model." + k: v
              for k, v in random_state_dict(text_state_dict_shapes(tc), dev, 0).items()}
        sd.update({"model.visual." + k: v for k, v in random_state_dict(vision_state_dict_shapes(vc), dev, 1).items()})
        enc_vl = QwenVLEncoder(tc, vc, dev, vision_cache_size=0).load_state_dict(sd)
        del sd
        # Edit-Plus prompt: 64 template tokens (dropped), "Picture 1:" + a 392^2 condition image
        # (28x28 patches -> 196 image tokens) + the instruction: 280 tokens -> 216 embeddings
        ids = torch.randint(0, 150000, (64 + S_TXT,), generator=torch.Generator().manual_seed(5))
        ids[70:70 + 196] = enc_vl.image_token_id
        gv = torch.Generator(device=dev).manual_seed(6)
        pvs = [torch.randn(28 * 28, vc.patch_dim, generator=gv, device=dev) for _ in range(nf)]
        vl_state["vl"] = (enc_vl, ids, pvs, [(1, 28, 28)])
        return vl_state["vl"]

    def run(workload: str, steps: int, warmup: int, probe: bool, vl_on: bool = False):
        """Time `steps` steps of one workload on this rank's frames; returns its result dict
        (rank 0) with the whole-job value. vl_on: re-encode the prompt with every frame."""
        vl = get_vl() if vl_on else None
        int8 = workload == "stream2-int8"
        cfg_pairs = workload == "stream2-cfg-pairs"
        cfg_on = workload in ("stream2-cfg", "stream2-cfg-pairs")
        if int8 and not model.int8:
            model.quantize_int8()
        model.int8 = int8
        shard = rank // pair_size if cfg_pairs else rank  # both ranks of a pair push the same frames
        conds, noises, frames = make_inputs(1000 + shard)
        frames_host = [f.cpu().pin_memory() for f in frames] if host_io else None

        def frame(i):
            if host_io:
                return frames_host[i % nf].to(dev, non_blocking=True)
            return frames[i % nf]

        head = True  # this rank decodes and delivers finished frames
        if workload == "cfg4":  # 4-step true-CFG 4.0, batched cond/uncond (B=2), one image per step
            pipe = QwenImageEditPlusPipeline(model)
            pipe.vae, pipe.vae_encoder = vae, vae_enc
            rows_local = rows_total = 2
            fwd_per_step = 4

            def step(i):
                src = dict(image=frame(i)) if encode else dict(image_latents=conds[i % nf])
                return pipe(prompt_embeds=pe, negative_prompt_embeds=ne, latents=noises[i % nf], true_cfg_scale=4.0,
                            num_inference_steps=4, output_type="uint8" if decode else "latent", **src).images
        else:
            if cfg_pairs:
                eng = parallel.CFGPairStreamDenoiser(model, num_steps=2, true_cfg_scale=4.0, latent_hw=(64, 64),
                                                     cond_hw=(64, 64), role=pair_role, group=pair_group,
                                                     group_size=pair_size)
                head = pair_role == 0
            else:
                eng = StreamBatchDenoiser(model, num_steps=2, true_cfg_scale=4.0 if cfg_on else 1.0,
                                          latent_hw=(64, 64), cond_hw=(64, 64))
            eng.set_conditions(pe, None, ne if cfg_on else None)
            rows_local = eng.rows
            rows_total = 4 if cfg_on else 2
            fwd_per_step = 1

            def step(i):
                cond = vae_enc.encode(frame(i)) if encode else conds[i % nf]
                if vl is not None:  # this frame's own prompt embedding: vision tower + language model
                    enc_vl, ids, pvs, grid = vl
                    h = enc_vl(ids, pvs[i % nf], grid)[64:]
                    return eng.push(noises[i % nf], cond, prompt_embeds=h, negative_prompt_embeds=None)
                return eng.push(noises[i % nf], cond)

        n_heads = world // pair_size if cfg_pairs else world
        grp = deliver_group if cfg_pairs else None
        gather_buf = None
        if dist_on and rank == 0:
            gather_buf = [torch.empty(1, 1024, 1024, 3, dtype=torch.uint8, device=dev) if decode else
                          torch.empty(1, S_NOISE, 64, dtype=BF16, device=dev) for _ in range(n_heads)]

        def deliver(res):
            if not head:  # the uncond rank of a pair holds the same latents; its partner delivers them
                return
            out = res[1] if isinstance(res, tuple) else res
            if decode and out.dtype != torch.uint8:  # stream engine: decode the frame that completed
                out = vae.decode(out, 128, 128)
            if host_io:  # D2H of the finished image, ordered on the compute stream
                out_host.copy_(out.reshape(out_host.shape), non_blocking=True)
            if dist_on:
                parallel.deliver_to_root(out, gather_buf, True, grp)

        for i in range(warmup):
            r = step(i)
            if r is not None:
                deliver(r)
        if workload != "cfg4" and warmup < 2:
            r = step(warmup)  # fill the 2-deep pipeline
            warmup += 1
            if r is not None:
                deliver(r)
        torch.cuda.synchronize()
        model.probe = {k: [] for k in ("attention", "mlp_up")} if probe else None
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.time()
        done = 0
        for i in range(steps):
            r = step(warmup + i)
            if r is not None:
                done += 1 if head else 0
                deliver(r)
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        el = time.time() - t0
        if dist_on:
            tt = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = tt.item()
            dn = torch.tensor([done], device=dev, dtype=torch.float64)
            dist.all_reduce(dn, op=dist.ReduceOp.SUM)
            done = int(dn.item())
        model_probe, model.probe = model.probe, None

        images = done
        S = S_NOISE + S_COND + S_TXT
        flops_fwd = model.flops_per_forward(S_NOISE + S_COND, S_TXT, B=rows_total)
        attn_fwd = attention_flops(rows_total, args.layers)
        vae_flops = (vae.flops(128, 128) if decode else 0.0) + (vae_enc.flops(1024, 1024) if encode else 0.0)
        flops_img = flops_fwd * fwd_per_step + vae_flops
        # time the MFMA roof allows per image: int8 runs the linears at the i8 rate, the attention
        # and the VAE at the bf16 rate (blended roof)
        lin_peak = PEAK_I8 if int8 else PEAK_BF16
        roof_s_img = ((flops_fwd - attn_fwd) * fwd_per_step / lin_peak +
                      (attn_fwd * fwd_per_step + vae_flops) / PEAK_BF16)
        kernels = {}
        if model_probe:
            alg = {"attention": attention_flops(rows_local),
                   "mlp_up": 2.0 * rows_local * (S_NOISE + S_COND) * F_MLP * D_MODEL}
            for k, evs in model_probe.items():
                if not evs:
                    continue
                ms = [a.elapsed_time(b) for a, b in evs]
                avg = sum(ms) / len(ms)
                kpeak = PEAK_BF16 if k == "attention" else lin_peak
                kernels[k] = {"avg_ms": avg, "launches": len(ms), "total_ms": sum(ms),
                              "tflops": alg[k] / (avg * 1e-3) / 1e12, "frac": alg[k] / (avg * 1e-3) / kpeak}
        roof = None
        if kernels:
            dom = max(kernels, key=lambda k: kernels[k]["total_ms"])
            kd = kernels[dom]
            kpeak = PEAK_BF16 if dom == "attention" else lin_peak
            # HBM bytes per launch of this kernel: NOT measured by this run (PMC counters need
            # rocprofv3 passes of their own); the figure of the committed passes over this same
            # command (tools/measure.sh -> profiles/pmc_traffic.json), for the headline workload only
            traffic = None
            tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
            if os.path.exists(tf) and workload == "stream2":
                t = json.load(open(tf)).get("traffic_per_launch", {}).get(dom)
                traffic = t and t.get("hbm_bytes_per_launch")
            roof = {"bound": "mfma", "kernel": dom, "achieved": kd["tflops"], "peak": kpeak / 1e12,
                    "unit": "TFLOP/s", "frac": kd["frac"], "traffic": traffic,
                    "traffic_source": "profiles/pmc_traffic.json (separate rocprofv3 --pmc passes)" if traffic else None,
                    "flops_per_launch": (attention_flops(rows_local) if dom == "attention"
                                         else 2.0 * rows_local * (S_NOISE + S_COND) * F_MLP * D_MODEL),
                    "avg_launch_ms": kd["avg_ms"]}
        par = "single"
        if world > 1 or cfg_pairs:
            par = (f"cfg-pair x{pair_size} x frame-shard x{n_heads}" if cfg_pairs else f"frame-shard x{world}")
        return {
            "value": images / el, "unit": "images/sec", "steps": steps, "warmup": warmup,
            "ms_per_step": el / steps * 1e3, "sec_per_image": el * n_heads / max(images, 1),
            "dtype": "int8" if int8 else "bf16",
            "config": {"workload": WORKLOADS[workload] + (", prompt re-encoded per frame by Qwen2.5-VL-7B "
                                                          "(random weights)" if vl is not None else ""),
                       "model": "Qwen-Image-Edit-2509 DiT (60 blocks, D=3072)" +
                                (" + AutoencoderKLQwenImage " + ("encoder/decoder" if encode else "decoder")
                                 if decode else ""),
                       "global_batch": rows_local * world, "seq_len": S, "layers": args.layers,
                       "parallelism": par},
            # fraction of the MFMA roof over the whole step: bf16 peak; int8: blended roof (linears
            # at the i8 rate, attention + VAE at the bf16 rate)
            "mfma_util": roof_s_img * images / el / world,
            "tflops_per_gpu": flops_img * images / el / world / 1e12,
            "roofline": roof, "kernels": kernels,
        }

    wl = "stream2-cfg-pairs" if args.cfg_parallel else args.workload
    res = run(wl, args.steps, args.warmup, not args.no_probe, args.vl_per_frame)

    def emit(secondary, cpu):
        line = {
            "metric": "images/sec, 1024x1024 2-step Lightning edit (" +
                      ("Qwen2.5-VL prompt encode + " if args.vl_per_frame else "") +
                      ("VAE encode + " if encode else "") + "DiT denoise" + (" + VAE decode" if decode else "") +
                      (", PCIe-inclusive: pinned host RGB in/out)" if host_io else ")"),
            "value": res["value"], "unit": "images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": res["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": res["dtype"],
            "data": "synthetic (randn latents/cond/prompt embeds; random-init weights of the real "
                    "60-block architecture)",
            "config": res["config"],
            "sec_per_image": res["sec_per_image"],
            "host_io": host_io,
            "hip_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES") or 0),
            "mfma_util": res["mfma_util"],
            "tflops_per_gpu": res["tflops_per_gpu"],
            "roofline": res["roofline"], "kernels": res["kernels"], "cpu_baseline": cpu,
            "secondary": secondary or None,
        }
        print(json.dumps(line), flush=True)

    # The secondary workloads must never cost the headline: every rank arms a timer before them;
    # if they have not finished by then (a rank that died, a collective that never completes),
    # rank 0 prints the line with what it has and every rank leaves without waiting for the rest.
    secondary = {}
    finished = threading.Event()

    def watchdog():
        if finished.wait(args.secondary_timeout):
            return
        if rank == 0:
            secondary.setdefault("error", f"secondary workloads not finished after {args.secondary_timeout:g} s; "
                                          "abandoned")
            emit(dict(secondary), None)
        sys.stdout.flush()
        os._exit(0)

    if args.workload == "stream2" and not args.no_secondary and not args.vl_per_frame and not host_io:
        threading.Thread(target=watchdog, daemon=True).start()
        names = ["stream2-cfg"]
        if pair_group is not None and world > 1:
            names.append("stream2-cfg-pairs")
        if world == 1:
            names.append("stream2-vl-per-frame")  # the headline with the prompt re-encoded per frame
        names.append("stream2-int8")  # last: it quantises the model's linears
        for name in names:
            try:
                if name == "stream2-vl-per-frame":
                    r = run("stream2", args.steps, min(args.warmup, 2), not args.no_probe, True)
                else:
                    r = run(name, args.steps, min(args.warmup, 2), not args.no_probe)
                secondary[name] = {k: r[k] for k in ("value", "unit", "ms_per_step", "sec_per_image", "dtype",
                                                     "mfma_util", "tflops_per_gpu", "roofline", "config")}
            except Exception as e:  # reported, never fatal to the headline (the watchdog covers the peers)
                secondary[name] = {"error": repr(e)}
                if dist_on:
                    break  # the ranks are out of step now: no further collectives

    finished.set()
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline()
        except Exception as e:  # reported, never fatal to the GPU number
            cpu = {"error": repr(e)}

    if rank == 0:
        emit(secondary, cpu)
    if dist_on:
        if any("error" in v for v in secondary.values() if isinstance(v, dict)):
            sys.stdout.flush()
            os._exit(0)  # a secondary workload failed mid-way: the group may not tear down cleanly
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
