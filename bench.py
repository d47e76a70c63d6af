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
path: the prompt embedding comes from the prompt cache.

Multi-GPU (torch.distributed.run, one process per GPU, RCCL): each rank runs
its own stream engine on its own frames (frame shard, weak scaling); rank 0
broadcasts the prompt embeddings once and gathers every finished image
(uint8 RGB, 3 MiB / frame; the 512 KiB latent with --no-decode) inside the
timed loop.  value = frames of all ranks / max
rank time.

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
import time

# HIP hardware queues per process, set before HIP initialises (first torch.cuda call). RCCL's own
# streams (process group, N > 1) otherwise share HIP's default 4 queues with the model's two
# streams, the text-stream overlap (transformer._side_stream) serialises behind the image stream
# and every step costs ~9 % more: 290.8 vs 266.4 ms at N = 1 under --force-dist, 265.7 with 8
# queues (tools/dist_ab.sh, profiles/round2_s5_dist_ab.txt).
if int(os.environ.get("GPU_MAX_HW_QUEUES") or 0) < 8:  # raise an inherited 4, keep a larger value
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import torch  # noqa: E402
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BF16 = torch.bfloat16
PEAK_BF16 = 2.5e15     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, spec)
PEAK_I8 = 5.0e15       # i8 MFMA: 2x bf16 per clock
S_NOISE = S_COND = 4096
S_TXT = 216


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_baseline(decode: bool = True, encode: bool = True):
    """Oracle (torch fp32 on the host cores) on a bounded sample of the SAME
    workload: one B=2 stream-batch forward with 1 of the 60 blocks (prologue +
    block + head) at full size, scaled x60 -> sec/image (1 forward/image)."""
    from oracle import dit_ref as R
    n = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(n)
    cfg = R.DiTConfig(num_layers=1)
    params = R.random_params(cfg, seed=0)
    g = torch.Generator().manual_seed(0)
    hs = torch.randn(2, S_NOISE + S_COND, 64, generator=g).to(BF16)
    enc = torch.randn(2, S_TXT, cfg.joint_attention_dim, generator=g).to(BF16)
    t = R.model_timestep(torch.tensor([1000.0, 20.0]))
    shapes = [(1, 64, 64), (1, 64, 64)]
    t0 = time.time()
    R.transformer_forward(params, cfg, hs, enc, t, shapes, [S_TXT, S_TXT], emulate_bf16=False)
    dt = time.time() - t0
    sec_per_image = dt * 60
    sample = (f"oracle fp32 torch-CPU: one B=2 stream-batch forward with 1 of 60 DiT blocks at full 1024^2 size "
              f"({dt:.1f} s), scaled x60")
    if decode:  # VAE decode of the real architecture at 32x32 latents (256^2), scaled by FLOPs to 128x128
        from oracle import vae_ref as V
        vc = V.VAEConfig()
        vp = V.random_params(vc, 1)
        packed = torch.randn(1, 256, 64, generator=g).to(BF16)
        t0 = time.time()
        V.decode(vp, packed, 32, 32, vc, emulate_bf16=False)
        dv = (time.time() - t0) * V.decode_flops(vc, 128, 128) / V.decode_flops(vc, 32, 32)
        sec_per_image += dv
        sample += f" + VAE decode (256^2 sample, FLOP-scaled to 1024^2: {dv:.1f} s)"
    if encode:  # VAE encode of a 256^2 frame, scaled by FLOPs to 1024^2
        from oracle import vae_ref as V
        vc = V.VAEConfig()
        ep = V.random_encoder_params(vc, 2)
        rgb = torch.randint(0, 256, (1, 256, 256, 3), generator=g, dtype=torch.uint8)
        t0 = time.time()
        V.encode(ep, rgb, vc, emulate_bf16=False)
        from qwen_image_edit_streamdiffusion_amd.vae import QwenImageVAEEncoder, VAEConfig
        ef = QwenImageVAEEncoder(VAEConfig(), "cpu")
        de = (time.time() - t0) * ef.flops(1024, 1024) / ef.flops(256, 256)
        sec_per_image += de
        sample += f" + VAE encode (256^2 sample, FLOP-scaled: {de:.1f} s)"
    return {"value": 1.0 / sec_per_image, "unit": "images/sec", "cores": n, "kind": "port",
            "sample": sample + f" = {sec_per_image:.0f} s/image", "sec_per_image": sec_per_image}


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
    if dist_on:
        # RCCL prints a version banner on stdout when the communicator is created; stdout must
        # carry only the one JSON line, so fd 1 points at stderr until the first barrier is done
        with _stdout_to_stderr():
            dist.init_process_group("nccl", device_id=dev)
            dist.barrier()

    from qwen_image_edit_streamdiffusion_amd import (QwenImageTransformer2DModel, StreamBatchDenoiser,
                                                     QwenImageEditPlusPipeline)
    from qwen_image_edit_streamdiffusion_amd.vae import QwenImageVAEDecoder, QwenImageVAEEncoder
    t_build = time.time()
    model = QwenImageTransformer2DModel(num_layers=args.layers, device=dev).random_init_(seed=0)
    if args.workload == "stream2-int8":
        model.quantize_int8()
    model.overlap_text_stream = not args.no_text_overlap
    model.fuse_qk_norm_rope = not args.no_qk_fusion
    model.log2q_attention = not args.no_log2q
    model.batched_modulation = not args.no_batched_mod
    model.cache_modulation = not args.no_mod_cache
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

    # ---- synthetic inputs, resident in HBM before timing
    g = torch.Generator(device=dev).manual_seed(44)
    pe = torch.randn(1, S_TXT, 3584, generator=g, device=dev, dtype=BF16)
    if dist_on:
        dist.broadcast(pe, 0)  # prompt-embed cache filled once, from rank 0
    gr = torch.Generator(device=dev).manual_seed(1000 + rank)
    nf = 8
    conds = [torch.randn(1, S_COND, 64, generator=gr, device=dev, dtype=BF16) for _ in range(nf)]
    noises = [torch.randn(1, S_NOISE, 64, generator=gr, device=dev, dtype=BF16) for _ in range(nf)]
    if encode:  # condition frames as camera images: uint8 RGB 1024x1024, resident in HBM
        frames = [torch.randint(0, 256, (1, 1024, 1024, 3), generator=gr, device=dev, dtype=torch.uint8)
                  for _ in range(nf)]
    host_io = args.host_io and encode and decode
    if args.host_io and not host_io:
        raise SystemExit("--host-io needs --vae both (RGB frames in and out)")
    if host_io:  # the frames live in pinned host memory; the step uploads them (stream-ordered)
        frames_host = [f.cpu().pin_memory() for f in frames]
        out_host = torch.empty(1, 1024, 1024, 3, dtype=torch.uint8).pin_memory()

    def frame(i):
        if host_io:
            return frames_host[i % nf].to(dev, non_blocking=True)
        return frames[i % nf]

    probe_keys = ("attention", "mlp_up")
    if args.workload.startswith("stream2"):
        cfg_on = args.workload == "stream2-cfg"
        eng = StreamBatchDenoiser(model, num_steps=2, true_cfg_scale=4.0 if cfg_on else 1.0,
                                  latent_hw=(64, 64), cond_hw=(64, 64))
        if cfg_on:  # true CFG 4.0 with a shorter negative prompt: cond + uncond rows, B = 4
            ne = torch.randn(1, 211, 3584, generator=g, device=dev, dtype=BF16)
            eng.set_conditions(pe, None, ne)
        else:
            eng.set_conditions(pe)
        rows = 4 if cfg_on else 2
        fwd_per_step = 1

        def step(i):
            cond = vae_enc.encode(frame(i)) if encode else conds[i % nf]
            return eng.push(noises[i % nf], cond)
    else:  # cfg4: 4-step true-CFG 4.0, batched cond/uncond (B=2), one image per step
        pipe = QwenImageEditPlusPipeline(model)
        ne = torch.randn(1, 211, 3584, generator=g, device=dev, dtype=BF16)
        rows = 2
        fwd_per_step = 4

        pipe.vae, pipe.vae_encoder = vae, vae_enc

        def step(i):
            src = dict(image=frame(i)) if encode else dict(image_latents=conds[i % nf])
            return pipe(prompt_embeds=pe, negative_prompt_embeds=ne, latents=noises[i % nf], true_cfg_scale=4.0,
                        num_inference_steps=4, output_type="uint8" if decode else "latent", **src).images

    gather_buf = None
    if dist_on and rank == 0:
        gather_buf = [torch.empty(1, 1024, 1024, 3, dtype=torch.uint8, device=dev) if decode else
                      torch.empty(1, S_NOISE, 64, dtype=BF16, device=dev) for _ in range(world)]

    def deliver(res):
        out = res[1] if isinstance(res, tuple) else res
        if decode and out.dtype != torch.uint8:  # stream engine: decode the frame that completed
            out = vae.decode(out, 128, 128)
        if host_io:  # D2H of the finished image, ordered on the compute stream
            out_host.copy_(out.reshape(out_host.shape), non_blocking=True)
        if dist_on:
            dist.gather(out, gather_buf if rank == 0 else None, dst=0)

    for i in range(args.warmup):
        r = step(i)
        if r is not None:
            deliver(r)
    if args.workload.startswith("stream2") and args.warmup < 2:
        step(args.warmup)  # fill the 2-deep pipeline
    torch.cuda.synchronize()
    if not args.no_probe:
        model.probe = {k: [] for k in probe_keys}
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.time()
    done = 0
    for i in range(args.steps):
        r = step(args.warmup + i)
        if r is not None:
            done += 1
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
    value = images / el
    sec_per_image = el * world / max(images, 1)
    S = S_NOISE + S_COND + S_TXT
    flops_fwd = model.flops_per_forward(S_NOISE + S_COND, S_TXT, B=rows)
    flops_img = (flops_fwd * fwd_per_step + (vae.flops(128, 128) if decode else 0.0) +
                 (vae_enc.flops(1024, 1024) if encode else 0.0))
    peak = PEAK_I8 if args.workload.endswith("int8") else PEAK_BF16

    kernels = {}
    if model_probe:
        D, F = 3072, 12288
        alg = {"attention": 4.0 * rows * S * S * D,
               "mlp_up": 2.0 * rows * (S_NOISE + S_COND) * F * D}
        for k, evs in model_probe.items():
            if not evs:
                continue
            ms = [a.elapsed_time(b) for a, b in evs]
            avg = sum(ms) / len(ms)
            kpeak = PEAK_BF16 if k == "attention" else peak
            kernels[k] = {"avg_ms": avg, "launches": len(ms), "total_ms": sum(ms),
                          "tflops": alg[k] / (avg * 1e-3) / 1e12, "frac": alg[k] / (avg * 1e-3) / kpeak}
    roof = None
    if kernels:
        dom = max(kernels, key=lambda k: kernels[k]["total_ms"])
        kd = kernels[dom]
        kpeak = PEAK_BF16 if dom == "attention" else peak
        # HBM bytes per launch of this kernel from the committed rocprofv3 FETCH_SIZE /
        # WRITE_SIZE passes (tools/measure.sh + tools/summarize_profile.py), if present
        traffic = None
        tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(tf) and args.workload == "stream2":
            t = json.load(open(tf)).get("traffic_per_launch", {}).get(dom)
            traffic = t and t.get("hbm_bytes_per_launch")
        roof = {"bound": "mfma", "kernel": dom, "achieved": kd["tflops"], "peak": kpeak / 1e12,
                "unit": "TFLOP/s", "frac": kd["frac"], "traffic": traffic,
                "flops_per_launch": (4.0 * rows * S * S * 3072 if dom == "attention"
                                     else 2.0 * rows * (S_NOISE + S_COND) * 12288 * 3072),
                "avg_launch_ms": kd["avg_ms"]}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(decode, encode)
        except Exception as e:  # reported, never fatal to the GPU number
            cpu = {"error": repr(e)}

    if rank == 0:
        workload = {"stream2": "lightning-2step stream-batch depth=2, cond-only, 1024x1024 (configs[2])",
                    "stream2-int8": "int8 W8A8 linears, lightning-2step stream-batch depth=2, 1024x1024 "
                                    "(configs[3])",
                    "stream2-cfg": "lightning-2step stream-batch depth=2 + true-CFG 4.0 (B=4), 1024x1024",
                    "cfg4": "4-step true-CFG 4.0 batched cond/uncond, 1024x1024 (configs[1])"}[args.workload]
        line = {
            "metric": "images/sec, 1024x1024 2-step Lightning edit (" +
                      ("VAE encode + " if encode else "") + "DiT denoise" + (" + VAE decode" if decode else "") +
                      (", PCIe-inclusive: pinned host RGB in/out)" if host_io else ")"),
            "value": value, "unit": "images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "int8" if args.workload.endswith("int8") else "bf16",
            "data": "synthetic (randn latents/cond/prompt embeds; random-init weights of the real "
                    "60-block architecture)",
            "config": {"workload": workload,
                       "model": "Qwen-Image-Edit-2509 DiT (60 blocks, D=3072)" +
                                (" + AutoencoderKLQwenImage " + ("encoder/decoder" if encode else "decoder")
                                 if decode else ""),
                       "global_batch": rows * world, "seq_len": S, "layers": args.layers,
                       "parallelism": f"frame-shard x{world}" if world > 1 else "single"},
            "sec_per_image": sec_per_image,
            "host_io": host_io,
            "hip_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES") or 0),
            "mfma_util": flops_img * images / el / (peak * world),
            "tflops_per_gpu": flops_img * images / el / world / 1e12,
            "roofline": roof, "kernels": kernels, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
