"""Stream-batch denoising: the replacement for qwen_realtime.py's denoise loop.

Reference: ``StreamConfig`` (qwen_realtime.py:39-66), ``CachedConditions``
(69-89; prompt-keyed ``is_valid`` 82-89), the never-called ``prepare_latent``
(201-224: prev-latent + 0.05*noise, keyframe every 20) and ``process_frame``
(226-268), which re-runs the whole diffusers pipeline per frame.
The reference holds no code for "stream batch depth=2"; it is defined here, following
StreamDiffusion (README.md:3, 207-217).

Design (MI355X-first): with N denoise steps the engine keeps N frames in
flight in one batched forward -- slot k holds a frame at step k (sigma_k), each
batch row carries its own timestep (per-row temb -> per-row AdaLN
modulation), and each row gets its own Euler dt.  After the pipeline fills,
every forward finishes one frame: N forwards per image become 1.  With true CFG
the cond/uncond rows of every slot ride in the same forward (batched CFG),
B = 2N.  Prompt embeddings are cached by prompt (CachedConditions) and the
padded text batch is built once per prompt, not per frame.

Because every libqie kernel computes each batch row independently with a
fixed reduction order, a frame's result is bitwise identical to a serial
N-step denoise of that frame (tests/test_gpu_pipeline.py checks this).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

from . import ops
from .scheduler import FlowMatchEulerDiscreteScheduler, calculate_shift, model_timesteps
from .transformer import QwenImageTransformer2DModel

BF16 = torch.bfloat16


@dataclass
class StreamConfig:
    """Fields of qwen_realtime.py:39-66 plus the stream-batch knobs."""

    width: int = 512
    height: int = 512
    num_inference_steps: int = 4
    guidance_scale: float = 1.0
    true_cfg_scale: float = 4.0
    noise_strength: float = 0.05
    keyframe_interval: int = 20
    camera_id: int = 0
    target_fps: int = 15
    model_name: str = "Qwen/Qwen-Image-Edit-2509"
    dtype: torch.dtype = BF16
    use_xformers: bool = True       # accepted, irrelevant on this path
    use_torch_compile: bool = True  # accepted, no tracing compiler on this path
    use_cuda_graph: bool = False
    # build additions: output/cond latent grids (Edit-Plus defaults to a 1024^2 area)
    output_size: Tuple[int, int] = (1024, 1024)
    cond_size: Tuple[int, int] = (1024, 1024)
    stream_batch: bool = True
    use_prev_latent: bool = False


class CachedConditions:
    """Prompt-keyed cache of text conditioning (qwen_realtime.py:69-89), now
    actually holding the embeddings and the padded batched text tensor."""

    def __init__(self):
        self.prompt: Optional[str] = None
        self.prompt_embeds: Optional[torch.Tensor] = None
        self.prompt_embeds_mask: Optional[torch.Tensor] = None
        self.negative_prompt_embeds: Optional[torch.Tensor] = None
        self.negative_prompt_embeds_mask: Optional[torch.Tensor] = None
        self.reference_latents: Optional[torch.Tensor] = None
        self.reference_key: Optional[str] = None

    @staticmethod
    def image_key(image) -> Optional[str]:
        """Content key of the image the prompt was encoded with (None: no image block)."""
        if image is None:
            return None
        import hashlib
        h = hashlib.sha1()
        if isinstance(image, torch.Tensor):  # raw bytes: numpy has no bfloat16
            h.update(f"{tuple(image.shape)}{image.dtype}".encode())
            h.update(image.detach().contiguous().view(-1).view(torch.uint8).cpu().numpy().tobytes())
        else:
            im = image.convert("RGB")
            h.update(str(im.size).encode())
            h.update(im.tobytes())
        return h.hexdigest()

    def is_valid(self, prompt: str, reference_image=None) -> bool:
        """qwen_realtime.py:82-89 keys on the prompt; the image block of the prompt is part of
        the key too, so re-encoding with a new frame is not served from the cache."""
        return (self.prompt_embeds is not None and prompt == self.prompt
                and self.image_key(reference_image) == self.reference_key)


class HipStreamCompute:
    """The arithmetic a stream engine needs, on the HIP path (libqie kernels behind the transformer
    and ``ops``). The engines take any object with these methods, so their slot / exchange logic
    also runs on the CPU with a checker's arithmetic behind it (tests, gloo)."""

    def __init__(self, transformer: QwenImageTransformer2DModel):
        self.tf = transformer
        self.device = transformer.device

    def empty(self, *shape) -> torch.Tensor:
        return torch.empty(*shape, dtype=BF16, device=self.device)

    def zeros(self, *shape) -> torch.Tensor:
        return torch.zeros(*shape, dtype=BF16, device=self.device)

    def timesteps(self, per_row: List[float]) -> torch.Tensor:
        return model_timesteps(per_row, self.device)

    def forward(self, inp, enc, t_rows, img_shapes, txt_lens) -> torch.Tensor:
        return self.tf(inp, enc, None, t_rows, img_shapes, txt_lens, return_dict=False)[0]

    def cfg_combine(self, cond, uncond, scale: float, out) -> torch.Tensor:
        return ops.cfg_combine(cond, uncond, scale, out=out)

    def euler_step(self, x, v, dts: List[float], out) -> None:
        ops.euler_step(x, v, dts, out)

    def copy(self, src, dst) -> None:
        ops.copy_batched(src, dst)


class StreamBatchDenoiser:
    """N frames in flight, one batched DiT forward per pushed frame.

    Row layout of the model input: one block of ``depth`` rows (slot k = a frame at step k) per
    CFG branch this engine computes -- ``branches`` = [0] (cond only), or [0, 1] with true CFG
    (cond rows then uncond rows: batched CFG). A subclass that computes a single branch and
    exchanges the predictions with its partner (parallel.CFGPairStreamDenoiser) overrides
    ``_local_branches`` and ``_exchange``."""

    def __init__(self, transformer: Optional[QwenImageTransformer2DModel], num_steps: int = 2,
                 true_cfg_scale: float = 1.0, latent_hw: Tuple[int, int] = (64, 64),
                 cond_hw: Tuple[int, int] = (64, 64),
                 scheduler: Optional[FlowMatchEulerDiscreteScheduler] = None, compute=None):
        self.tf = transformer
        self.cx = compute if compute is not None else HipStreamCompute(transformer)
        self.depth = int(num_steps)
        self.cfg_scale = float(true_cfg_scale)
        self.lh, self.lw = latent_hw
        self.ch, self.cw = cond_hw
        self.S_noise = self.lh * self.lw
        self.S_cond = self.ch * self.cw
        self.S_img = self.S_noise + self.S_cond
        sch = scheduler or FlowMatchEulerDiscreteScheduler()
        c = sch.config
        mu = calculate_shift(self.S_noise, c.base_image_seq_len, c.max_image_seq_len, c.base_shift,
                             c.max_shift)
        sch.set_timesteps(self.depth, mu=mu)
        self.sigmas = sch.sigmas.clone()
        self.timesteps = sch.timesteps.tolist()
        self.dts = [sch.dt(i) for i in range(self.depth)]
        self.cfg = False
        self.branches: List[int] = [0]
        self.stage: List[int] = [-1] * self.depth  # -1 = empty slot
        self.frame_id: List[int] = [-1] * self.depth
        self._next_frame = 0
        self._inp: Optional[torch.Tensor] = None
        self._enc = None
        self._txt_lens = None
        self._comb = None
        self._tcache: Dict[Tuple[int, ...], torch.Tensor] = {}
        self.img_shapes = [[(1, self.lh, self.lw), (1, self.ch, self.cw)]]

    @property
    def rows(self) -> int:
        return self.depth * len(self.branches)

    def _local_branches(self) -> List[int]:
        """CFG branches whose rows this engine computes (0 = cond, 1 = uncond)."""
        return [0, 1] if self.cfg else [0]

    def set_conditions(self, prompt_embeds: torch.Tensor, prompt_embeds_mask: Optional[torch.Tensor] = None,
                       negative_prompt_embeds: Optional[torch.Tensor] = None,
                       negative_prompt_embeds_mask: Optional[torch.Tensor] = None):
        """Cache the (padded, batched) text conditioning once per prompt. Both branches' text is
        padded to the longer of the two, whichever branches this engine computes, so a branch's
        rows see the same shapes in every engine layout."""
        dev = self.cx.device
        pe = prompt_embeds.to(dev, BF16)
        if pe.dim() == 2:
            pe = pe[None]
        lc = int(prompt_embeds_mask.sum()) if prompt_embeds_mask is not None else pe.shape[1]
        self.cfg = negative_prompt_embeds is not None and self.cfg_scale > 1.0
        embeds, lens = [pe], [lc]
        if self.cfg:
            ne = negative_prompt_embeds.to(dev, BF16)
            if ne.dim() == 2:
                ne = ne[None]
            ln = int(negative_prompt_embeds_mask.sum()) if negative_prompt_embeds_mask is not None else ne.shape[1]
            embeds.append(ne)
            lens.append(ln)
        S_txt = max(e.shape[1] for e in embeds)
        self.branches = self._local_branches()
        D = self.depth
        enc = self.cx.zeros(self.rows, S_txt, pe.shape[2])
        tl: List[int] = []
        for j, br in enumerate(self.branches):
            enc[j * D:(j + 1) * D, : embeds[br].shape[1]] = embeds[br][0]
            tl += [lens[br]] * D
        self._enc, self._txt_lens = enc, tl
        self._inp = self.cx.zeros(self.rows, self.S_img, 64)
        self._comb = self.cx.empty(D, self.S_noise, 64) if self.cfg else None
        self.stage = [-1] * D
        self.frame_id = [-1] * D

    def _t_rows(self) -> torch.Tensor:
        st = tuple(max(s, 0) for s in self.stage)
        key = st + (len(self.branches),)
        t = self._tcache.get(key)
        if t is None:
            per_slot = [self.timesteps[s] for s in st]
            t = self.cx.timesteps(per_slot * len(self.branches))
            self._tcache[key] = t
        return t

    def _set_slot_text(self, slot: int, embeds: List[Optional[torch.Tensor]]):
        """Per-frame text conditioning: overwrite the text rows of ``slot`` (the reference's
        realtime call re-encodes the prompt with every frame, qwen_realtime.py:247-255).
        ``embeds`` = [cond, uncond]; each must fit the text length set_conditions() allocated."""
        D, S_txt = self.depth, self._enc.shape[1]
        for j, br in enumerate(self.branches):
            e = embeds[br]
            if e is None:
                continue
            e = e.to(self.cx.device, BF16)
            e = e[0] if e.dim() == 3 else e
            if e.shape[0] > S_txt:
                raise ValueError(f"per-frame prompt has {e.shape[0]} tokens; set_conditions() sized the text "
                                 f"rows for {S_txt}")
            row = self._enc[j * D + slot]
            row.zero_()
            row[: e.shape[0]] = e
            self._txt_lens[j * D + slot] = int(e.shape[0])

    def begin(self, noise: Optional[torch.Tensor], cond_latents: Optional[torch.Tensor],
              prompt_embeds: Optional[torch.Tensor] = None,
              negative_prompt_embeds: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
        """First half of push(): insert the frame and run the batched forward of this engine's
        branches. Returns the local noise predictions [len(branches) * depth, S_noise, 64]
        (a view of the model output), or None when no frame is in flight."""
        if self._inp is None:
            raise RuntimeError("call set_conditions() first")
        D, cx = self.depth, self.cx
        if noise is not None:
            slot = self.stage.index(-1) if -1 in self.stage else None
            if slot is None:
                raise RuntimeError("no free slot (internal invariant broken)")
            inp = self._inp
            cx.copy(noise.reshape(1, self.S_noise, 64).to(BF16), inp[slot:slot + 1, : self.S_noise])
            cx.copy(cond_latents.reshape(1, self.S_cond, 64).to(BF16), inp[slot:slot + 1, self.S_noise:])
            for j in range(1, len(self.branches)):
                cx.copy(inp[slot:slot + 1], inp[j * D + slot:j * D + slot + 1])
            if prompt_embeds is not None or negative_prompt_embeds is not None:
                self._set_slot_text(slot, [prompt_embeds, negative_prompt_embeds])
            self.stage[slot] = 0
            self.frame_id[slot] = self._next_frame
            self._next_frame += 1
        if all(s < 0 for s in self.stage):
            return None
        out = cx.forward(self._inp, self._enc, self._t_rows(), self.img_shapes * self.rows, self._txt_lens)
        return out[:, : self.S_noise]

    def _exchange(self, v_local: torch.Tensor) -> List[torch.Tensor]:
        """[cond, uncond] predictions, each [depth, S_noise, 64]. Here both are local rows."""
        D = self.depth
        return [v_local[j * D:(j + 1) * D] for j in range(len(self.branches))]

    def finish(self, parts: List[torch.Tensor]) -> Optional[Tuple[int, torch.Tensor]]:
        """Second half of push(): true-CFG combine of [cond, uncond] (when on), per-row Euler
        step, slot bookkeeping. Returns (frame_id, latents) of the frame that completed."""
        D, cx = self.depth, self.cx
        v = parts[0]
        if self.cfg:
            v = cx.cfg_combine(parts[0], parts[1], self.cfg_scale, self._comb)
        dts = [self.dts[s] if s >= 0 else 0.0 for s in self.stage]
        x = self._inp[:D, : self.S_noise]
        cx.euler_step(x, v, dts, x)
        for j in range(1, len(self.branches)):
            cx.copy(self._inp[:D, : self.S_noise], self._inp[j * D:(j + 1) * D, : self.S_noise])
        done = None
        for k in range(D):
            if self.stage[k] >= 0:
                self.stage[k] += 1
                if self.stage[k] == D:
                    res = cx.empty(1, self.S_noise, 64)
                    cx.copy(self._inp[k:k + 1, : self.S_noise], res)
                    done = (self.frame_id[k], res)
                    self.stage[k] = -1
                    self.frame_id[k] = -1
        return done

    def push(self, noise: Optional[torch.Tensor], cond_latents: Optional[torch.Tensor],
             prompt_embeds: Optional[torch.Tensor] = None,
             negative_prompt_embeds: Optional[torch.Tensor] = None) -> Optional[Tuple[int, torch.Tensor]]:
        """Insert a frame (packed noise [1,S_noise,64], packed cond [1,S_cond,64]);
        run one batched forward; return (frame_id, latents [1,S_noise,64]) for
        the frame that completed, or None while the pipeline fills.  Passing
        ``None`` drains without inserting. ``prompt_embeds`` / ``negative_prompt_embeds``: this
        frame's own text conditioning (default: the prompt given to set_conditions())."""
        v_local = self.begin(noise, cond_latents, prompt_embeds, negative_prompt_embeds)
        if v_local is None:
            return None
        return self.finish(self._exchange(v_local))

    def flush(self) -> List[Tuple[int, torch.Tensor]]:
        outs = []
        while any(s >= 0 for s in self.stage):
            r = self.push(None, None)
            if r is not None:
                outs.append(r)
        return outs


class QwenRealtimePipeline:
    """API mirror of qwen_realtime.QwenRealtimePipeline on the HIP engine.

    Frames are handed over as packed condition latents (plug ``vae.QwenImageVAEEncoder``
    in via ``image_encoder`` to accept PIL frames)."""

    def __init__(self, config: StreamConfig, image_encoder=None, prompt_encoder=None, latent_decoder=None):
        self.config = config
        self.transformer: Optional[QwenImageTransformer2DModel] = None
        self.engine: Optional[StreamBatchDenoiser] = None
        self.cache = CachedConditions()
        self.prev_latent: Optional[torch.Tensor] = None
        self.frame_count = 0
        self.is_keyframe = True
        self.inference_times: List[float] = []
        self.image_encoder = image_encoder
        self.prompt_encoder = prompt_encoder
        self.latent_decoder = latent_decoder
        self.vae = None  # vae.QwenImageVAEDecoder: finished frames come out as uint8 RGB [H, W, 3]
        self.vae_encoder = None  # vae.QwenImageVAEEncoder: uint8 RGB frames in
        self.generator: Optional[torch.Generator] = None

    def load_model(self, transformer: Optional[QwenImageTransformer2DModel] = None, seed: int = 0,
                   vae=None, **config_overrides):
        """``vae``: a QwenImageVAEDecoder, or "random" for a seeded random one (benchmarks).
        Without a transformer, ``config.model_name`` naming a local diffusers snapshot loads
        everything from it as qwen_realtime.py:116-122 does -- DiT, VAE encoder / decoder and the
        Qwen2.5-VL prompt encoder, all on the HIP path; otherwise a seeded random DiT."""
        if transformer is None and os.path.isdir(self.config.model_name):
            from .pipeline import QwenImageEditPlusPipeline
            pipe = QwenImageEditPlusPipeline.from_pretrained(self.config.model_name, torch_dtype=self.config.dtype)
            transformer = pipe.transformer
            if vae is None and pipe.vae is not None:
                vae = (pipe.vae, pipe.vae_encoder)
            if self.prompt_encoder is None:
                self.prompt_encoder = pipe.prompt_encoder
        if transformer is None:
            transformer = QwenImageTransformer2DModel(**config_overrides).random_init_(seed)
        self.transformer = transformer
        if isinstance(vae, str) and vae == "random":
            from .vae import QwenImageVAEDecoder, QwenImageVAEEncoder
            vae = (QwenImageVAEDecoder(device=transformer.device).random_init_(seed + 1),
                   QwenImageVAEEncoder(device=transformer.device).random_init_(seed + 2))
        if isinstance(vae, tuple):
            self.vae, self.vae_encoder = vae
        else:
            self.vae = vae
        self.generator = torch.Generator(device=transformer.device).manual_seed(42)

    def precompute_conditions(self, prompt: str, reference_image=None, prompt_embeds=None,
                              prompt_embeds_mask=None, negative_prompt_embeds=None,
                              negative_prompt_embeds_mask=None):
        """Encode the prompt once and build the stream engine (qwen_realtime.py:140-165).

        Deliberate approximation: the reference's per-frame pipeline call encodes each camera
        frame into the Qwen2.5-VL prompt ("Picture 1: <frame>"); here the prompt is encoded once,
        with ``reference_image`` (usually None, so no image block), and every later frame reuses
        those embeddings -- the frame still conditions the DiT through its VAE latents. Call this
        again with ``reference_image=<frame>`` (e.g. on keyframes) to refresh the image block; the
        prompt encoder's VLM / LRU caches keep that cheap."""
        if self.cache.is_valid(prompt, reference_image) and prompt_embeds is None:
            return
        if prompt_embeds is None:
            if self.prompt_encoder is None:
                raise NotImplementedError("no prompt encoder: load_model() from a local snapshot with "
                                          "text_encoder/ + processor/, pass prompt_encoder=, or prompt_embeds=")
            prompt_embeds, prompt_embeds_mask = self.prompt_encoder(prompt, reference_image)
            if self.config.true_cfg_scale > 1:
                negative_prompt_embeds, negative_prompt_embeds_mask = self.prompt_encoder(" ", reference_image)
        c = self.cache
        c.prompt, c.prompt_embeds, c.prompt_embeds_mask = prompt, prompt_embeds, prompt_embeds_mask
        c.reference_key = c.image_key(reference_image)
        c.negative_prompt_embeds, c.negative_prompt_embeds_mask = negative_prompt_embeds, negative_prompt_embeds_mask
        oh, ow = self.config.output_size
        chh, cww = self.config.cond_size
        self.engine = StreamBatchDenoiser(self.transformer, self.config.num_inference_steps,
                                          self.config.true_cfg_scale, (oh // 16, ow // 16),
                                          (chh // 16, cww // 16))
        self.engine.set_conditions(prompt_embeds, prompt_embeds_mask, negative_prompt_embeds,
                                   negative_prompt_embeds_mask)

    def prepare_latent(self, cond_latents: torch.Tensor) -> torch.Tensor:
        """qwen_realtime.py:201-224: fresh noise on keyframes, else prev + 0.05*noise."""
        e = self.engine
        self.is_keyframe = (self.frame_count % self.config.keyframe_interval == 0) or self.prev_latent is None
        noise = torch.randn((1, e.S_noise, 64), generator=self.generator, device=self.transformer.device,
                            dtype=BF16)
        if self.is_keyframe or not self.config.use_prev_latent:
            return noise
        return (self.prev_latent.float() + self.config.noise_strength * noise.float()).to(BF16)

    def frame_to_rgb(self, frame) -> torch.Tensor:
        """A camera frame as the uint8 RGB [1, H, W, 3] condition image the engine was built for.

        qwen_realtime.py:239-243 first resizes every frame to (config.width, config.height) with
        LANCZOS; Edit-Plus then resizes its VAE input to the 1024^2-area size of that aspect
        (LANCZOS again), which is ``config.cond_size`` here -- so a 640x480 webcam frame becomes
        512x512, then 1024x1024, and never changes the engine's token count. uint8 tensors must
        already have the cond size."""
        import numpy as np
        from PIL import Image
        ch, cw = self.config.cond_size
        dev = self.transformer.device
        if isinstance(frame, torch.Tensor):
            t = frame if frame.dim() == 4 else frame[None]
            if t.dtype != torch.uint8 or tuple(t.shape[1:]) != (ch, cw, 3):
                raise ValueError(f"uint8 frames must be RGB [(1,) {ch}, {cw}, 3] (config.cond_size); "
                                 f"got {tuple(frame.shape)} {frame.dtype}")
            return t.to(dev).contiguous()
        if isinstance(frame, np.ndarray):
            frame = Image.fromarray(frame)
        im = frame.convert("RGB")
        if im.size != (self.config.width, self.config.height):
            im = im.resize((self.config.width, self.config.height), Image.LANCZOS)
        if im.size != (cw, ch):
            im = im.resize((cw, ch), Image.LANCZOS)
        return torch.from_numpy(np.asarray(im).copy())[None].to(dev)

    @torch.no_grad()
    def process_frame(self, frame) -> Optional[torch.Tensor]:
        """Push one frame (packed cond latents, or anything image_encoder accepts);
        return the latents of the frame that completed (None while filling)."""
        t0 = time.time()
        if isinstance(frame, torch.Tensor) and frame.dtype != torch.uint8:
            cond = frame  # packed condition latents
        elif self.image_encoder is not None:
            cond = self.image_encoder(frame)
        elif self.vae_encoder is not None:  # qwen_realtime.py:167-186 encode_image, on the HIP path
            cond = self.vae_encoder.encode(self.frame_to_rgb(frame))
        else:
            raise NotImplementedError("frames must be packed latents, or set vae_encoder / image_encoder")
        noise = self.prepare_latent(cond)
        r = self.engine.push(noise, cond)
        self.frame_count += 1
        out = None
        if r is not None:
            out = r[1]
            self.prev_latent = out
            if self.latent_decoder is not None:
                out = self.latent_decoder(out, *self.config.output_size)
            elif self.vae is not None:  # qwen_realtime.py:188-199 decode_latent, on the HIP path
                oh, ow = self.config.output_size
                out = self.vae.decode(out, oh // 8, ow // 8)[0]
        self.inference_times.append(time.time() - t0)
        return out

    def warmup(self, frame, n: int = 3):
        for _ in range(n):
            self.process_frame(frame)
        torch.cuda.synchronize()
        self.frame_count = 0
        self.inference_times.clear()

    def get_stats(self) -> Dict:
        if not self.inference_times:
            return {}
        last = self.inference_times[-30:]
        avg = sum(last) / len(last)
        return {"avg_inference_time": avg, "fps": 1.0 / avg if avg > 0 else 0.0,
                "frame_count": self.frame_count,
                "gpu_memory_gb": torch.cuda.max_memory_allocated() / 1e9}
