"""Stream-batch denoising: the replacement for qwen_realtime.py's denoise loop.

Reference: ``StreamConfig`` (qwen_realtime.py:39-66), ``CachedConditions``
(69-89; prompt-keyed ``is_valid`` 82-89), the never-called ``prepare_latent``
(201-224: prev-latent + 0.05*noise, keyframe every 20) and ``process_frame``
(226-268), which re-runs the whole diffusers pipeline per frame.  SURVEY.md
§0.4 / §8 a18: "stream batch depth=2" is defined by the build, following
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
        if isinstance(image, torch.Tensor):
            h.update(str(tuple(image.shape)).encode())
            h.update(image.detach().cpu().contiguous().numpy().tobytes())
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


class StreamBatchDenoiser:
    """N frames in flight, one batched DiT forward per pushed frame."""

    def __init__(self, transformer: QwenImageTransformer2DModel, num_steps: int = 2,
                 true_cfg_scale: float = 1.0, latent_hw: Tuple[int, int] = (64, 64),
                 cond_hw: Tuple[int, int] = (64, 64),
                 scheduler: Optional[FlowMatchEulerDiscreteScheduler] = None):
        self.tf = transformer
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
        self.stage: List[int] = [-1] * self.depth  # -1 = empty slot
        self.frame_id: List[int] = [-1] * self.depth
        self._next_frame = 0
        self._inp: Optional[torch.Tensor] = None
        self._enc = None
        self._txt_lens = None
        self._comb = None
        dev = transformer.device
        self._tcache: Dict[Tuple[int, ...], torch.Tensor] = {}
        self.img_shapes = [[(1, self.lh, self.lw), (1, self.ch, self.cw)]]

    @property
    def rows(self) -> int:
        return self.depth * (2 if self.cfg else 1)

    def set_conditions(self, prompt_embeds: torch.Tensor, prompt_embeds_mask: Optional[torch.Tensor] = None,
                       negative_prompt_embeds: Optional[torch.Tensor] = None,
                       negative_prompt_embeds_mask: Optional[torch.Tensor] = None):
        """Cache the (padded, batched) text conditioning once per prompt."""
        dev = self.tf.device
        pe = prompt_embeds.to(dev, BF16)
        if pe.dim() == 2:
            pe = pe[None]
        lc = int(prompt_embeds_mask.sum()) if prompt_embeds_mask is not None else pe.shape[1]
        self.cfg = negative_prompt_embeds is not None and self.cfg_scale > 1.0
        if self.cfg:
            ne = negative_prompt_embeds.to(dev, BF16)
            if ne.dim() == 2:
                ne = ne[None]
            ln = int(negative_prompt_embeds_mask.sum()) if negative_prompt_embeds_mask is not None else ne.shape[1]
            S_txt = max(pe.shape[1], ne.shape[1])
        else:
            S_txt = pe.shape[1]
        enc = torch.zeros(self.rows, S_txt, pe.shape[2], dtype=BF16, device=dev)
        enc[: self.depth, : pe.shape[1]] = pe[0]
        lens = [lc] * self.depth
        if self.cfg:
            enc[self.depth:, : ne.shape[1]] = ne[0]
            lens += [ln] * self.depth
        self._enc, self._txt_lens = enc, lens
        self._inp = torch.zeros(self.rows, self.S_img, 64, dtype=BF16, device=dev)
        self._comb = torch.empty(self.depth, self.S_noise, 64, dtype=BF16, device=dev) if self.cfg else None
        self.stage = [-1] * self.depth
        self.frame_id = [-1] * self.depth

    def _t_rows(self) -> torch.Tensor:
        st = tuple(max(s, 0) for s in self.stage)
        t = self._tcache.get(st)
        if t is None:
            per_slot = [self.timesteps[s] for s in st]
            t = model_timesteps(per_slot * (2 if self.cfg else 1), self.tf.device)
            self._tcache[st] = t
        return t

    def push(self, noise: Optional[torch.Tensor], cond_latents: Optional[torch.Tensor]
             ) -> Optional[Tuple[int, torch.Tensor]]:
        """Insert a frame (packed noise [1,S_noise,64], packed cond [1,S_cond,64]);
        run one batched forward; return (frame_id, latents [1,S_noise,64]) for
        the frame that completed, or None while the pipeline fills.  Passing
        ``None`` drains without inserting."""
        if self._inp is None:
            raise RuntimeError("call set_conditions() first")
        D = self.depth
        if noise is not None:
            slot = self.stage.index(-1) if -1 in self.stage else None
            if slot is None:
                raise RuntimeError("no free slot (internal invariant broken)")
            inp = self._inp
            ops.copy_batched(noise.reshape(1, self.S_noise, 64).to(BF16), inp[slot:slot + 1, : self.S_noise])
            ops.copy_batched(cond_latents.reshape(1, self.S_cond, 64).to(BF16),
                             inp[slot:slot + 1, self.S_noise:])
            if self.cfg:
                ops.copy_batched(inp[slot:slot + 1], inp[D + slot:D + slot + 1])
            self.stage[slot] = 0
            self.frame_id[slot] = self._next_frame
            self._next_frame += 1
        if all(s < 0 for s in self.stage):
            return None
        out = self.tf(self._inp, self._enc, None, self._t_rows(), self.img_shapes * self.rows,
                      self._txt_lens, return_dict=False)[0]
        v = out[:D, : self.S_noise]
        if self.cfg:
            v = ops.cfg_combine(v, out[D:, : self.S_noise], self.cfg_scale, out=self._comb)
        dts = [self.dts[s] if s >= 0 else 0.0 for s in self.stage]
        x = self._inp[:D, : self.S_noise]
        ops.euler_step(x, v, dts, x)
        if self.cfg:
            ops.copy_batched(self._inp[:D, : self.S_noise], self._inp[D:, : self.S_noise])
        done = None
        for k in range(D):
            if self.stage[k] >= 0:
                self.stage[k] += 1
                if self.stage[k] == D:
                    res = torch.empty(1, self.S_noise, 64, dtype=BF16, device=self.tf.device)
                    ops.copy_batched(self._inp[k:k + 1, : self.S_noise], res)
                    done = (self.frame_id[k], res)
                    self.stage[k] = -1
                    self.frame_id[k] = -1
        return done

    def flush(self) -> List[Tuple[int, torch.Tensor]]:
        outs = []
        while any(s >= 0 for s in self.stage):
            r = self.push(None, None)
            if r is not None:
                outs.append(r)
        return outs


class QwenRealtimePipeline:
    """API mirror of qwen_realtime.QwenRealtimePipeline on the HIP engine.

    Frames are handed over as packed condition latents (the VAE encoder is the
    §8 f1 next row; plug one in via ``image_encoder`` to accept PIL frames)."""

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
