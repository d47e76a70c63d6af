"""``QwenImageEditPlusPipeline``-compatible denoise pipeline on the HIP DiT.

Drop-in for the calls the reference makes (server.py:64-79, 137-153;
qwen_realtime.py:116-122, 247-255; benchmark_lightning.py:41-49):
``from_pretrained(path, torch_dtype=bf16)``, ``.to('cuda')``,
``load_lora_weights(...)``, ``enable_model_cpu_offload()`` (no-op: the model is
41 GB against 288 GB of HBM) and
``pipe(image=[...], prompt=..., negative_prompt=..., true_cfg_scale=4.0,
num_inference_steps=N, guidance_scale=..., generator=...) -> .images``.

What runs here is the hot path: latent prep + pack, the
FlowMatch schedule, and the denoise loop with **batched CFG** (the absent
``batched_cfg_pipeline.py`` of README.md:126: cond and uncond stacked on the
batch axis in ONE forward, unequal text lengths key-masked so the result equals
the reference's two sequential forwards), the true-CFG norm rescale and
the Euler step, then the VAE decode (``vae.QwenImageVAEDecoder``: unpack,
de-normalise, decoder, uint8 RGB, all on the HIP path).  The condition image is
VAE-encoded on the HIP path (``vae.QwenImageVAEEncoder``) and the prompt is encoded
by Qwen2.5-VL on the HIP path (``text_encoder.QwenImageEditPromptEncoder``
behind the snapshot's processor); callers may still pass ``prompt_embeds`` /
``image_latents`` directly or plug their own encoders into the ``prompt_encoder`` /
``image_encoder`` hooks (``latent_decoder`` overrides the HIP decoder).  ``output_type="latent"`` returns packed latents, as diffusers does.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Any, Callable, Optional, Sequence, Tuple

import torch

from . import ops
from .scheduler import FlowMatchEulerDiscreteScheduler, calculate_shift, model_timesteps
from .transformer import QwenImageTransformer2DModel
from .vae import QwenImageVAEDecoder, QwenImageVAEEncoder
from . import weights as W

BF16 = torch.bfloat16
CONDITION_IMAGE_SIZE = 384 * 384
VAE_IMAGE_SIZE = 1024 * 1024
VAE_SCALE_FACTOR = 8


def calculate_dimensions(target_area: int, ratio: float) -> Tuple[int, int]:
    """Edit-Plus ``calculate_dimensions`` [U]: (width, height), multiples of 32."""
    width = math.sqrt(target_area * ratio)
    height = width / ratio
    return int(round(width / 32) * 32), int(round(height / 32) * 32)


@dataclass
class QwenImagePipelineOutput:
    images: Any


def to_output(rgb: torch.Tensor, output_type: str):
    """uint8 RGB [B, H, W, 3] (device) -> the image processor's output types: "pil" (list of
    PIL.Image), "np" (float [B, H, W, 3] in [0, 1]), "pt" (float [B, 3, H, W] in [0, 1]), "uint8"."""
    if output_type == "uint8":
        return rgb
    if output_type == "pt":
        return rgb.permute(0, 3, 1, 2).float() / 255.0
    arr = rgb.cpu().numpy()
    if output_type == "np":
        return arr.astype("float32") / 255.0
    from PIL import Image
    return [Image.fromarray(a) for a in arr]


def images_to_rgb(image, device) -> torch.Tensor:
    """The condition image(s) as uint8 RGB [n, H, W, 3] on the device at the VAE size: PIL images
    are resized (LANCZOS) to calculate_dimensions(1024^2, aspect) as Edit-Plus does for its VAE
    input; uint8 tensors [H, W, 3] / [n, H, W, 3] are taken as they are (H, W % 16 == 0)."""
    if isinstance(image, torch.Tensor):
        t = image if image.dim() == 4 else image[None]
        if t.dtype != torch.uint8 or t.shape[-1] != 3:
            raise ValueError("image tensors must be uint8 RGB [(n,) H, W, 3]")
        return t.to(device).contiguous()
    ims = image if isinstance(image, (list, tuple)) else [image]
    if len(ims) != 1:
        raise ValueError("images_to_rgb takes one PIL image (the pipeline encodes a list image by image)")
    import numpy as np
    from PIL import Image
    im = ims[0].convert("RGB")
    w, h = calculate_dimensions(VAE_IMAGE_SIZE, im.size[0] / im.size[1])
    w, h = w // 16 * 16, h // 16 * 16
    if im.size != (w, h):
        im = im.resize((w, h), Image.LANCZOS)
    return torch.from_numpy(np.asarray(im).copy())[None].to(device)


class QwenImageEditPlusPipeline:
    def __init__(self, transformer: QwenImageTransformer2DModel,
                 scheduler: Optional[FlowMatchEulerDiscreteScheduler] = None,
                 prompt_encoder: Optional[Callable] = None, image_encoder: Optional[Callable] = None,
                 latent_decoder: Optional[Callable] = None):
        self.transformer = transformer
        self.scheduler = scheduler or FlowMatchEulerDiscreteScheduler()
        self.prompt_encoder = prompt_encoder
        self.image_encoder = image_encoder
        self.latent_decoder = latent_decoder
        self.vae = None          # QwenImageVAEDecoder (HIP): latents -> uint8 RGB
        self.vae_encoder = None  # QwenImageVAEEncoder (HIP): condition image -> packed latents
        self.text_encoder = None
        self.vae_scale_factor = VAE_SCALE_FACTOR
        self._buf = {}

    # ------------------------------------------------------------------ loading
    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path: Optional[str] = None,
                        torch_dtype: torch.dtype = BF16, device: str = "cuda",
                        random_init_seed: Optional[int] = None, int8: bool = False, **config_overrides):
        """Local diffusers snapshot, or seeded random init (no network: hub
        names resolve only if a local snapshot directory of that name exists)."""
        if torch_dtype not in (BF16, None):
            raise ValueError("the HIP path computes in bf16 (the reference's torch_dtype)")
        path = pretrained_model_name_or_path
        if path is not None and W.find_int8_files(path) and not W.find_transformer_files(path):
            # pre-quantised image (weights.save_int8): int8 weights only, LoRA must be pre-fused
            return cls(W.load_int8(path, device=device))
        model = QwenImageTransformer2DModel(device=device, **config_overrides)
        if path is not None and W.find_transformer_files(path):
            W.load_transformer_weights(model, path)
        elif random_init_seed is not None or path is None:
            model.random_init_(seed=random_init_seed or 0)
        else:
            raise FileNotFoundError(
                f"{path!r}: no local diffusers snapshot (network model downloads are unavailable); "
                "pass a local directory or random_init_seed=")
        if int8:
            model.quantize_int8()
        pipe = cls(model)
        if path is not None and W.find_vae_files(path):
            pipe.vae = W.load_vae_decoder(path, device=device)
            pipe.vae_encoder = W.load_vae_encoder(path, device=device)
        elif random_init_seed is not None or path is None:
            pipe.vae = QwenImageVAEDecoder(device=device).random_init_(seed=(random_init_seed or 0) + 1)
            pipe.vae_encoder = QwenImageVAEEncoder(device=device).random_init_(seed=(random_init_seed or 0) + 2)
        if path is not None and os.path.isdir(os.path.join(path, "text_encoder")):
            pipe.prompt_encoder = cls._snapshot_prompt_encoder(path, device)
        return pipe

    @staticmethod
    def _snapshot_prompt_encoder(path: str, device):
        """The snapshot's Qwen2.5-VL on the HIP path behind the snapshot's own processor
        (``processor/``: tokenizer + Qwen2VLImageProcessor, loaded from local files only)."""
        from transformers import AutoProcessor
        from .text_encoder import QwenImageEditPromptEncoder
        proc_dir = os.path.join(path, "processor")
        processor = AutoProcessor.from_pretrained(proc_dir if os.path.isdir(proc_dir) else path,
                                                  local_files_only=True)
        return QwenImageEditPromptEncoder(W.load_prompt_encoder(path, device=device), processor)

    def to(self, device=None, *a, **k):
        return self

    def enable_model_cpu_offload(self, *a, **k):
        """No-op: the whole model stays resident in HBM (qwen_realtime.py:122 calls it)."""

    def load_lora_weights(self, pretrained_model_name_or_path_or_dict, weight_name: Optional[str] = None,
                          adapter_name: Optional[str] = None, lora_scale: float = 1.0, **kw) -> int:
        """Fuse a LoRA file / state dict into the transformer (W += s*B@A); returns the adapter
        count. Raises ``weights.LoraKeyError`` when no adapter fuses or a key maps onto no linear
        (peft, diffusion_model.* lora_down/up and kohya lora_unet_* forms are all accepted)."""
        sd = pretrained_model_name_or_path_or_dict
        if not isinstance(sd, dict):
            sd = W.load_lora_file(sd, weight_name)
        return W.fuse_lora(self.transformer, sd, scale=lora_scale)

    # ------------------------------------------------------------------ helpers
    def _embeds(self, prompt, image, embeds, mask):
        if embeds is None:
            if self.prompt_encoder is None:
                raise NotImplementedError(
                    "no prompt encoder: load a snapshot with text_encoder/ + processor/, set pipe.prompt_encoder "
                    "(text_encoder.QwenImageEditPromptEncoder), or pass prompt_embeds=")
            embeds, mask = self.prompt_encoder(prompt, image)
        if mask is None:
            mask = torch.ones(embeds.shape[:2], dtype=torch.long, device=embeds.device)
        return embeds.to(BF16), mask

    def _image_latents(self, image, image_latents, B):
        """Packed condition latents, and their (h, w) token grid when the HIP encoder made them."""
        shape = None
        if image_latents is None:
            if self.image_encoder is not None:
                image_latents = self.image_encoder(image)
            elif self.vae_encoder is not None:
                # Edit-Plus takes up to several condition images ("Picture 1", "Picture 2", ...): each
                # is resized to the VAE area of its own aspect ratio and encoded on its own; their
                # packed latents follow each other in the sequence, one img_shapes entry apiece
                ims = image if isinstance(image, (list, tuple)) else [image]
                if isinstance(image, torch.Tensor):
                    ims = [image]
                lat, shape = [], []
                for im in ims:
                    rgb = images_to_rgb(im, self.transformer.device)
                    lat.append(self.vae_encoder.encode(rgb))
                    shape.append((rgb.shape[1] // 16, rgb.shape[2] // 16))
                image_latents = lat[0] if len(lat) == 1 else torch.cat(lat, 1)
                shape = shape[0] if len(shape) == 1 else shape
            else:
                raise NotImplementedError(
                    "no VAE encoder: pass image_latents= (packed [B, S, 64]), set pipe.vae_encoder or "
                    "pipe.image_encoder")
        if image_latents.dim() != 3:
            raise ValueError("image_latents must be packed [B, S, 64]")
        if image_latents.shape[0] == 1 and B > 1:
            image_latents = image_latents.expand(B, -1, -1)
        return image_latents.to(BF16), shape

    @staticmethod
    def prepare_noise(batch: int, height: int, width: int, generator: Optional[torch.Generator],
                      device) -> torch.Tensor:
        """randn((B,1,16,H/8,W/8), bf16) from the caller's generator, packed to
        [B, (H/16)(W/16), 64] by the HIP pack kernel (diffusers prepare_latents)."""
        h, w = 2 * (height // (VAE_SCALE_FACTOR * 2)), 2 * (width // (VAE_SCALE_FACTOR * 2))
        gdev = generator.device if generator is not None else torch.device(device)
        x = torch.randn((batch, 1, 16, h, w), generator=generator, device=gdev, dtype=BF16)
        return ops.pack_latents(x.to(device))

    # ------------------------------------------------------------------ call
    @torch.no_grad()
    def __call__(self, image=None, prompt=None, negative_prompt=None, true_cfg_scale: float = 4.0,
                 height: Optional[int] = None, width: Optional[int] = None,
                 num_inference_steps: int = 40, sigmas: Optional[Sequence[float]] = None,
                 guidance_scale: Optional[float] = None, num_images_per_prompt: int = 1,
                 generator: Optional[torch.Generator] = None, latents: Optional[torch.Tensor] = None,
                 prompt_embeds=None, prompt_embeds_mask=None, negative_prompt_embeds=None,
                 negative_prompt_embeds_mask=None, image_latents=None,
                 cond_shape=None, output_type: str = "pil",
                 return_dict: bool = True, batched_cfg: bool = True, **unused):
        # guidance_scale is a no-op for this non-guidance-distilled model [U]
        dev = self.transformer.device
        if height is None or width is None:
            im = image[-1] if isinstance(image, list) else image
            if isinstance(im, torch.Tensor):  # uint8 RGB [(n,) H, W, 3]
                width, height = calculate_dimensions(VAE_IMAGE_SIZE, im.shape[-2] / im.shape[-3])
            elif im is not None and hasattr(im, "size"):
                width, height = calculate_dimensions(VAE_IMAGE_SIZE, im.size[0] / im.size[1])
            else:
                width, height = 1024, 1024
        pe, pm = self._embeds(prompt, image, prompt_embeds, prompt_embeds_mask)
        B = pe.shape[0] * num_images_per_prompt
        if num_images_per_prompt > 1:
            pe, pm = pe.repeat_interleave(num_images_per_prompt, 0), pm.repeat_interleave(num_images_per_prompt, 0)
        has_neg = negative_prompt is not None or negative_prompt_embeds is not None
        do_cfg = true_cfg_scale > 1 and has_neg
        if do_cfg:
            ne, nm = self._embeds(negative_prompt, image, negative_prompt_embeds, negative_prompt_embeds_mask)
            if ne.shape[0] != B:
                ne, nm = ne.expand(B, -1, -1), nm.expand(B, -1)
        cond, enc_shape = self._image_latents(image, image_latents, B)
        if cond_shape is None and enc_shape is not None:
            cond_shape = enc_shape
        if latents is None:
            latents = self.prepare_noise(B, height, width, generator, dev)
        S_noise = latents.shape[1]
        lh, lw = height // VAE_SCALE_FACTOR // 2, width // VAE_SCALE_FACTOR // 2
        if lh * lw != S_noise:
            raise ValueError(f"latents carry {S_noise} tokens, expected {lh}x{lw}")
        if cond_shape is None:
            side = int(round(math.sqrt(cond.shape[1])))
            cond_shape = (side, cond.shape[1] // side)
        cond_shapes = [tuple(cond_shape)] if isinstance(cond_shape[0], int) else [tuple(c) for c in cond_shape]
        if sum(h * w for h, w in cond_shapes) != cond.shape[1]:
            raise ValueError(f"cond_shape {cond_shapes} does not cover the {cond.shape[1]} condition tokens")
        img_shapes = [[(1, lh, lw)] + [(1, h, w) for h, w in cond_shapes]] * B

        sch = self.scheduler
        c = sch.config
        mu = calculate_shift(S_noise, c.base_image_seq_len, c.max_image_seq_len, c.base_shift, c.max_shift)
        sch.set_timesteps(num_inference_steps, sigmas=sigmas, mu=mu)
        ts = sch.timesteps.tolist()

        rows = 2 * B if (do_cfg and batched_cfg) else B
        S_img = S_noise + cond.shape[1]
        inp = torch.empty(rows, S_img, 64, dtype=BF16, device=dev)
        ops.copy_batched(latents.to(BF16).contiguous(), inp[:B, :S_noise])
        ops.copy_batched(cond.contiguous(), inp[:B, S_noise:])
        lens_c = [int(x) for x in pm.sum(1).tolist()]
        if do_cfg:
            lens_n = [int(x) for x in nm.sum(1).tolist()]
        if do_cfg and batched_cfg:
            ops.copy_batched(inp[:B], inp[B:])
            S_txt = max(pe.shape[1], ne.shape[1])
            enc = torch.zeros(rows, S_txt, pe.shape[2], dtype=BF16, device=dev)
            enc[:B, : pe.shape[1]] = pe
            enc[B:, : ne.shape[1]] = ne
            txt_lens = lens_c + lens_n
        else:
            enc, txt_lens = pe.contiguous(), lens_c
        comb = torch.empty(B, S_noise, 64, dtype=BF16, device=dev) if do_cfg else None
        tf = self.transformer
        for i, t in enumerate(ts):
            tb = model_timesteps([t] * rows, dev)
            out = tf(inp, enc, None, tb, img_shapes * (rows // B), txt_lens, return_dict=False)[0]
            v = out[:B, :S_noise]
            if do_cfg:
                if batched_cfg:
                    vn = out[B:, :S_noise]
                else:
                    outn = tf(inp, ne.contiguous(), None, tb, img_shapes, lens_n, return_dict=False)[0]
                    vn = outn[:, :S_noise]
                v = ops.cfg_combine(v, vn, true_cfg_scale, out=comb)
            dt = sch.dt(i)
            ops.euler_step(inp[:B, :S_noise], v, [dt] * B, inp[:B, :S_noise])
            if do_cfg and batched_cfg:
                ops.copy_batched(inp[:B, :S_noise], inp[B:, :S_noise])
        final = torch.empty(B, S_noise, 64, dtype=BF16, device=dev)
        ops.copy_batched(inp[:B, :S_noise], final)
        if output_type == "latent":
            images = final
        elif self.latent_decoder is not None:
            images = self.latent_decoder(final, 2 * lh, 2 * lw)
        elif self.vae is not None:  # HIP VAE decoder (vae.py): uint8 RGB [B, H, W, 3] on the device
            images = to_output(self.vae.decode(final, 2 * lh, 2 * lw), output_type)
        else:
            raise NotImplementedError("no VAE decoder: load a snapshot with vae/, set pipe.vae / "
                                      "pipe.latent_decoder, or use output_type='latent'")
        if not return_dict:
            return (images,)
        return QwenImagePipelineOutput(images=images)
