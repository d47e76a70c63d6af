"""Weight loading: local diffusers-format safetensors + Lightning-LoRA fuse.

The reference loads by hub name (server.py:64-69 ``from_pretrained(
"Qwen/Qwen-Image-Edit-2509")``, server.py:76-79 ``load_lora_weights(
"lightx2v/Qwen-Image-Lightning", weight_name="Qwen-Image-Edit-Lightning-4steps-
V1.0.safetensors")``).  There is no network here, so this module reads LOCAL
paths only with the safe loader (``safetensors``; never
pickle), and fuses LoRA deltas into the packed bf16 weights at load time
(W += scale * B @ A), so the Lightning adapters cost nothing per step.
"""
from __future__ import annotations

import glob
import os
import re
from typing import Dict, Iterable, Optional

import torch

BF16 = torch.bfloat16


def find_transformer_files(path: str):
    """Locate transformer safetensors shards under a diffusers repo snapshot."""
    if os.path.isfile(path) and path.endswith(".safetensors"):
        return [path]
    for sub in ("transformer", "."):
        files = sorted(glob.glob(os.path.join(path, sub, "*.safetensors")))
        if files:
            return files
    return []


def iter_safetensors(files: Iterable[str]):
    from safetensors import safe_open
    for f in files:
        with safe_open(f, framework="pt", device="cpu") as fh:
            for k in fh.keys():
                yield k, fh.get_tensor(k)


def load_transformer_weights(model, path: str, strict: bool = True) -> int:
    files = find_transformer_files(path)
    if not files:
        raise FileNotFoundError(f"no transformer *.safetensors under {path}")
    n = 0
    names = set(model.diffusers_names())
    seen = set()
    with torch.no_grad():
        for k, v in iter_safetensors(files):
            if k not in names:
                if strict:
                    raise KeyError(f"unexpected parameter {k}")
                continue
            model._param_slot(k).copy_(v.to(model.device, BF16))
            seen.add(k)
            n += 1
    if strict and seen != names:
        raise KeyError(f"missing {len(names - seen)} parameters, e.g. {sorted(names - seen)[:3]}")
    model._requantize_if_needed()
    return n


# Key forms a Qwen-Image LoRA file comes in (diffusers accepts all of them through
# `_convert_non_diffusers_qwen_lora_to_diffusers` [U] before peft loads the adapters):
#   peft / diffusers   [transformer.]<stem>.lora_A[.default].weight, .lora_B[...]
#   ComfyUI / lightx2v [diffusion_model.]<stem>.lora_down.weight, .lora_up.weight, .alpha
#   kohya              lora_unet_<stem with "." -> "_">.lora_down.weight, ...
# The stem prefixes are stripped in every form; kohya stems are resolved against the
# model's own module names (each "." of a diffusers stem read as "_").
_LORA_PREFIXES = ("base_model.model.", "model.diffusion_model.", "diffusion_model.", "transformer.")
_LORA_SUFFIXES = [
    (re.compile(r"^(.+)\.lora_A(?:\.default)?\.weight$"), "A"),
    (re.compile(r"^(.+)\.lora_B(?:\.default)?\.weight$"), "B"),
    (re.compile(r"^(.+)\.lora_down\.weight$"), "A"),
    (re.compile(r"^(.+)\.lora_up\.weight$"), "B"),
    (re.compile(r"^(.+)\.lora\.down\.weight$"), "A"),
    (re.compile(r"^(.+)\.lora\.up\.weight$"), "B"),
    (re.compile(r"^(.+)\.alpha$"), "alpha"),
]


class LoraKeyError(KeyError):
    """A LoRA state dict that does not map onto the transformer's linears."""


def _lora_stem(key: str):
    """(stem, kind) of one LoRA tensor name, prefixes stripped; None when it is no LoRA key."""
    k = key
    stripped = True
    while stripped:
        stripped = False
        for p in _LORA_PREFIXES:
            if k.startswith(p):
                k, stripped = k[len(p):], True
    for pat, kind in _LORA_SUFFIXES:
        m = pat.match(k)
        if m:
            return m.group(1), kind
    return None


def parse_lora(sd: Dict[str, torch.Tensor], known_stems: Optional[Iterable[str]] = None):
    """Group a LoRA state dict into {module_stem: {"A": [r,in], "B": [out,r], "alpha": ()}}.

    Returns (groups, unparsed_keys). ``known_stems`` (the model's diffusers module names)
    resolves kohya ``lora_unet_*`` stems, whose dots are underscores."""
    flat = {s.replace(".", "_"): s for s in (known_stems or ())}
    groups: Dict[str, Dict[str, torch.Tensor]] = {}
    unparsed = []
    for k, v in sd.items():
        r = _lora_stem(k)
        if r is None:
            unparsed.append(k)
            continue
        stem, kind = r
        if stem.startswith("lora_unet_"):
            stem = flat.get(stem[len("lora_unet_"):], stem)
        groups.setdefault(stem, {})[kind] = v
    return groups, unparsed


def _linear_stems(model):
    return sorted({n[:-len(".weight")] for n in model.diffusers_names() if n.endswith(".weight")})


@torch.no_grad()
def fuse_lora(model, lora_sd: Dict[str, torch.Tensor], scale: float = 1.0, strict: bool = True) -> int:
    """W[stem] += scale * (alpha / r) * B @ A for every adapter in the dict; returns the count.

    Raises ``LoraKeyError`` when nothing fuses, and -- with ``strict`` (the default, as the
    reference's diffusers loader refuses a state dict with keys left over after conversion) --
    when a key is no LoRA key, an adapter lacks its A or B half, or a stem names no linear of
    the model. ``strict=False`` skips those instead. A shape mismatch always raises."""
    groups, unparsed = parse_lora(lora_sd, _linear_stems(model))
    problems = [f"not a LoRA key: {k}" for k in unparsed]
    todo = []
    for stem, g in groups.items():
        if "A" not in g or "B" not in g:
            problems.append(f"{stem}: lora {'B' if 'A' in g else 'A'} half missing")
            continue
        try:
            w = model._param_slot(stem + ".weight")
        except (KeyError, IndexError, AttributeError, ValueError):
            problems.append(f"{stem}: no such linear in the transformer")
            continue
        A, B = g["A"], g["B"]
        if A.dim() != 2 or B.dim() != 2 or A.shape[0] != B.shape[1] or (B.shape[0], A.shape[1]) != tuple(w.shape):
            raise LoraKeyError(f"{stem}: lora A {tuple(A.shape)} / B {tuple(B.shape)} do not fit weight "
                               f"{tuple(w.shape)}")
        todo.append((stem, w, g))
    if problems and strict:
        raise LoraKeyError(f"{len(problems)} LoRA entries do not map onto the transformer, e.g. "
                           f"{problems[:3]}")
    if not todo:
        raise LoraKeyError(f"no LoRA adapter fused ({len(lora_sd)} keys; {problems[:3]})")
    for stem, w, g in todo:
        A = g["A"].to(model.device, torch.float32)
        B = g["B"].to(model.device, torch.float32)
        r = A.shape[0]
        s = scale * (float(g["alpha"]) / r if "alpha" in g else 1.0)
        w.copy_((w.float() + s * (B @ A)).to(BF16))
    model._requantize_if_needed()
    return len(todo)


def load_lora_file(path: str, weight_name: Optional[str] = None) -> Dict[str, torch.Tensor]:
    f = os.path.join(path, weight_name) if weight_name and os.path.isdir(path) else path
    if not os.path.isfile(f):
        raise FileNotFoundError(
            f"LoRA file {f} not found (hub names such as 'lightx2v/Qwen-Image-Lightning' need a "
            "local snapshot: there is no network access)")
    return dict(iter_safetensors([f]))


# ---------------------------------------------------------------------------------------------
# Pre-quantised int8 image (the reference quantises at start-up with
# bitsandbytes, benchmark_int8.py:72-84, and has no on-disk int8 format). The image holds the
# W8A8 weights this build computes with: int8 [N, K] + fp32 per-row scales for the eight block
# linears (packed: q|k|v in one matrix), bf16 for everything else. Loading it allocates no bf16
# copy of those linears, so the DiT needs ~21 GB of HBM instead of 41 + 20.
INT8_FORMAT = "qie-int8-v1"


def save_int8(model, directory: str, blocks_per_shard: int = 10) -> list:
    """Write ``model.int8_state_dict()`` as safetensors shards under ``directory``; the config and
    format tag ride in each shard's metadata. Returns the written file names."""
    import json
    from safetensors.torch import save_file
    sd = model.int8_state_dict()
    L = model.config.num_layers
    n_shards = max(1, (L + blocks_per_shard - 1) // blocks_per_shard)
    import dataclasses
    cfg = json.dumps(dataclasses.asdict(model.config))
    os.makedirs(directory, exist_ok=True)

    def shard_of(name: str) -> int:
        if name.startswith("transformer_blocks."):
            return int(name.split(".")[1]) // blocks_per_shard
        return 0

    files = []
    for k in range(n_shards):
        part = {n: t.detach().contiguous().cpu() for n, t in sd.items() if shard_of(n) == k}
        fn = os.path.join(directory, f"qie_int8-{k + 1:05d}-of-{n_shards:05d}.safetensors")
        save_file(part, fn, metadata={"format": INT8_FORMAT, "config": cfg, "shard": str(k)})
        files.append(fn)
    return files


def find_int8_files(path: str):
    if os.path.isfile(path) and path.endswith(".safetensors"):
        return [path]
    for sub in ("transformer_int8", "."):
        files = sorted(glob.glob(os.path.join(path, sub, "qie_int8-*.safetensors")))
        if files:
            return files
    return []


def load_int8(path: str, device="cuda"):
    """Build a ``QwenImageTransformer2DModel`` from a pre-quantised image (no bf16 copy of the
    quantised linears is allocated). Safe loader only (safetensors)."""
    import json
    from safetensors import safe_open
    from .transformer import QwenImageTransformer2DModel
    files = find_int8_files(path)
    if not files:
        raise FileNotFoundError(f"no qie_int8-*.safetensors under {path}")
    with safe_open(files[0], framework="pt", device="cpu") as fh:
        meta = fh.metadata() or {}
    if meta.get("format") != INT8_FORMAT:
        raise ValueError(f"{files[0]}: format {meta.get('format')!r}, expected {INT8_FORMAT!r}")
    cfg = json.loads(meta["config"])
    model = QwenImageTransformer2DModel(device=device, int8_only=True, **cfg)
    sd = {}
    for f in files:
        with safe_open(f, framework="pt", device="cpu") as fh:
            for k in fh.keys():
                sd[k] = fh.get_tensor(k).to(device)
    return model.load_int8_state_dict(sd)


# ---------------------------------------------------------------------------- VAE
def find_vae_files(path: str):
    """VAE safetensors of a diffusers snapshot (``vae/*.safetensors``)."""
    return sorted(glob.glob(os.path.join(path, "vae", "*.safetensors"))) if os.path.isdir(path) else []


def _vae_config(path: str):
    import json
    from .vae import VAEConfig
    cfg = VAEConfig()
    cj = os.path.join(path, "vae", "config.json")
    if os.path.isfile(cj):
        with open(cj) as fh:
            c = json.load(fh)
        for k in ("base_dim", "z_dim", "num_res_blocks"):
            if k in c:
                setattr(cfg, k, int(c[k]))
        for k in ("dim_mult", "temperal_downsample", "latents_mean", "latents_std"):
            if k in c:
                setattr(cfg, k, tuple(c[k]))
    return cfg


def _vae_tensors(path: str, prefixes):
    files = find_vae_files(path)
    if not files:
        raise FileNotFoundError(f"no vae/*.safetensors under {path}")
    from safetensors import safe_open
    sd = {}
    for f in files:
        with safe_open(f, framework="pt", device="cpu") as fh:
            for k in fh.keys():
                if k.startswith(prefixes):
                    sd[k] = fh.get_tensor(k)
    return sd


def load_vae_decoder(path: str, device="cuda"):
    """QwenImageVAEDecoder from a diffusers snapshot: ``vae/config.json`` (dims, latents_mean /
    latents_std) and the decode half of the AutoencoderKLQwenImage state_dict (``decoder.*``,
    ``post_quant_conv.*``; the other keys are skipped without being read)."""
    from .vae import QwenImageVAEDecoder
    return QwenImageVAEDecoder(_vae_config(path), device).load_state_dict(
        _vae_tensors(path, ("decoder.", "post_quant_conv.")))


def load_vae_encoder(path: str, device="cuda"):
    """QwenImageVAEEncoder from the same snapshot (``encoder.*``, ``quant_conv.*``)."""
    from .vae import QwenImageVAEEncoder
    return QwenImageVAEEncoder(_vae_config(path), device).load_state_dict(
        _vae_tensors(path, ("encoder.", "quant_conv.")))


# ---------------------------------------------------------------------------- prompt encoder
def _prompt_encoder_configs(path: str):
    """(TextEncoderConfig, VisionConfig, image_token_id) from ``text_encoder/config.json`` -- the
    Qwen2_5_VLConfig of the snapshot; text fields at the top level (transformers 4.x checkpoints)
    or under ``text_config``."""
    import json
    from .text_encoder import QwenVLEncoder, TextEncoderConfig
    from .vision import VisionConfig
    tc, vc, img = TextEncoderConfig(), VisionConfig(), QwenVLEncoder.IMAGE_TOKEN_ID
    cj = os.path.join(path, "text_encoder", "config.json")
    if os.path.isfile(cj):
        with open(cj) as fh:
            c = json.load(fh)
        t = dict(c)
        t.update(c.get("text_config") or {})
        for k in ("vocab_size", "hidden_size", "intermediate_size", "num_hidden_layers", "num_attention_heads",
                  "num_key_value_heads"):
            if k in t:
                setattr(tc, k, int(t[k]))
        if "rms_norm_eps" in t:
            tc.rms_norm_eps = float(t["rms_norm_eps"])
        rope = t.get("rope_parameters") or t.get("rope_scaling") or {}
        if "rope_theta" in t or "rope_theta" in rope:
            tc.rope_theta = float(rope.get("rope_theta", t.get("rope_theta")))
        if "mrope_section" in rope:
            tc.mrope_section = tuple(int(v) for v in rope["mrope_section"])
        v = c.get("vision_config") or {}
        for k in ("depth", "hidden_size", "intermediate_size", "num_heads", "in_channels", "patch_size",
                  "temporal_patch_size", "spatial_merge_size", "window_size", "out_hidden_size"):
            if k in v:
                setattr(vc, k, int(v[k]))
        if "fullatt_block_indexes" in v:
            vc.fullatt_block_indexes = tuple(int(i) for i in v["fullatt_block_indexes"])
        img = int(c.get("image_token_id", img))
    return tc, vc, img


def load_prompt_encoder(path: str, device="cuda"):
    """QwenVLEncoder (Qwen2.5-VL vision tower + language model) from a diffusers snapshot's
    ``text_encoder/`` (config.json + safetensors shards; ``lm_head`` is skipped unread)."""
    from safetensors import safe_open
    from .text_encoder import QwenVLEncoder
    files = sorted(glob.glob(os.path.join(path, "text_encoder", "*.safetensors"))) if os.path.isdir(path) else []
    if not files:
        raise FileNotFoundError(f"no text_encoder/*.safetensors under {path}")
    tc, vc, img = _prompt_encoder_configs(path)
    sd = {}
    for f in files:
        with safe_open(f, framework="pt", device="cpu") as fh:
            for k in fh.keys():
                if not k.startswith("lm_head"):
                    sd[k] = fh.get_tensor(k)
    return QwenVLEncoder(tc, vc, device, image_token_id=img).load_state_dict(sd)
