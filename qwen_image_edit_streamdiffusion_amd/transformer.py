"""HIP-backed drop-in for diffusers ``QwenImageTransformer2DModel`` [U].

The reference swaps this module in as ``pipeline.transformer = <module>``
(benchmark_compile.py:102-106, benchmark_lightning_compile.py:89-93,
test_compiled.py:39-43) and the Edit-Plus pipeline calls it once per denoise
step per CFG branch.  Same constructor config, same
``forward`` signature and return convention, same diffusers state_dict names
(``load_state_dict`` / LoRA fuse address them), plus ``.config``, ``.dtype``,
``.device`` and a no-op ``cache_context``.

Every arithmetic op of the forward runs in libqie.so (include/qie.h); torch
only owns the HBM buffers and the stream.  Weights are kept packed for the
kernels: q|k|v fused into one [3D, D] matrix per stream.

HBM layout per forward (B rows, S_img image tokens, S_txt text tokens):
  x_img [B*S_img, D], x_txt [B*S_txt, D]      residual streams (bf16)
  h_*                                          LN+modulate outputs
  qkv   [3][B][H][S_pad][128]                  joint [image; text; pad] sequence
  att_* [B*S_*, D], mlp_* [B*S_*, 4D]          attention / GELU outputs
"""
from __future__ import annotations

import contextlib
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import torch
from torch import nn

from . import ops
from .rope import rope_tables

BF16 = torch.bfloat16


@dataclass
class TransformerConfig:
    """``QwenImageTransformer2DModel.config``."""

    patch_size: int = 2
    in_channels: int = 64
    out_channels: int = 16
    num_layers: int = 60
    attention_head_dim: int = 128
    num_attention_heads: int = 24
    joint_attention_dim: int = 3584
    guidance_embeds: bool = False
    axes_dims_rope: Tuple[int, int, int] = (16, 56, 56)

    @property
    def inner_dim(self) -> int:
        return self.num_attention_heads * self.attention_head_dim

    def __getitem__(self, k):  # diffusers FrozenDict-style access
        return getattr(self, k)

    def get(self, k, default=None):
        return getattr(self, k, default)


@dataclass
class Transformer2DModelOutput:
    sample: torch.Tensor


class _Block(nn.Module):
    """Packed weights of one QwenImageTransformerBlock."""

    def __init__(self, D: int, Dh: int, F: int, device, dtype=BF16, int8_only: bool = False,
                 mod_w: Optional[torch.Tensor] = None, mod_b: Optional[torch.Tensor] = None,
                 mod_off: int = 0):
        """``mod_w`` / ``mod_b``: the model's packed modulation weights [L * 2 * 6D, D] / [L * 2 * 6D];
        this block's img_mod / txt_mod rows start at ``mod_off`` / ``mod_off + 6D``."""
        super().__init__()
        e = dict(device=device, dtype=dtype)

        def lin(*shape):  # bf16 weight of a quantised linear: absent when loaded pre-quantised
            return torch.empty(0, **e) if int8_only else torch.empty(*shape, **e)

        self.mod_off = mod_off
        for j, s in enumerate(("img", "txt")):
            o = mod_off + j * 6 * D
            self.register_buffer(f"w_mod_{s}", mod_w[o:o + 6 * D] if mod_w is not None
                                 else torch.empty(6 * D, D, **e))
            self.register_buffer(f"b_mod_{s}", mod_b[o:o + 6 * D] if mod_b is not None
                                 else torch.empty(6 * D, **e))
            self.register_buffer(f"w_qkv_{s}", lin(3 * D, D))
            self.register_buffer(f"b_qkv_{s}", torch.empty(3 * D, **e))
            self.register_buffer(f"w_out_{s}", lin(D, D))
            self.register_buffer(f"b_out_{s}", torch.empty(D, **e))
            self.register_buffer(f"w_up_{s}", lin(F, D))
            self.register_buffer(f"b_up_{s}", torch.empty(F, **e))
            self.register_buffer(f"w_down_{s}", lin(D, F))
            self.register_buffer(f"b_down_{s}", torch.empty(D, **e))
        for n in ("norm_q", "norm_k", "norm_added_q", "norm_added_k"):
            self.register_buffer(n, torch.empty(Dh, **e))
        self.q8: Dict[str, Tuple[torch.Tensor, torch.Tensor]] = {}


class _Workspace:
    def __init__(self, cfg: TransformerConfig, B: int, S_img: int, S_txt: int, device, int8: bool):
        D, H, Dh = cfg.inner_dim, cfg.num_attention_heads, cfg.attention_head_dim
        F = 4 * D
        self.S_pad = ((S_img + S_txt + 255) // 256) * 256
        e = dict(device=device, dtype=BF16)
        R_i, R_t = B * S_img, B * S_txt
        self.x_img = torch.empty(R_i, D, **e)
        self.x_txt = torch.empty(max(R_t, 1), D, **e)
        self.h_img = torch.empty(R_i, D, **e)
        self.h_txt = torch.empty(max(R_t, 1), D, **e)
        self.att_img = torch.empty(R_i, D, **e)
        self.att_txt = torch.empty(max(R_t, 1), D, **e)
        self.mlp_img = torch.empty(R_i, F, **e)
        self.mlp_txt = torch.empty(max(R_t, 1), F, **e)
        self.qkv = torch.zeros(3, B, H, self.S_pad, Dh, **e)  # pad rows stay 0 (finite V)
        # fp32 partials of the key-split last query block of every (b, h) (attention tail)
        nb = ops.attention_workspace_bytes(B, H, self.S_pad, S_img, S_txt)
        self.attn_split = torch.empty(max(nb // 4, 4), device=device, dtype=torch.float32)
        # split-K partial sums of the text-stream linears (fp32 / int32)
        sk = max(ops.splitk_splits(n, k, int8) * n for n, k in ((3 * D, D), (D, D), (F, D), (D, F)))
        self.splitk = torch.empty(max(R_t * sk, 4), device=device, dtype=torch.float32)
        self.txt_norm = torch.empty(max(R_t, 1), cfg.joint_attention_dim, **e)
        self.tproj = torch.empty(B, 256, **e)
        self.t_h = torch.empty(B, D, **e)
        self.t_hs = torch.empty(B, D, **e)
        self.temb = torch.empty(B, D, **e)
        self.stemb = torch.empty(B, D, **e)
        self.mod_img = torch.empty(B, 6 * D, **e)
        self.mod_txt = torch.empty(B, 6 * D, **e)
        # every block's img/txt modulation vectors, from one GEMV launch per forward
        self.mod_all = torch.empty(B, cfg.num_layers * 2 * 6 * D, **e)
        self.emb_out = torch.empty(B, 2 * D, **e)
        self.t_bf = torch.empty(B, **e)
        if int8:
            i8 = dict(device=device, dtype=torch.int8)
            f32 = dict(device=device, dtype=torch.float32)
            self.q_img = torch.empty(R_i, F, **i8)
            self.q_txt = torch.empty(max(R_t, 1), F, **i8)
            self.s_img = torch.empty(R_i, **f32)
            self.s_txt = torch.empty(max(R_t, 1), **f32)


class QwenImageTransformer2DModel(nn.Module):
    """HIP-backed QwenImageTransformer2DModel (diffusers-compatible surface)."""

    def __init__(self, patch_size: int = 2, in_channels: int = 64, out_channels: int = 16,
                 num_layers: int = 60, attention_head_dim: int = 128, num_attention_heads: int = 24,
                 joint_attention_dim: int = 3584, guidance_embeds: bool = False,
                 axes_dims_rope: Tuple[int, int, int] = (16, 56, 56), device="cuda",
                 int8_only: bool = False):
        """``int8_only``: allocate no bf16 copy of the eight quantised block linears; the
        weights then come from a pre-quantised file (``weights.load_int8``)."""
        super().__init__()
        self.config = TransformerConfig(patch_size, in_channels, out_channels, num_layers,
                                        attention_head_dim, num_attention_heads, joint_attention_dim,
                                        guidance_embeds, tuple(axes_dims_rope))
        if guidance_embeds:
            raise NotImplementedError("guidance_embeds=True is not used by Qwen-Image-Edit-2509")
        if attention_head_dim != 128:
            raise NotImplementedError("the attention kernel is specialised for head_dim 128")
        cfg = self.config
        D, Dh = cfg.inner_dim, cfg.attention_head_dim
        F = 4 * D
        P = patch_size * patch_size * out_channels
        e = dict(device=device, dtype=BF16)
        self.register_buffer("img_in_w", torch.empty(D, in_channels, **e))
        self.register_buffer("img_in_b", torch.empty(D, **e))
        self.register_buffer("txt_norm_w", torch.empty(joint_attention_dim, **e))
        self.register_buffer("txt_in_w", torch.empty(D, joint_attention_dim, **e))
        self.register_buffer("txt_in_b", torch.empty(D, **e))
        self.register_buffer("t_l1_w", torch.empty(D, 256, **e))
        self.register_buffer("t_l1_b", torch.empty(D, **e))
        self.register_buffer("t_l2_w", torch.empty(D, D, **e))
        self.register_buffer("t_l2_b", torch.empty(D, **e))
        self.register_buffer("norm_out_w", torch.empty(2 * D, D, **e))
        self.register_buffer("norm_out_b", torch.empty(2 * D, **e))
        self.register_buffer("proj_out_w", torch.empty(P, D, **e))
        self.register_buffer("proj_out_b", torch.empty(P, **e))
        # AdaLN modulation weights of all blocks packed [L * 2 * 6D, D] (block-major, img then txt):
        # the per-block w_mod_* buffers are views, and one GEMV produces every block's modulation
        # vectors at the top of the forward (13.6 GB streamed in one launch that fills the chip,
        # instead of 120 launches of 113 MB each on the blocks' critical path)
        self._mod_w = torch.empty(num_layers * 12 * D, D, **e)
        self._mod_b = torch.empty(num_layers * 12 * D, **e)
        self.transformer_blocks = nn.ModuleList(
            _Block(D, Dh, F, device, int8_only=int8_only, mod_w=self._mod_w, mod_b=self._mod_b,
                   mod_off=i * 12 * D) for i in range(num_layers))
        self.int8 = False
        self.int8_only = int8_only
        # optional kernel probe: {"attention": [...], "mlp_up": [...]} lists of
        # (start, end) torch.cuda.Event pairs recorded on the launch stream
        self.probe: Optional[Dict[str, list]] = None
        self._ws: Dict[Tuple, _Workspace] = {}
        self._rope: Dict[Tuple, Tuple[torch.Tensor, ...]] = {}
        # Text-stream work (M = B * S_txt rows: too few tiles to fill the chip) runs on a second
        # HIP stream beside the image stream; the two only meet at the joint attention (see
        # _block). False: everything on the caller's stream, in the same order (A/B switch).
        self.overlap_text_stream = True
        # With the overlap: the text stream's post-attention linears (out-proj, MLP) of block i start
        # only once the image stream's (persistent, one work-group per CU) have finished, i.e. beside
        # the next block's image LN1 + QKV launch, which is not persistent. A text work-group that
        # holds a CU when a persistent grid starts makes one of its work-groups start late, and the
        # whole launch then ends late by as much (A/B switch: False = right after the attention).
        self.defer_text_post = True
        # the text stream's post-attention half of the LAST block feeds nothing (the head reads the
        # image stream only): skipped
        self.skip_dead_text_tail = True
        # K ranges of the text-stream linears: None = ops.splitk_splits (latency-oriented), 1 =
        # one launch of full-K tiles (least CU-time: the text launches share the chip with the
        # image stream's, so what they cost is their CU-time, not their latency)
        self.text_splits: Optional[int] = 1
        self._side: Optional[torch.cuda.Stream] = None
        # image-stream QKV projection with the QK RMSNorm + RoPE in its epilogue (one launch);
        # False: the GEMM, then qie_qk_norm_rope_bf16 (A/B switch)
        self.fuse_qk_norm_rope = True
        # q is written pre-multiplied by scale*log2(e) (q_scale of the QK-norm producers, before
        # their one bf16 rounding) and the attention takes log2-unit logits straight from the
        # MFMA (qie_attention_fwd_log2q_bf16); False: plain q, scale inside (A/B switch)
        self.log2q_attention = True
        # all 120 modulation GEMVs as one launch before the blocks; False: one launch per block and
        # stream, inside the block (A/B switch)
        self.batched_modulation = True
        # Modulation cache (computed once per (timesteps, weights) and kept):
        # the timestep MLP, the 120 AdaLN modulation vectors and norm_out's vector depend only on
        # the weights and the per-row timesteps, which repeat every forward in the stream-batch
        # loop. Keyed on the host copy of the timestep values (scheduler.model_timesteps tags its
        # tensors) and on the weights' in-place version counters, and also cleared by the loaders.
        # False: recompute every forward (A/B switch).
        self.cache_modulation = True
        self._mod_cache: "OrderedDict[tuple, tuple]" = OrderedDict()
        # K % 64 requirement of the GEMM kernels for the small input projections
        if in_channels % 64 or joint_attention_dim % 64:
            raise NotImplementedError("in_channels and joint_attention_dim must be multiples of 64")

    # ------------------------------------------------------------------ diffusers-like surface
    @property
    def dtype(self) -> torch.dtype:
        return BF16

    @property
    def device(self) -> torch.device:
        return self.img_in_w.device

    @contextlib.contextmanager
    def cache_context(self, name: str):
        yield

    def _param_slot(self, name: str) -> torch.Tensor:
        """Map a diffusers state_dict name to the (view of the) packed tensor."""
        D = self.config.inner_dim
        top = {
            "img_in.weight": self.img_in_w, "img_in.bias": self.img_in_b,
            "txt_norm.weight": self.txt_norm_w,
            "txt_in.weight": self.txt_in_w, "txt_in.bias": self.txt_in_b,
            "time_text_embed.timestep_embedder.linear_1.weight": self.t_l1_w,
            "time_text_embed.timestep_embedder.linear_1.bias": self.t_l1_b,
            "time_text_embed.timestep_embedder.linear_2.weight": self.t_l2_w,
            "time_text_embed.timestep_embedder.linear_2.bias": self.t_l2_b,
            "norm_out.linear.weight": self.norm_out_w, "norm_out.linear.bias": self.norm_out_b,
            "proj_out.weight": self.proj_out_w, "proj_out.bias": self.proj_out_b,
        }
        if name in top:
            return top[name]
        parts = name.split(".")
        if parts[0] != "transformer_blocks":
            raise KeyError(name)
        blk = self.transformer_blocks[int(parts[1])]
        rest = ".".join(parts[2:])
        kind = "w" if rest.endswith("weight") else "b"
        stem = rest.rsplit(".", 1)[0]
        qkv = {"attn.to_q": ("img", 0), "attn.to_k": ("img", 1), "attn.to_v": ("img", 2),
               "attn.add_q_proj": ("txt", 0), "attn.add_k_proj": ("txt", 1),
               "attn.add_v_proj": ("txt", 2)}
        if stem in qkv:
            s, j = qkv[stem]
            return getattr(blk, f"{kind}_qkv_{s}")[j * D:(j + 1) * D]
        simple = {"img_mod.1": "mod_img", "txt_mod.1": "mod_txt", "attn.to_out.0": "out_img",
                  "attn.to_add_out": "out_txt", "img_mlp.net.0.proj": "up_img",
                  "img_mlp.net.2": "down_img", "txt_mlp.net.0.proj": "up_txt",
                  "txt_mlp.net.2": "down_txt"}
        if stem in simple:
            return getattr(blk, f"{kind}_{simple[stem]}")
        if stem.startswith("attn.norm_"):
            return getattr(blk, stem[len("attn."):])
        raise KeyError(name)

    def diffusers_names(self) -> List[str]:
        names = ["img_in.weight", "img_in.bias", "txt_norm.weight", "txt_in.weight", "txt_in.bias"]
        names += [f"time_text_embed.timestep_embedder.linear_{i}.{k}" for i in (1, 2) for k in ("weight", "bias")]
        for i in range(self.config.num_layers):
            p = f"transformer_blocks.{i}."
            for s in ("img", "txt"):
                names += [p + f"{s}_mod.1.weight", p + f"{s}_mod.1.bias"]
            for n in ("to_q", "to_k", "to_v", "add_q_proj", "add_k_proj", "add_v_proj",
                      "to_out.0", "to_add_out"):
                names += [p + f"attn.{n}.weight", p + f"attn.{n}.bias"]
            names += [p + f"attn.{n}.weight" for n in ("norm_q", "norm_k", "norm_added_q", "norm_added_k")]
            for s in ("img", "txt"):
                names += [p + f"{s}_mlp.net.{j}.weight" for j in ("0.proj", "2")]
                names += [p + f"{s}_mlp.net.{j}.bias" for j in ("0.proj", "2")]
        names += ["norm_out.linear.weight", "norm_out.linear.bias", "proj_out.weight", "proj_out.bias"]
        return names

    @torch.no_grad()
    def load_diffusers_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        """Copy diffusers-named tensors into the packed buffers."""
        seen = set()
        for k, v in sd.items():
            try:
                slot = self._param_slot(k)
            except (KeyError, IndexError):
                if strict:
                    raise KeyError(f"unexpected parameter {k}")
                continue
            if tuple(slot.shape) != tuple(v.shape):
                raise ValueError(f"{k}: shape {tuple(v.shape)} != {tuple(slot.shape)}")
            slot.copy_(v.to(slot.device, BF16))
            seen.add(k)
        if strict:
            missing = set(self.diffusers_names()) - seen
            if missing:
                raise KeyError(f"missing parameters: {sorted(missing)[:5]} ...")
        self._requantize_if_needed()

    def diffusers_state_dict(self) -> Iterator[Tuple[str, torch.Tensor]]:
        for n in self.diffusers_names():
            yield n, self._param_slot(n)

    @torch.no_grad()
    def random_init_(self, seed: int = 0, std: float = 0.02):
        """Seeded N(0, std) init of every Linear weight/bias, 1 + N(0, std) for
        RMSNorm weights, generated directly in HBM."""
        g = torch.Generator(device=self.device).manual_seed(seed)
        for n in self.diffusers_names():
            t = self._param_slot(n)
            t.normal_(0.0, std, generator=g)
            if n == "txt_norm.weight" or ".attn.norm_" in n:
                t.add_(1.0)
        self._requantize_if_needed()
        return self

    # ------------------------------------------------------------------ int8
    _I8_LINEARS = ("qkv_img", "qkv_txt", "out_img", "out_txt", "up_img", "up_txt", "down_img", "down_txt")

    @torch.no_grad()
    def quantize_int8(self):
        """Int8Linear replacement pass (README.md:136-138 'replace nn.Linear with
        Int8Linear in transformer'): per-output-channel int8 weights + fp32
        scales for every block linear, computed by the HIP quantiser."""
        if self.int8_only:
            raise RuntimeError("int8_only model: already quantised, the bf16 weights are absent")
        for blk in self.transformer_blocks:
            blk.q8 = {}
            for n in self._I8_LINEARS:
                w = getattr(blk, f"w_{n}")
                q = torch.empty(w.shape, dtype=torch.int8, device=w.device)
                s = torch.empty(w.shape[0], dtype=torch.float32, device=w.device)
                ops.quantize_rows(w, q, s)
                blk.q8[n] = (q, s)
        self.int8 = True
        self._ws.clear()
        return self

    def clear_modulation_cache(self):
        """Drop cached modulation vectors. Not needed after weight changes: in-place writes change
        the cache key (version counters) and the loaders clear it themselves."""
        self._mod_cache.clear()

    def _requantize_if_needed(self):
        self._mod_cache.clear()
        if self.int8_only:
            raise RuntimeError("this model was loaded pre-quantised (int8_only): its bf16 linear weights "
                               "are absent, so they cannot be changed and re-quantised; fuse LoRA "
                               "before weights.save_int8")
        if self.int8:
            self.quantize_int8()

    def int8_state_dict(self) -> Dict[str, torch.Tensor]:
        """On-disk int8 image: ``transformer_blocks.{i}.{linear}.q8`` (int8
        [N, K]) and ``.scale`` (fp32 [N]) for the eight quantised linears, every other packed
        buffer under its own name. Block linears are stored packed (q|k|v in one [3D, D])."""
        if not self.int8:
            raise RuntimeError("call quantize_int8() first")
        out = {}
        skip = {f"w_{n}" for n in self._I8_LINEARS}
        for name, t in self.named_buffers():
            if name.split(".")[-1] in skip:
                continue
            out[name] = t
        for i, blk in enumerate(self.transformer_blocks):
            for n, (q, sc) in blk.q8.items():
                out[f"transformer_blocks.{i}.{n}.q8"] = q
                out[f"transformer_blocks.{i}.{n}.scale"] = sc
        return out

    @torch.no_grad()
    def load_int8_state_dict(self, sd: Dict[str, torch.Tensor]):
        """Inverse of :meth:`int8_state_dict` (strict: every key, every shape)."""
        self._mod_cache.clear()
        bufs = dict(self.named_buffers())
        skip = {f"w_{n}" for n in self._I8_LINEARS}
        want = {n for n in bufs if n.split(".")[-1] not in skip}
        for i in range(self.config.num_layers):
            for n in self._I8_LINEARS:
                want |= {f"transformer_blocks.{i}.{n}.q8", f"transformer_blocks.{i}.{n}.scale"}
        if set(sd) != want:
            missing, extra = sorted(want - set(sd)), sorted(set(sd) - want)
            raise KeyError(f"int8 image mismatch: missing {missing[:4]} extra {extra[:4]}")
        dev = self.device
        for n in want:
            if n.endswith(".q8") or n.endswith(".scale"):
                continue
            if tuple(bufs[n].shape) != tuple(sd[n].shape):
                raise ValueError(f"{n}: shape {tuple(sd[n].shape)} != {tuple(bufs[n].shape)}")
            bufs[n].copy_(sd[n].to(dev, BF16))
        D, F = self.config.inner_dim, 4 * self.config.inner_dim
        shapes = {"qkv": (3 * D, D), "out": (D, D), "up": (F, D), "down": (D, F)}
        for i, blk in enumerate(self.transformer_blocks):
            blk.q8 = {}
            for n in self._I8_LINEARS:
                q, sc = sd[f"transformer_blocks.{i}.{n}.q8"], sd[f"transformer_blocks.{i}.{n}.scale"]
                if q.dtype != torch.int8 or sc.dtype != torch.float32 or tuple(q.shape) != shapes[n[:-4]] \
                        or tuple(sc.shape) != (q.shape[0],):
                    raise ValueError(f"block {i} {n}: bad int8 tensors {q.dtype}{tuple(q.shape)} "
                                     f"{sc.dtype}{tuple(sc.shape)}")
                blk.q8[n] = (q.to(dev).contiguous(), sc.to(dev).contiguous())
        self.int8 = True
        self._ws.clear()
        return self

    # ------------------------------------------------------------------ forward
    def _workspace(self, B, S_img, S_txt) -> _Workspace:
        key = (B, S_img, S_txt, self.int8)
        ws = self._ws.get(key)
        if ws is None:
            if len(self._ws) > 4:
                self._ws.clear()
            ws = _Workspace(self.config, B, S_img, S_txt, self.device, self.int8)
            self._ws[key] = ws
        return ws

    def _rope_tables(self, img_shapes, S_txt):
        key = (tuple(tuple(x) for x in img_shapes), S_txt)
        t = self._rope.get(key)
        if t is None:
            t = rope_tables(img_shapes, S_txt, self.device, self.config.axes_dims_rope)
            self._rope[key] = t
        return t

    @torch.no_grad()
    def forward(self, hidden_states: torch.Tensor, encoder_hidden_states: torch.Tensor = None,
                encoder_hidden_states_mask: Optional[torch.Tensor] = None,
                timestep: torch.Tensor = None, img_shapes=None, txt_seq_lens: Optional[Sequence[int]] = None,
                guidance: Optional[torch.Tensor] = None, attention_kwargs=None,
                controlnet_block_samples=None, return_dict: bool = True, out: Optional[torch.Tensor] = None):
        cfg = self.config
        D, H = cfg.inner_dim, cfg.num_attention_heads
        B, S_img, Cin = hidden_states.shape
        S_txt = encoder_hidden_states.shape[1]
        if controlnet_block_samples is not None:
            raise NotImplementedError("controlnet residuals are not on the reference's path")
        if txt_seq_lens is None:
            if encoder_hidden_states_mask is not None:
                txt_seq_lens = [int(x) for x in encoder_hidden_states_mask.sum(dim=1).tolist()]
            else:
                txt_seq_lens = [S_txt] * B
        txt_seq_lens = [int(x) for x in txt_seq_lens]
        if len(txt_seq_lens) != B or max(txt_seq_lens) > S_txt or min(txt_seq_lens) < 0:
            raise ValueError("txt_seq_lens must give one length <= S_txt per batch row")
        if img_shapes is None:
            raise ValueError("img_shapes is required")
        shapes = img_shapes[0] if isinstance(img_shapes[0], (list, tuple)) and \
            isinstance(img_shapes[0][0], (list, tuple)) else img_shapes
        if sum(f * h * w for f, h, w in shapes) != S_img:
            raise ValueError(f"img_shapes {shapes} do not cover {S_img} image tokens")
        if B > 16:
            raise ValueError("at most 16 batch rows per forward")

        x_in = hidden_states.to(BF16).contiguous().view(B * S_img, Cin)
        enc = encoder_hidden_states.to(BF16).contiguous().view(B * S_txt, cfg.joint_attention_dim)
        ws = self._workspace(B, S_img, S_txt)
        t = timestep.reshape(-1)
        if t.numel() not in (1, B):
            raise ValueError("timestep must have 1 or B entries")
        if t.dtype == BF16 and t.numel() == B and t.is_cuda and t.is_contiguous():
            t_bf = t
        else:
            t_bf = ws.t_bf
            t_bf.copy_(t.to(BF16).expand(B))
        icos, isin, tcos, tsin = self._rope_tables(shapes, S_txt)
        t_key = None
        host = getattr(timestep, "_qie_host", None)
        if (self.cache_modulation and self.batched_modulation and host is not None and len(host) in (1, B)
                and timestep._version == getattr(timestep, "_qie_version", None)):
            # the in-place version counters of every weight the cached vectors are made from are part
            # of the key (the per-block w_mod_* / _param_slot views share their base's counter), so a
            # write through copy_ / a state_dict view / named_buffers misses the cache
            t_key = (tuple(host) * (B // len(host)), B) + tuple(
                w._version for w in (self.t_l1_w, self.t_l1_b, self.t_l2_w, self.t_l2_b, self._mod_w,
                                     self._mod_b, self.norm_out_w, self.norm_out_b))
        if out is None:
            out = torch.empty(B, S_img, cfg.patch_size ** 2 * cfg.out_channels, dtype=BF16,
                              device=self.device)
        self._forward_impl(ws, x_in, enc, t_bf, B, S_img, S_txt, txt_seq_lens, icos, isin, tcos, tsin,
                           out.view(B * S_img, -1), t_key)
        if not return_dict:
            return (out,)
        return Transformer2DModelOutput(sample=out)

    def _forward_impl(self, ws: _Workspace, x_in, enc, t_bf, B, S_img, S_txt, txt_lens, icos, isin, tcos,
                      tsin, out2d, t_key=None):
        cfg = self.config
        D = cfg.inner_dim
        eps = 1e-6
        has_txt = S_txt > 0
        R_t = B * S_txt
        # ---- prologue: img_in, txt_norm + txt_in, timestep embedding
        ops.linear(x_in, self.img_in_w, self.img_in_b, out=ws.x_img)
        if has_txt:
            ops.rmsnorm(enc, self.txt_norm_w, out=ws.txt_norm[:R_t], eps=eps)
            ops.linear(ws.txt_norm[:R_t], self.txt_in_w, self.txt_in_b, out=ws.x_txt[:R_t])
        hit = self._mod_cache.get(t_key) if t_key is not None else None
        if hit is not None:  # same weights, same per-row timesteps: the vectors of a previous forward
            self._mod_cache.move_to_end(t_key)
            ws.mod_all.copy_(hit[0])
            ws.emb_out.copy_(hit[1])
        else:
            ops.timestep_embed(t_bf, 256, out=ws.tproj)
            ops.gemv(ws.tproj, self.t_l1_w, self.t_l1_b, out=ws.t_h)
            ops.silu(ws.t_h, out=ws.t_hs)
            ops.gemv(ws.t_hs, self.t_l2_w, self.t_l2_b, out=ws.temb)
            ops.silu(ws.temb, out=ws.stemb)
            if self.batched_modulation:
                ops.gemv(ws.stemb, self._mod_w, self._mod_b, out=ws.mod_all)
            # head modulation (AdaLayerNormContinuous, scale first): depends on temb only
            ops.gemv(ws.stemb, self.norm_out_w, self.norm_out_b, out=ws.emb_out)
            if t_key is not None:
                self._mod_cache[t_key] = (ws.mod_all.clone(), ws.emb_out.clone())
                while len(self._mod_cache) > 8:
                    self._mod_cache.popitem(last=False)
        kv_len = [S_img + l for l in txt_lens]
        side = self._side_stream() if has_txt else None
        if side is not None:  # the text stream starts from the prologue's x_txt and stemb
            side.wait_stream(torch.cuda.current_stream())
        last = len(self.transformer_blocks) - 1
        for i, blk in enumerate(self.transformer_blocks):
            self._block(blk, ws, B, S_img, S_txt, kv_len, icos, isin, tcos, tsin, eps, side,
                        txt_post=not (self.skip_dead_text_tail and i == last))
        if side is not None:  # the next forward's prologue rewrites x_txt
            torch.cuda.current_stream().wait_stream(side)
        # ---- head: AdaLayerNormContinuous (scale first; emb_out from the prologue) + proj_out
        ops.layernorm_modulate(ws.x_img, ws.emb_out[:, D:], ws.emb_out[:, :D], S_img, out=ws.h_img,
                               eps=eps)
        ops.linear(ws.h_img, self.proj_out_w, self.proj_out_b, out=out2d)

    def _side_stream(self) -> Optional[torch.cuda.Stream]:
        if not self.overlap_text_stream:
            return None
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)  # default priority, like the main stream
        return self._side

    def _block(self, blk: _Block, ws: _Workspace, B, S_img, S_txt, kv_len, icos, isin, tcos, tsin, eps,
               side: Optional[torch.cuda.Stream] = None, txt_post: bool = True):
        """One dual-stream block. The image and text streams are independent except at the
        joint attention, so with ``side`` the text stream's kernels go to that HIP stream:
          side: mod_txt, LN1, QKV (text rows of qkv), QK-norm+RoPE  -> joins main before attention
          main: mod_img, LN1, QKV (image rows of qkv), QK-norm+RoPE, [join] attention
          main: out-proj, LN2, MLP of the image stream
          side: [fork after the image MLP, or after the attention] out-proj, LN2, MLP of the text stream
        Each stream writes only its own buffers (x/h/att/mlp/mod/split-K workspace, disjoint row
        ranges of qkv); att_txt and the qkv text rows change hands at the join/fork, and the
        next block's attention waits for the side stream's next QKV, which follows this block's
        text out-proj in stream order."""
        R_t = B * S_txt
        has_txt = S_txt > 0
        main = torch.cuda.current_stream() if side is not None else None
        if self.batched_modulation:
            D6, o = 6 * self.config.inner_dim, blk.mod_off
            m_img, m_txt = ws.mod_all[:, o:o + D6], ws.mod_all[:, o + D6:o + 2 * D6]
        else:
            m_img, m_txt = ws.mod_img, ws.mod_txt
        img = ("img", ws.x_img, ws.h_img, ws.att_img, ws.mlp_img, m_img, S_img, 0)
        txt = ("txt", ws.x_txt[:R_t], ws.h_txt[:R_t], ws.att_txt[:R_t], ws.mlp_txt[:R_t], m_txt,
               S_txt, S_img)
        # ---- modulation, LN1 + modulate, fused QKV projection, QK RMSNorm + RoPE
        if has_txt:
            with self._on(side):
                self._stream_pre(blk, ws, txt, tcos, tsin, eps)
        self._stream_pre(blk, ws, img, icos, isin, eps)
        if side is not None:
            main.wait_stream(side)
        # ---- joint attention
        with self._probe("attention"):
            ops.attention(ws.qkv, kv_len, ws.att_img, ws.att_txt[:R_t] if has_txt else None, S_img, S_txt,
                          workspace=ws.attn_split, log2q=self.log2q_attention)
        # ---- out-proj + gated residual, LN2 + modulate, MLP + gated residual
        if side is not None and self.defer_text_post:
            self._stream_post(blk, ws, img, eps)
            if has_txt and txt_post:
                side.wait_stream(main)  # behind the image stream's persistent GEMMs
                with self._on(side):
                    self._stream_post(blk, ws, txt, eps)
            return
        if side is not None:
            side.wait_stream(main)
        if has_txt and txt_post:
            with self._on(side):
                self._stream_post(blk, ws, txt, eps)
        self._stream_post(blk, ws, img, eps)

    @staticmethod
    def _on(stream: Optional[torch.cuda.Stream]):
        return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()

    def _stream_pre(self, blk: _Block, ws: _Workspace, st, cos, sin, eps):
        """mod = W_mod SiLU(temb) + b; h = LN1(x)(1 + scale1) + shift1; q|k|v = h W + b into the
        stream's rows of the joint qkv buffer; per-head RMSNorm + RoPE of q and k."""
        s, x, h, att, mlp, m, rpb, seq_off = st
        D = self.config.inner_dim
        if not self.batched_modulation:
            ops.gemv(ws.stemb, getattr(blk, f"w_mod_{s}"), getattr(blk, f"b_mod_{s}"), out=m)
        # chunks of m: shift1 scale1 gate1 shift2 scale2 gate2
        nq, nk = (blk.norm_q, blk.norm_k) if s == "img" else (blk.norm_added_q, blk.norm_added_k)
        if self.int8:
            qD, sc = self._q8(ws, s, x.shape[0], D)
            ops.layernorm_modulate_i8(x, m[:, 0:D], m[:, D:2 * D], rpb, qD, sc, eps)
            inp = (qD, sc)
        else:
            ops.layernorm_modulate(x, m[:, 0:D], m[:, D:2 * D], rpb, out=h, eps=eps)
            inp = h
        qs = ops.LOG2Q_SCALE if self.log2q_attention else 1.0
        # one launch: GEMM + per-head RMSNorm + RoPE (the text stream too when its linears run unsplit)
        if self.fuse_qk_norm_rope and (s == "img" or self._txt_splits("qkv", 3 * D, D) == 1):
            if self.int8:
                wq8, sw = blk.q8[f"qkv_{s}"]
                ops.linear_qkv_norm_rope_i8(qD, sc, wq8, sw, getattr(blk, f"b_qkv_{s}"), ws.qkv, rpb, seq_off,
                                            nq, nk, cos, sin, eps, q_scale=qs)
            else:
                ops.linear_qkv_norm_rope(h, getattr(blk, f"w_qkv_{s}"), getattr(blk, f"b_qkv_{s}"), ws.qkv, rpb,
                                         seq_off, nq, nk, cos, sin, eps, q_scale=qs)
            return
        self._linear(ws, blk, s, "qkv", inp, ops.EPI_QKV, ws.qkv, rpb=rpb, seq_off=seq_off)
        ops.qk_norm_rope(ws.qkv, seq_off, rpb, nq, nk, cos, sin, eps, q_scale=qs)

    def _stream_post(self, blk: _Block, ws: _Workspace, st, eps):
        """x += gate1 (att W_out + b); h = LN2(x)(1 + scale2) + shift2;
        x += gate2 (GELU_tanh(h W_up + b) W_down + b)."""
        s, x, h, att, mlp, m, rpb, seq_off = st
        D = self.config.inner_dim
        GATE, GELU = ops.EPI_GATED_RESIDUAL, ops.EPI_GELU
        if self.int8:
            rows, F = x.shape[0], mlp.shape[1]
            qD, sc = self._q8(ws, s, rows, D)
            ops.quantize_rows(att, qD, sc)
            self._linear(ws, blk, s, "out", (qD, sc), GATE, x, gate=m[:, 2 * D:3 * D], rpb=rpb)
            ops.layernorm_modulate_i8(x, m[:, 3 * D:4 * D], m[:, 4 * D:5 * D], rpb, qD, sc, eps)
            with self._probe("mlp_up" if s == "img" else None):
                self._linear(ws, blk, s, "up", (qD, sc), GELU, mlp)
            qF, sc = self._q8(ws, s, rows, F)
            ops.quantize_rows(mlp, qF, sc)
            self._linear(ws, blk, s, "down", (qF, sc), GATE, x, gate=m[:, 5 * D:6 * D], rpb=rpb)
        else:
            self._linear(ws, blk, s, "out", att, GATE, x, gate=m[:, 2 * D:3 * D], rpb=rpb)
            ops.layernorm_modulate(x, m[:, 3 * D:4 * D], m[:, 4 * D:5 * D], rpb, out=h, eps=eps)
            with self._probe("mlp_up" if s == "img" else None):
                self._linear(ws, blk, s, "up", h, GELU, mlp)
            self._linear(ws, blk, s, "down", mlp, GATE, x, gate=m[:, 5 * D:6 * D], rpb=rpb)

    def _linear(self, ws, blk, s: str, name: str, inp, kind: int, out, gate=None, rpb: int = 1,
                seq_off: int = 0):
        """One block linear (+ fused epilogue). ``inp`` is a bf16 activation or an int8 (q, scale)
        pair. Image stream: one launch of the ring / 2-stage kernel. Text stream (M = B * S_txt,
        too few tiles to fill the chip): split-K into ``ws.splitk`` with a K-only split rule."""
        b = getattr(blk, f"b_{name}_{s}")
        if isinstance(inp, tuple):
            (xq, sx), (wq, sw) = inp, blk.q8[f"{name}_{s}"]
            if s == "txt":
                sp = self._txt_splits(name, wq.shape[0], wq.shape[1], int8=True)
                return ops.linear_splitk_i8(xq, sx, wq, sw, b, kind, out, ws.splitk, sp, gate, rpb, seq_off)
            if kind == ops.EPI_QKV:
                return ops.linear_qkv_i8(xq, sx, wq, sw, b, out, rpb, seq_off)
            if kind == ops.EPI_GATED_RESIDUAL:
                return ops.linear_gated_residual_i8(xq, sx, wq, sw, b, gate, rpb, out)
            return ops.linear_i8(xq, sx, wq, sw, b, out, act=ops.ACT_GELU if kind == ops.EPI_GELU else ops.ACT_NONE)
        w = getattr(blk, f"w_{name}_{s}")
        if s == "txt":
            sp = self._txt_splits(name, w.shape[0], w.shape[1])
            return ops.linear_splitk(inp, w, b, kind, out, ws.splitk, sp, gate, rpb, seq_off)
        if kind == ops.EPI_QKV:
            return ops.linear_qkv(inp, w, b, out, rpb, seq_off)
        if kind == ops.EPI_GATED_RESIDUAL:
            return ops.linear_gated_residual(inp, w, b, gate, rpb, out)
        return ops.linear(inp, w, b, out=out, act=ops.ACT_GELU if kind == ops.EPI_GELU else ops.ACT_NONE)

    def _txt_splits(self, name: str, N: int, K: int, int8: bool = False) -> int:
        """K ranges of text-stream linear ``name`` (qkv / out / up / down): ``text_splits`` is one
        count for all, or a {name: count} dict (missing names: 1); 0 or None = ops.splitk_splits."""
        ts = self.text_splits
        if isinstance(ts, dict):
            ts = ts.get(name, 1)
        return ts or ops.splitk_splits(N, K, int8=int8)

    @contextlib.contextmanager
    def _probe(self, name: Optional[str]):
        """Record a (start, end) event pair around one kernel launch when probing."""
        if self.probe is None or name is None or name not in self.probe:
            yield
            return
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        yield
        b.record()
        self.probe[name].append((a, b))

    @staticmethod
    def _q8(ws: _Workspace, s: str, rows: int, K: int):
        """[rows, K] int8 view of the stream's quantisation buffer + its scales."""
        q = ws.q_img if s == "img" else ws.q_txt
        sc = ws.s_img if s == "img" else ws.s_txt
        return q.view(-1)[: rows * K].view(rows, K), sc[:rows]

    # ------------------------------------------------------------------ bookkeeping
    def flops_per_forward(self, S_img: int, S_txt: int, B: int = 1) -> float:
        """Algorithmic FLOPs (2 per multiply-add of every linear and both attention products; padded rows not counted)."""
        c = self.config
        D, L = c.inner_dim, c.num_layers
        S = S_img + S_txt
        f = (L * (24 * S * D * D + 4 * S * S * D + 24 * D * D) + 2 * S_img * c.in_channels * D
             + 2 * S_txt * c.joint_attention_dim * D + 2 * (256 * D + D * D) + 4 * D * D
             + 2 * S_img * D * c.patch_size ** 2 * c.out_channels)
        return float(f) * B
