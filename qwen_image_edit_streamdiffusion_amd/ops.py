"""Tensor-level wrappers over the libqie C ABI (include/qie.h).

Every function validates shapes/dtypes/strides on the host before launching
(a bad launch on a shared GPU box is expensive), launches on the caller's
current HIP stream and raises ``QieError`` on any failure.  PyTorch only
provides device memory and the stream here.
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional, Sequence

import torch

from . import _lib

BF16 = torch.bfloat16
ACT_NONE, ACT_GELU = 0, 1


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _chk(cond: bool, msg: str):
    if not cond:
        raise ValueError(msg)


def _is2d_rowmajor(t: torch.Tensor) -> bool:
    return t.dim() == 2 and t.stride(1) == 1


def _dev(*ts):
    for t in ts:
        if t is not None:
            _chk(t.is_cuda, "libqie ops need device tensors")


# ---------------------------------------------------------------------------- linears
def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None,
           act: int = ACT_NONE) -> torch.Tensor:
    """y = act(bf16(x @ w.T + b)); x [M,K] (row stride may exceed K), w [N,K]."""
    _dev(x, w, b)
    _chk(x.dtype == BF16 and w.dtype == BF16 and b.dtype == BF16, "bf16 operands required")
    _chk(_is2d_rowmajor(x) and w.is_contiguous() and b.is_contiguous(), "row-major operands")
    M, K = x.shape
    N = w.shape[0]
    _chk(w.shape[1] == K and b.numel() == N, f"shape mismatch x{tuple(x.shape)} w{tuple(w.shape)}")
    _chk(K % 64 == 0 and N % 4 == 0, "K % 64 == 0 and N % 4 == 0 required")
    if out is None:
        out = torch.empty(M, N, dtype=BF16, device=x.device)
    _chk(_is2d_rowmajor(out) and out.shape == (M, N) and out.dtype == BF16, "bad out")
    if M <= 16 and act == ACT_NONE:
        _lib.call("qie_gemv_bf16", _p(x), x.stride(0), _p(w), _p(b), _p(out), out.stride(0), M, N, K,
                  _stream())
    else:
        _lib.call("qie_linear_bf16", _p(x), x.stride(0), _p(w), _p(b), _p(out), out.stride(0), M, N,
                  K, act, _stream())
    return out


def gemv(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None):
    """Skinny linear for M <= 16 (modulation / timestep linears)."""
    _dev(x, w, b)
    M, K = x.shape
    N = w.shape[0]
    _chk(M <= 16 and w.shape[1] == K and K % 8 == 0 and _is2d_rowmajor(x), "gemv shapes")
    _chk(w.is_contiguous() and b.numel() == N, "gemv weight [N, K] contiguous, bias [N]")
    if out is None:
        out = torch.empty(M, N, dtype=BF16, device=x.device)
    _chk(tuple(out.shape) == (M, N) and out.stride(1) == 1, "gemv out [M, N] (row stride any)")
    _lib.call("qie_gemv_bf16", _p(x), x.stride(0), _p(w), _p(b), _p(out), out.stride(0), M, N, K,
              _stream())
    return out


def linear_gated_residual(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, gate: torch.Tensor,
                          rows_per_batch: int, resid: torch.Tensor) -> torch.Tensor:
    """resid += gate[b(m)] * (x @ w.T + b) with the reference's bf16 rounding."""
    _dev(x, w, b, gate, resid)
    M, K = x.shape
    N = w.shape[0]
    _chk(_is2d_rowmajor(x) and w.shape[1] == K and resid.shape == (M, N), "gated residual shapes")
    _chk(gate.dim() == 2 and gate.stride(1) == 1 and gate.shape[1] >= N, "gate [B, >=N]")
    _chk(M % rows_per_batch == 0 and gate.shape[0] >= M // rows_per_batch, "gate batch")
    _chk(K % 64 == 0 and N % 4 == 0, "K % 64, N % 4")
    _lib.call("qie_linear_gated_residual_bf16", _p(x), x.stride(0), _p(w), _p(b), _p(gate),
              gate.stride(0), rows_per_batch, _p(resid), resid.stride(0), M, N, K, _stream())
    return resid


def linear_qkv(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, qkv: torch.Tensor,
               rows_per_batch: int, seq_offset: int) -> None:
    """Fused q|k|v projection scattered into qkv [3, B, H, S_pad, Dh]."""
    _dev(x, w, b, qkv)
    M, K = x.shape
    _, B, H, S_pad, Dh = qkv.shape
    _chk(qkv.is_contiguous() and w.shape == (3 * H * Dh, K) and b.numel() == 3 * H * Dh, "qkv shapes")
    _chk(M == B * rows_per_batch and seq_offset + rows_per_batch <= S_pad, "qkv rows")
    _chk(K % 64 == 0 and _is2d_rowmajor(x), "qkv K")
    _lib.call("qie_linear_qkv_bf16", _p(x), x.stride(0), _p(w), _p(b), _p(qkv), M, K, rows_per_batch,
              seq_offset, B, H, Dh, S_pad, _stream())


def _rope_chk(qkv, rows_per_batch, wq, wk, cos_tab, sin_tab):
    _dev(wq, wk, cos_tab, sin_tab)
    Dh = qkv.shape[-1]
    _chk(Dh == 128 and wq.numel() == Dh and wk.numel() == Dh and wq.is_contiguous() and wk.is_contiguous(),
         "norm weights [128]")
    _chk(cos_tab.dtype == torch.float32 and cos_tab.is_contiguous() and sin_tab.is_contiguous() and
         cos_tab.shape == sin_tab.shape and cos_tab.shape[0] >= rows_per_batch and cos_tab.shape[1] == 64,
         "rope table [rows_per_batch, 64] fp32")


def linear_qkv_norm_rope(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, qkv: torch.Tensor,
                         rows_per_batch: int, seq_offset: int, wq: torch.Tensor, wk: torch.Tensor,
                         cos_tab: torch.Tensor, sin_tab: torch.Tensor, eps: float = 1e-6,
                         q_scale: float = 1.0) -> None:
    """linear_qkv followed by qk_norm_rope on the same rows, fused into the GEMM epilogue
    where the shape allows (qie_linear_qkv_norm_rope_bf16)."""
    _dev(x, w, b, qkv)
    M, K = x.shape
    _, B, H, S_pad, Dh = qkv.shape
    _chk(qkv.is_contiguous() and w.shape == (3 * H * Dh, K) and b.numel() == 3 * H * Dh, "qkv shapes")
    _chk(M == B * rows_per_batch and seq_offset + rows_per_batch <= S_pad, "qkv rows")
    _chk(K % 64 == 0 and _is2d_rowmajor(x), "qkv K")
    _rope_chk(qkv, rows_per_batch, wq, wk, cos_tab, sin_tab)
    _lib.call("qie_linear_qkv_norm_rope_bf16", _p(x), x.stride(0), _p(w), _p(b), _p(qkv), M, K, rows_per_batch,
              seq_offset, B, H, Dh, S_pad, _p(wq), _p(wk), _p(cos_tab), _p(sin_tab), eps, q_scale, _stream())


# ---------------------------------------------------------------------------- norms
def layernorm_modulate(x: torch.Tensor, shift: torch.Tensor, scale: torch.Tensor, rows_per_batch: int,
                       out: Optional[torch.Tensor] = None, eps: float = 1e-6) -> torch.Tensor:
    """bf16(LN(x) * (1 + scale[b]) + shift[b]); shift/scale: [B, D] views (row stride any)."""
    _dev(x, shift, scale)
    R, D = x.shape
    _chk(_is2d_rowmajor(x) and shift.stride(1) == 1 and scale.stride(1) == 1, "ln rows")
    _chk(shift.stride(0) == scale.stride(0), "shift/scale must share a batch stride")
    _chk(R % rows_per_batch == 0 and shift.shape[0] >= R // rows_per_batch and D % 8 == 0, "ln shapes")
    if out is None:
        out = torch.empty(R, D, dtype=BF16, device=x.device)
    _lib.call("qie_layernorm_modulate_bf16", _p(x), x.stride(0), _p(shift), _p(scale), shift.stride(0),
              rows_per_batch, _p(out), out.stride(0), R, D, eps, _stream())
    return out


def layernorm_modulate_i8(x, shift, scale, rows_per_batch: int, q: torch.Tensor, qscale: torch.Tensor,
                          eps: float = 1e-6):
    _dev(x, shift, scale, q, qscale)
    R, D = x.shape
    _chk(q.dtype == torch.int8 and q.shape == (R, D) and qscale.dtype == torch.float32, "i8 out")
    _chk(shift.stride(0) == scale.stride(0) and R % rows_per_batch == 0, "ln i8")
    _lib.call("qie_layernorm_modulate_i8", _p(x), x.stride(0), _p(shift), _p(scale), shift.stride(0),
              rows_per_batch, _p(q), q.stride(0), _p(qscale), R, D, eps, _stream())


def rmsnorm(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None, eps: float = 1e-6):
    _dev(x, w)
    R, D = x.shape
    _chk(x.is_contiguous() and w.numel() == D and D % 8 == 0 and D <= 4096, "rmsnorm shapes")
    if out is None:
        out = torch.empty_like(x)
    _lib.call("qie_rmsnorm_bf16", _p(x), _p(w), _p(out), R, D, eps, _stream())
    return out


def qk_norm_rope(qkv: torch.Tensor, seg_start: int, seg_len: int, wq: torch.Tensor, wk: torch.Tensor,
                 cos_tab: torch.Tensor, sin_tab: torch.Tensor, eps: float = 1e-6, q_scale: float = 1.0):
    """Per-head RMSNorm + RoPE of the q and k rows of one segment, in place; q rows are also
    multiplied by ``q_scale`` before their rounding (LOG2Q_SCALE feeds attention(log2q=True))."""
    _dev(qkv, wq, wk, cos_tab, sin_tab)
    _, B, H, S_pad, Dh = qkv.shape
    _chk(Dh == 128 and seg_start + seg_len <= S_pad, "qk_norm_rope segment")
    _chk(cos_tab.dtype == torch.float32 and cos_tab.shape[0] >= seg_len and cos_tab.shape[1] == 64,
         "rope table [seg_len, 64] fp32")
    _chk(cos_tab.is_contiguous() and sin_tab.is_contiguous() and sin_tab.shape == cos_tab.shape, "rope")
    _lib.call("qie_qk_norm_rope_bf16", _p(qkv), B, H, Dh, S_pad, seg_start, seg_len, _p(wq), _p(wk),
              _p(cos_tab), _p(sin_tab), eps, q_scale, _stream())


def quantize_rows(x: torch.Tensor, q: torch.Tensor, scale: torch.Tensor):
    _dev(x, q, scale)
    R, D = x.shape
    _chk(q.shape == (R, D) and q.dtype == torch.int8 and scale.numel() >= R, "quantize shapes")
    _lib.call("qie_quantize_rows_i8", _p(x), x.stride(0), _p(q), q.stride(0), _p(scale), R, D, _stream())


# ---------------------------------------------------------------------------- attention
LOG2Q_SCALE = 1.4426950408889634 / math.sqrt(128)  # q_scale for attention(log2q=True), head_dim 128

def attention_workspace_bytes(B: int, H: int, S_pad: int, s_img: int, txt_rows: int) -> int:
    """Bytes of the split-key workspace ``attention(..., workspace=)`` uses (0: no split)."""
    n = ctypes.c_int64(0)
    _lib.call("qie_attention_workspace_bytes", B, H, S_pad, s_img, txt_rows, ctypes.byref(n))
    return n.value


def attention(qkv: torch.Tensor, kv_len: Sequence[int], out_img: torch.Tensor,
              out_txt: Optional[torch.Tensor], s_img: int, txt_rows: int,
              scale: Optional[float] = None, workspace: Optional[torch.Tensor] = None,
              log2q: bool = False) -> None:
    """Joint attention. With ``workspace`` (>= attention_workspace_bytes) the last query block
    of every (b, h) is split over the key range (qie_attention_fwd_split_bf16). ``log2q``: the q
    plane already holds q * scale * log2(e) (producers' ``q_scale``; qie_attention_fwd_log2q_bf16)."""
    _dev(qkv, out_img, out_txt)
    _, B, H, S_pad, Dh = qkv.shape
    _chk(Dh == 128 and S_pad % 256 == 0 and len(kv_len) == B and B <= 16, "attention shapes")
    _chk(out_img.shape == (B * s_img, H * Dh) and out_img.is_contiguous(), "out_img")
    if txt_rows:
        _chk(out_txt is not None and out_txt.shape == (B * txt_rows, H * Dh), "out_txt")
    _chk(all(0 < k <= S_pad for k in kv_len), "kv_len")
    arr = (ctypes.c_int * B)(*[int(k) for k in kv_len])
    if workspace is not None:
        _dev(workspace)
    if log2q:
        _chk(scale is None, "log2q: the scale is folded into q")
        _lib.call("qie_attention_fwd_log2q_bf16", _p(qkv), B, H, S_pad, arr, _p(out_img), _p(out_txt), s_img,
                  txt_rows, _p(workspace), 0 if workspace is None else workspace.numel() * workspace.element_size(),
                  _stream())
        return
    sc = 1.0 / math.sqrt(Dh) if scale is None else scale
    if workspace is None:
        _lib.call("qie_attention_fwd_bf16", _p(qkv), B, H, S_pad, arr, _p(out_img), _p(out_txt), s_img,
                  txt_rows, sc, _stream())
    else:
        _lib.call("qie_attention_fwd_split_bf16", _p(qkv), B, H, S_pad, arr, _p(out_img), _p(out_txt),
                  s_img, txt_rows, sc, _p(workspace), workspace.numel() * workspace.element_size(), _stream())


# ---------------------------------------------------------------------------- small ops
def timestep_embed(t: torch.Tensor, dim: int = 256, out: Optional[torch.Tensor] = None):
    _dev(t)
    _chk(t.dtype == BF16 and t.dim() == 1 and t.is_contiguous(), "t: bf16 [B]")
    if out is None:
        out = torch.empty(t.numel(), dim, dtype=BF16, device=t.device)
    _lib.call("qie_timestep_embed_bf16", _p(t), _p(out), t.numel(), dim, _stream())
    return out


def silu(x: torch.Tensor, out: Optional[torch.Tensor] = None):
    _dev(x)
    _chk(x.is_contiguous() and x.dtype == BF16, "silu")
    if out is None:
        out = torch.empty_like(x)
    _lib.call("qie_silu_bf16", _p(x), _p(out), x.numel(), _stream())
    return out


def cfg_combine(cond: torch.Tensor, uncond: torch.Tensor, scale: float,
                out: Optional[torch.Tensor] = None):
    """True-CFG combine + norm rescale over [B, rows, C] views whose per-batch
    slices are contiguous (e.g. ``out[:, :S_noise]`` of a model output)."""
    _dev(cond, uncond, out)
    _chk(cond.shape == uncond.shape and cond.dim() == 3, "cfg: [B, rows, C] views")
    B, rows, C = cond.shape
    for t in (cond, uncond):
        _chk(t.stride(2) == 1 and t.stride(1) == C, "cfg: contiguous per-batch slices")
    if out is None:
        out = torch.empty(B, rows, C, dtype=BF16, device=cond.device)
    _chk(out.shape == cond.shape and out.stride(2) == 1 and out.stride(1) == C, "cfg out")
    _lib.call("qie_cfg_combine_bf16", _p(cond), cond.stride(0), _p(uncond), uncond.stride(0), _p(out),
              out.stride(0), B, rows, C, float(scale), _stream())
    return out


def euler_step(x: torch.Tensor, v: torch.Tensor, dt: Sequence[float], out: torch.Tensor):
    """out[b] = bf16(x[b] + bf16(dt[b] * v[b])) for 2-D/3-D [B, ...] views whose
    per-batch slices are contiguous."""
    _dev(x, v, out)
    B = x.shape[0]
    n = x[0].numel()
    for t in (x, v, out):
        _chk(t.shape[0] == B and t[0].is_contiguous() and t[0].numel() == n, "euler shapes")
    _chk(len(dt) == B and B <= 16, "dt per batch row")
    arr = (ctypes.c_float * B)(*[float(d) for d in dt])
    _lib.call("qie_euler_step_bf16", _p(x), x.stride(0), _p(v), v.stride(0), _p(out), out.stride(0), B,
              n, arr, _stream())
    return out


def copy_batched(src: torch.Tensor, dst: torch.Tensor):
    """dst[b] = src[b] for [B, ...] views with contiguous per-batch slices."""
    _dev(src, dst)
    B = src.shape[0]
    n = src[0].numel()
    _chk(dst.shape[0] == B and dst[0].numel() == n and src[0].is_contiguous() and dst[0].is_contiguous(),
         "copy shapes")
    _lib.call("qie_copy_bf16", _p(src), src.stride(0), _p(dst), dst.stride(0), B, n, _stream())
    return dst


def pack_latents(x: torch.Tensor) -> torch.Tensor:
    """[B, C, H, W] (or 5-D [B, 1, C, H, W] / [B, C, 1, H, W]) -> [B, (H/2)(W/2), 4C]
    (diffusers _pack_latents views the 5-D noise by memory order)."""
    _dev(x)
    if x.dim() == 5:
        x = x.reshape(x.shape[0], x.shape[1] * x.shape[2], x.shape[3], x.shape[4])
    x = x.contiguous()
    B, C, H, W = x.shape
    y = torch.empty(B, (H // 2) * (W // 2), 4 * C, dtype=BF16, device=x.device)
    _lib.call("qie_pack_latents_bf16", _p(x), _p(y), B, C, H, W, _stream())
    return y


def unpack_latents(x: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """[B, (H/2)(W/2), 4C] -> [B, C, 1, H, W] (H, W in latent pixels)."""
    _dev(x)
    x = x.contiguous()
    B, N, C4 = x.shape
    C = C4 // 4
    _chk(N == (H // 2) * (W // 2), "unpack shape")
    y = torch.empty(B, C, 1, H, W, dtype=BF16, device=x.device)
    _lib.call("qie_unpack_latents_bf16", _p(x), _p(y), B, C, H, W, _stream())
    return y


# ---------------------------------------------------------------------------- int8 linears
def linear_i8(xq, sx, wq, sw, b, out, act: int = ACT_NONE):
    M, K = xq.shape
    N = wq.shape[0]
    _chk(xq.dtype == torch.int8 and wq.dtype == torch.int8 and wq.shape[1] == K and K % 128 == 0, "i8")
    _chk(out.shape == (M, N) and out.dtype == BF16, "i8 out")
    _lib.call("qie_linear_i8", _p(xq), xq.stride(0), _p(sx), _p(wq), _p(sw), _p(b), _p(out),
              out.stride(0), M, N, K, act, _stream())
    return out


def linear_gated_residual_i8(xq, sx, wq, sw, b, gate, rows_per_batch: int, resid):
    M, K = xq.shape
    N = wq.shape[0]
    _chk(xq.dtype == torch.int8 and wq.shape[1] == K and K % 128 == 0 and resid.shape == (M, N), "i8 gr")
    _chk(M % rows_per_batch == 0 and gate.shape[0] >= M // rows_per_batch, "i8 gate")
    _lib.call("qie_linear_gated_residual_i8", _p(xq), xq.stride(0), _p(sx), _p(wq), _p(sw), _p(b),
              _p(gate), gate.stride(0), rows_per_batch, _p(resid), resid.stride(0), M, N, K, _stream())
    return resid


def linear_qkv_i8(xq, sx, wq, sw, b, qkv, rows_per_batch: int, seq_offset: int):
    M, K = xq.shape
    _, B, H, S_pad, Dh = qkv.shape
    _chk(xq.dtype == torch.int8 and wq.shape == (3 * H * Dh, K) and K % 128 == 0, "i8 qkv")
    _chk(M == B * rows_per_batch and seq_offset + rows_per_batch <= S_pad, "i8 qkv rows")
    _lib.call("qie_linear_qkv_i8", _p(xq), xq.stride(0), _p(sx), _p(wq), _p(sw), _p(b), _p(qkv), M, K,
              rows_per_batch, seq_offset, B, H, Dh, S_pad, _stream())


def linear_qkv_norm_rope_i8(xq, sx, wq8, sw, b, qkv, rows_per_batch: int, seq_offset: int, wq, wk,
                            cos_tab, sin_tab, eps: float = 1e-6, q_scale: float = 1.0):
    M, K = xq.shape
    _, B, H, S_pad, Dh = qkv.shape
    _chk(xq.dtype == torch.int8 and wq8.shape == (3 * H * Dh, K) and K % 128 == 0, "i8 qkv")
    _chk(M == B * rows_per_batch and seq_offset + rows_per_batch <= S_pad, "i8 qkv rows")
    _rope_chk(qkv, rows_per_batch, wq, wk, cos_tab, sin_tab)
    _lib.call("qie_linear_qkv_norm_rope_i8", _p(xq), xq.stride(0), _p(sx), _p(wq8), _p(sw), _p(b), _p(qkv), M,
              K, rows_per_batch, seq_offset, B, H, Dh, S_pad, _p(wq), _p(wk), _p(cos_tab), _p(sin_tab), eps,
              q_scale, _stream())


# ---------------------------------------------------------------------------- split-K linears
EPI_BIAS, EPI_GELU, EPI_GATED_RESIDUAL, EPI_QKV = (_lib.EPI_BIAS, _lib.EPI_GELU, _lib.EPI_GATED_RESIDUAL,
                                                    _lib.EPI_QKV)

def splitk_splits(N: int, K: int, int8: bool = False) -> int:
    """K-range count for the text-stream (short-M) linears. A function of (N, K) only -- never
    of M -- so a row's arithmetic is the same at every batch size (batched CFG == sequential).
    Sized for the 256x256 gemm_pp tiles: M ~ 432 is 2 row tiles, so 2 * ceil(N / 256) tiles x
    splits should stay within one round of the 256 CUs, with >= 12 K tiles (128 B) per range."""
    steps = (K * (1 if int8 else 2)) // 128
    tiles = 2 * -(-N // 256)
    for s in range(min(max(1, 256 // tiles), steps // 12), 1, -1):
        if steps % s == 0:
            return s
    return 1


def splitk_workspace_bytes(M: int, N: int, splits: int) -> int:
    return splits * M * N * 4


def _epilogue(kind: int, out: torch.Tensor, gate=None, rows_per_batch: int = 1, seq_offset: int = 0):
    e = _lib.Epilogue()
    e.kind = kind
    e.out = _p(out)
    if kind == _lib.EPI_QKV:
        _chk(out.dim() == 5 and out.is_contiguous() and out.shape[0] == 3, "qkv [3,B,H,S_pad,Dh]")
        _, e.batch, e.heads, e.s_pad, e.head_dim = out.shape
        e.rows_per_batch, e.seq_offset = rows_per_batch, seq_offset
        _chk(seq_offset + rows_per_batch <= e.s_pad, "qkv rows")
    else:
        _chk(out.dim() == 2 and out.stride(1) == 1 and out.dtype == BF16, "out [M, N] bf16")
        e.ldo = out.stride(0)
        if kind == _lib.EPI_GATED_RESIDUAL:
            _chk(gate is not None and gate.dim() == 2 and gate.stride(1) == 1, "gate [B, >=N]")
            e.gate, e.gate_bstride, e.rows_per_batch = _p(gate), gate.stride(0), rows_per_batch
    return e


def linear_splitk(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, kind: int, out: torch.Tensor,
                  workspace: torch.Tensor, splits: int, gate=None, rows_per_batch: int = 1,
                  seq_offset: int = 0):
    """Split-K form of linear / linear_gated_residual / linear_qkv (``kind`` = _lib.EPI_*)."""
    _dev(x, w, b, out, workspace)
    M, K = x.shape
    N = w.shape[0]
    _chk(_is2d_rowmajor(x) and w.shape[1] == K and b.numel() == N, "split-K shapes")
    _chk(splits == 1 or workspace.numel() * workspace.element_size() >= splitk_workspace_bytes(M, N, splits),
         "workspace")
    e = _epilogue(kind, out, gate, rows_per_batch, seq_offset)
    _lib.call("qie_linear_splitk_bf16", _p(x), x.stride(0), _p(w), _p(b), ctypes.addressof(e), M, N, K,
              splits, _p(workspace), workspace.numel() * workspace.element_size(), _stream())
    return out


def linear_splitk_i8(xq, sx, wq, sw, b, kind: int, out: torch.Tensor, workspace: torch.Tensor,
                     splits: int, gate=None, rows_per_batch: int = 1, seq_offset: int = 0):
    M, K = xq.shape
    N = wq.shape[0]
    _chk(xq.dtype == torch.int8 and wq.dtype == torch.int8 and wq.shape[1] == K, "i8 split-K")
    _chk(splits == 1 or workspace.numel() * workspace.element_size() >= splitk_workspace_bytes(M, N, splits),
         "workspace")
    e = _epilogue(kind, out, gate, rows_per_batch, seq_offset)
    _lib.call("qie_linear_splitk_i8", _p(xq), xq.stride(0), _p(sx), _p(wq), _p(sw), _p(b),
              ctypes.addressof(e), M, N, K, splits, _p(workspace),
              workspace.numel() * workspace.element_size(), _stream())
    return out


# ---------------------------------------------------------------------------- VAE decoder
def conv_kpad(C: int, ksize: int) -> int:
    """Row length of a conv2d weight in the [Cout][ky][kx][C] layout qie_conv2d_bf16 reads."""
    return -(-(ksize * ksize * C) // 64) * 64


def conv2d(x: torch.Tensor, H: int, W: int, w: torch.Tensor, b: torch.Tensor, ksize: int = 3, up: bool = False,
           out: Optional[torch.Tensor] = None, residual: bool = False, down: bool = False) -> torch.Tensor:
    """NHWC conv as an implicit GEMM: x [H*W, C] -> [H'*W', N]. Default pad ksize//2, H' = H; ``up``:
    nearest-2x folded into the gather (H' = 2H); ``down``: stride 2 after ZeroPad2d((0,1,0,1))
    (H' = H/2). w [N, conv_kpad(C, ksize)] bf16. ``residual``: ``out`` holds the shortcut and
    receives bf16(out + bf16(conv + b))."""
    _dev(x, w, b, out)
    _chk(x.dtype == BF16 and w.dtype == BF16 and b.dtype == BF16, "bf16 operands required")
    _chk(x.dim() == 2 and x.is_contiguous() and x.shape[0] == H * W, "x: [H*W, C] contiguous")
    C = x.shape[1]
    N = w.shape[0]
    _chk(C % 8 == 0 and N % 4 == 0 and w.is_contiguous() and w.shape[1] >= conv_kpad(C, ksize), "conv shapes")
    _chk(b.numel() == N, "bias")
    _chk(not (up and down) and (not down or (ksize == 3 and H % 2 == 0 and W % 2 == 0)), "conv mode")
    P = H * W * 4 if up else (H // 2) * (W // 2) if down else H * W
    if out is None:
        _chk(not residual, "residual needs out")
        out = torch.empty(P, N, dtype=BF16, device=x.device)
    _chk(out.shape == (P, N) and out.is_contiguous() and out.dtype == BF16, "out [P, N]")
    _lib.call("qie_conv2d_bf16", _p(x), H, W, C, 1 if up else 2 if down else 0, ksize, _p(w), w.stride(0), _p(b),
              _p(out) if residual else None, _p(out), N, _stream())
    return out


def conv2d_rmsnorm(x: torch.Tensor, H: int, W: int, w: torch.Tensor, b: torch.Tensor, gamma: torch.Tensor,
                   silu: bool, ksize: int = 3, up: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """conv2d (no residual) then vae_rms_norm(+SiLU) of its output with ``gamma`` [N], in one launch
    where the kernel allows (qie_conv2d_rmsnorm_bf16)."""
    _dev(x, w, b, gamma, out)
    _chk(x.dtype == BF16 and w.dtype == BF16 and b.dtype == BF16 and gamma.dtype == BF16, "bf16 operands required")
    _chk(x.dim() == 2 and x.is_contiguous() and x.shape[0] == H * W, "x: [H*W, C] contiguous")
    C = x.shape[1]
    N = w.shape[0]
    _chk(C % 8 == 0 and N % 4 == 0 and w.is_contiguous() and w.shape[1] >= conv_kpad(C, ksize), "conv shapes")
    _chk(b.numel() == N and gamma.numel() == N and gamma.is_contiguous(), "bias / gamma")
    P = H * W * 4 if up else H * W
    if out is None:
        out = torch.empty(P, N, dtype=BF16, device=x.device)
    _chk(out.shape == (P, N) and out.is_contiguous() and out.dtype == BF16, "out [P, N]")
    _lib.call("qie_conv2d_rmsnorm_bf16", _p(x), H, W, C, 1 if up else 0, ksize, _p(w), w.stride(0), _p(b), _p(gamma),
              int(silu), _p(out), N, _stream())
    return out


def matmul_f32out(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Raw fp32 x @ w.T for bf16 row-major views (row strides may exceed K)."""
    _dev(x, w, out)
    _chk(x.dtype == BF16 and w.dtype == BF16 and _is2d_rowmajor(x) and _is2d_rowmajor(w), "bf16 row-major")
    M, K = x.shape
    N = w.shape[0]
    _chk(w.shape[1] == K and K % 64 == 0 and N % 4 == 0, "matmul shapes")
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=x.device)
    _chk(out.shape == (M, N) and out.is_contiguous() and out.dtype == torch.float32, "out fp32 [M, N]")
    _lib.call("qie_matmul_f32out_bf16", _p(x), x.stride(0), _p(w), w.stride(0), _p(out), M, N, K, _stream())
    return out


def softmax_rows(s: torch.Tensor, scale: float, out: Optional[torch.Tensor] = None,
                 causal: bool = False, ranges: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16 softmax(scale * s) per row of fp32 s [R, N]; ``out`` [R, >=N] (contiguous; columns past
    N -- the K padding of a following GEMM -- are zero-filled). ``causal``: row r keeps columns
    0..r; ``ranges`` (device int32 [P, 2], R % P == 0): row r keeps columns [ranges[r % P, 0],
    ranges[r % P, 1]) -- P rows per head when R stacks the score blocks of several heads."""
    _dev(s, out, ranges)
    _chk(s.dtype == torch.float32 and _is2d_rowmajor(s), "fp32 [rows, N]")
    R, N = s.shape
    if out is None:
        out = torch.empty(R, N, dtype=BF16, device=s.device)
    _chk(out.is_contiguous() and out.shape[0] == R and out.shape[1] >= N and out.dtype == BF16, "out")
    if ranges is not None:
        P = ranges.shape[0]
        _chk(not causal and ranges.dtype == torch.int32 and ranges.is_contiguous() and ranges.shape == (P, 2)
             and R % P == 0, "ranges int32 [period, 2], rows % period == 0")
        _lib.call("qie_softmax_rows_ranged_f32_bf16", _p(s), s.stride(0), _p(out), out.shape[1], R, N, scale,
                  _p(ranges), P, _stream())
    else:
        _lib.call("qie_softmax_rows_f32_bf16", _p(s), s.stride(0), _p(out), out.shape[1], R, N, scale,
                  int(causal), _stream())
    return out


def _span_ok(t: torch.Tensor, batch: int, bs: int) -> bool:
    """The last batch entry of a 2-D row-major view stays inside its storage."""
    R, C = t.shape
    end = t.storage_offset() + (batch - 1) * bs + (R - 1) * t.stride(0) + C
    return end * t.element_size() <= t.untyped_storage().nbytes()


def matmul_heads(x: torch.Tensor, bsx: int, w: torch.Tensor, bsw: int, out: torch.Tensor, bsy: int, batch: int,
                 group: int = 1, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Head-batched x_z . w_{z // group}^T for z < batch: x / w / out are the views of entry 0
    (row-major, [M, K] / [N, K] / [M, N]) and bs* the element strides between entries. fp32 out:
    raw scores (contiguous rows, ldy == N); bf16 out: bf16(x.w^T + bias)."""
    _dev(x, w, out, bias)
    _chk(x.dtype == BF16 and w.dtype == BF16 and _is2d_rowmajor(x) and _is2d_rowmajor(w) and _is2d_rowmajor(out),
         "bf16 row-major operands")
    M, K = x.shape
    N = w.shape[0]
    _chk(w.shape[1] == K and out.shape == (M, N) and batch >= 1 and group >= 1, "shapes")
    _chk(K % 64 == 0 and N % 4 == 0, "K % 64 == 0 and N % 4 == 0 required")
    _chk(_span_ok(x, batch, bsx) and _span_ok(w, -(-batch // group), bsw) and _span_ok(out, batch, bsy),
         "batched views exceed their storage")
    f32 = out.dtype == torch.float32
    if f32:
        _chk(out.stride(0) == N, "fp32 scores need ldy == N")
    else:
        _chk(out.dtype == BF16 and bias is not None and bias.numel() == N and bias.dtype == BF16, "bf16 out + bias")
    _lib.call("qie_matmul_batched_bf16", _p(x), x.stride(0), bsx, _p(w), w.stride(0), bsw, group,
              _p(bias) if bias is not None else None, _p(out), out.stride(0), bsy, M, N, K, batch, int(f32),
              _stream())
    return out


def vae_attention_workspace_bytes(P: int, C: int) -> int:
    n = ctypes.c_int64(0)
    _lib.call("qie_vae_attention_workspace", P, C, ctypes.byref(n))
    return int(n.value)


def vae_attention(qkv: torch.Tensor, vt: torch.Tensor, out: torch.Tensor, workspace: torch.Tensor) -> torch.Tensor:
    """Single-head flash attention of the VAE mid-block: ``qkv`` [P, >=3C] bf16 rows (q | k | v),
    ``vt`` [C, >=roundup(P, 32)] bf16 = v transposed, zero past column P; ``out`` [P, C] bf16
    (row stride may exceed C); ``workspace`` >= vae_attention_workspace_bytes(P, C) bytes."""
    _dev(qkv, vt, out, workspace)
    _chk(qkv.dtype == BF16 and vt.dtype == BF16 and out.dtype == BF16, "bf16 operands")
    _chk(_is2d_rowmajor(qkv) and _is2d_rowmajor(vt) and _is2d_rowmajor(out), "row-major 2-D views")
    P = qkv.shape[0]
    C = vt.shape[0]
    _chk(qkv.shape[1] >= 3 * C and out.shape == (P, C) and vt.shape[1] >= -(-P // 32) * 32, "vae attention shapes")
    nbytes = workspace.numel() * workspace.element_size()
    _lib.call("qie_vae_attention_bf16", _p(qkv), qkv.stride(0), _p(vt), vt.stride(0), P, C, _p(out), out.stride(0),
              _p(workspace), nbytes, _stream())
    return out


def transpose(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _dev(x, out)
    _chk(x.dtype == BF16 and _is2d_rowmajor(x), "bf16 row-major")
    R, C = x.shape
    if out is None:
        out = torch.empty(C, R, dtype=BF16, device=x.device)
    _chk(out.shape == (C, R) and _is2d_rowmajor(out), "out [C, R]")
    _lib.call("qie_transpose_bf16", _p(x), x.stride(0), _p(out), out.stride(0), R, C, _stream())
    return out


def vae_latents_in(packed: torch.Tensor, h: int, w: int, sinv: torch.Tensor, mean: torch.Tensor,
                   pq_w: torch.Tensor, pq_b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Packed latents [B, (h/2)(w/2), 64] -> post_quant_conv(z) NHWC [B*h*w, 16]."""
    _dev(packed, sinv, mean, pq_w, pq_b, out)
    B = packed.shape[0]
    _chk(packed.dtype == BF16 and packed.is_contiguous() and packed.shape[1:] == (h * w // 4, 64), "packed")
    _chk(pq_w.shape == (16, 16) and pq_w.is_contiguous() and sinv.numel() == 16 and mean.numel() == 16, "consts")
    if out is None:
        out = torch.empty(B * h * w, 16, dtype=BF16, device=packed.device)
    _chk(out.shape == (B * h * w, 16) and out.is_contiguous(), "out")
    _lib.call("qie_vae_latents_in_bf16", _p(packed), B, h, w, _p(sinv), _p(mean), _p(pq_w), _p(pq_b), _p(out),
              _stream())
    return out


def vae_rms_norm(x: torch.Tensor, gamma: torch.Tensor, silu: bool, out: Optional[torch.Tensor] = None):
    """QwenImageRMS_norm over channels (+ SiLU) of NHWC [P, C]; out may be x (in place)."""
    _dev(x, gamma, out)
    _chk(x.dtype == BF16 and x.dim() == 2 and x.is_contiguous() and gamma.numel() == x.shape[1], "rms shapes")
    if out is None:
        out = torch.empty_like(x)
    _chk(out.shape == x.shape and out.is_contiguous(), "out")
    _lib.call("qie_vae_rms_norm_bf16", _p(x), _p(gamma), _p(out), x.shape[0], x.shape[1], int(silu), _stream())
    return out


def vae_rgb_out(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Decoder output [P, >=3] bf16 -> uint8 RGB [P, 3] (clamp, postprocess, round)."""
    _dev(x, out)
    _chk(x.dtype == BF16 and _is2d_rowmajor(x) and x.shape[1] >= 3, "x [P, >=3]")
    if out is None:
        out = torch.empty(x.shape[0], 3, dtype=torch.uint8, device=x.device)
    _chk(out.shape == (x.shape[0], 3) and out.is_contiguous() and out.dtype == torch.uint8, "out")
    _lib.call("qie_vae_rgb_out", _p(x), x.stride(0), _p(out), x.shape[0], _stream())
    return out


def vae_rgb_in(rgb: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """uint8 RGB [P, 3] -> bf16 NHWC [P, 8] in [-1, 1] (channels 3..7 zero)."""
    _dev(rgb, out)
    _chk(rgb.dtype == torch.uint8 and rgb.dim() == 2 and rgb.shape[1] == 3 and rgb.is_contiguous(), "rgb [P, 3]")
    if out is None:
        out = torch.empty(rgb.shape[0], 8, dtype=BF16, device=rgb.device)
    _chk(out.shape == (rgb.shape[0], 8) and out.is_contiguous() and out.dtype == BF16, "out [P, 8]")
    _lib.call("qie_vae_rgb_in", _p(rgb), _p(out), rgb.shape[0], _stream())
    return out


def vae_latents_out(x: torch.Tensor, B: int, h: int, w: int, mean: torch.Tensor, std: torch.Tensor,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """quant_conv output NHWC [B*h*w, >=16] -> normalised, packed latents [B, (h/2)(w/2), 64]."""
    _dev(x, mean, std, out)
    _chk(x.dtype == BF16 and _is2d_rowmajor(x) and x.shape[0] == B * h * w and x.shape[1] >= 16, "x")
    if out is None:
        out = torch.empty(B, h * w // 4, 64, dtype=BF16, device=x.device)
    _chk(out.shape == (B, h * w // 4, 64) and out.is_contiguous(), "out")
    _lib.call("qie_vae_latents_out_bf16", _p(x), x.stride(0), B, h, w, _p(mean), _p(std), _p(out), _stream())
    return out


# ---------------------------------------------------------------------------- prompt encoder
def embed_rows(table: torch.Tensor, ids: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _dev(table, ids, out)
    _chk(table.dtype == BF16 and table.is_contiguous() and ids.dtype == torch.int32 and ids.is_contiguous(), "embed")
    V, D = table.shape
    if out is None:
        out = torch.empty(ids.numel(), D, dtype=BF16, device=table.device)
    _chk(out.shape == (ids.numel(), D) and out.is_contiguous(), "out")
    _lib.call("qie_embed_rows_bf16", _p(table), _p(ids), ids.numel(), D, V, _p(out), _stream())
    return out


def rope_half(x: torch.Tensor, h0: int, nh: int, head_dim: int, cos: torch.Tensor, sin: torch.Tensor,
              head_stride: Optional[int] = None):
    """In-place rotate-half RoPE on heads [h0, h0 + nh) of the rows of x (row-major view), heads
    ``head_stride`` (default head_dim) elements apart. bf16 tables: the language model's rounding;
    fp32 tables: the vision tower's (one rounding)."""
    _dev(x, cos, sin)
    hs = head_dim if head_stride is None else head_stride
    f32 = cos.dtype == torch.float32
    _chk(x.dtype == BF16 and _is2d_rowmajor(x) and cos.dtype == sin.dtype and cos.dtype in (BF16, torch.float32),
         "rope dtypes")
    _chk(cos.shape == sin.shape == (x.shape[0], head_dim) and cos.is_contiguous() and sin.is_contiguous(), "tables")
    _chk(hs >= head_dim and (h0 + nh - 1) * hs + head_dim <= x.shape[1], "heads exceed the row")
    _lib.call("qie_rope_half_bf16", _p(x), x.stride(0), x.shape[0], h0, nh, head_dim, hs, _p(cos), _p(sin),
              int(f32), _stream())


def gelu_erf_(x: torch.Tensor) -> torch.Tensor:
    """In-place nn.GELU() (erf form) on a bf16 row-major block."""
    _dev(x)
    _chk(x.dtype == BF16 and _is2d_rowmajor(x) and x.shape[1] % 8 == 0, "bf16 [rows, n % 8]")
    _lib.call("qie_gelu_erf_bf16", _p(x), x.stride(0), x.shape[0], x.shape[1], _stream())
    return x


def silu_mul(gu: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[g | u] rows -> bf16(bf16(silu(g)) * u)."""
    _dev(gu, out)
    _chk(gu.dtype == BF16 and _is2d_rowmajor(gu) and gu.shape[1] % 2 == 0, "gu [R, 2F]")
    R, F = gu.shape[0], gu.shape[1] // 2
    if out is None:
        out = torch.empty(R, F, dtype=BF16, device=gu.device)
    _chk(_is2d_rowmajor(out) and out.shape == (R, F), "out [R, F]")
    _lib.call("qie_silu_mul_bf16", _p(gu), gu.stride(0), R, F, _p(out), out.stride(0), _stream())
    return out
