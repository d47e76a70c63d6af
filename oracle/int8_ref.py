"""Integer restatement of the Int8Linear path (W8A8, per-token x per-channel).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Reference semantics.  The snapshot's only int8 code is bitsandbytes LLM.int8
on the transformer (benchmark_int8.py:72-76, test_quantized.py:40-43); the
README names an ``Int8Linear`` "INT8 Linear layer using cuBLAS Lt GEMM" and a
"fused INT8 GEMM (quantize + matmul + dequantize)" (README.md:136-141) whose
sources are absent.  BASELINE.json north_star asks for that path as a native
int8 MFMA GEMM.  The build therefore defines W8A8 as below
and this module is its exact integer specification:

  weight   s_w[n] = max_k |W[n,k]| / 127          (fp32; 1.0 if the row is 0)
           Wq[n,k] = clamp(rint(W[n,k] * (127 / max|W[n,:]|)), -127, 127)
  act      s_a[m], xq[m,k]: same rule per row of x (dynamic, per token)
  acc      acc[m,n] = sum_k xq[m,k] * Wq[n,k]      (int32, exact)
  out      y = bf16( fma(float(acc), s_a[m]*s_w[n], bias[n]) )

``rint`` is round-half-to-even, all fp32 arithmetic is IEEE single with
round-to-nearest-even, exactly what the HIP kernels compute, so the int8
tensors and scales are bit-exact and ``acc`` is bit-exact; the bf16 output is
compared within 1 bf16 ulp (fma vs separate mul/add rounding).
"""
from __future__ import annotations

import numpy as np


def quantize_rows(x: np.ndarray):
    """Per-row symmetric int8 quantisation.  x: [R, K] float32 (bf16 values).
    Returns (q int8 [R, K], scale float32 [R])."""
    x = np.asarray(x, dtype=np.float32)
    amax = np.max(np.abs(x), axis=1).astype(np.float32)
    safe = np.where(amax > 0, amax, np.float32(1.0)).astype(np.float32)
    inv = (np.float32(127.0) / safe).astype(np.float32)
    q = np.rint((x * inv[:, None]).astype(np.float32))
    q = np.clip(q, -127, 127).astype(np.int8)
    scale = np.where(amax > 0, (amax / np.float32(127.0)).astype(np.float32), np.float32(1.0))
    q[amax == 0] = 0
    return q, scale.astype(np.float32)


def int8_gemm_acc(xq: np.ndarray, wq: np.ndarray) -> np.ndarray:
    """acc[m, n] = sum_k xq[m,k] * wq[n,k] in exact integer arithmetic."""
    return (xq.astype(np.int64) @ wq.astype(np.int64).T).astype(np.int32)


def dequant(acc: np.ndarray, sa: np.ndarray, sw: np.ndarray, bias=None) -> np.ndarray:
    """fp32 epilogue value before the bf16 rounding (computed in fp64 then
    rounded once to fp32, i.e. the fma result)."""
    scale = (sa[:, None].astype(np.float32) * sw[None, :].astype(np.float32)).astype(np.float32)
    v = acc.astype(np.float64) * scale.astype(np.float64)
    if bias is not None:
        v = v + np.asarray(bias, dtype=np.float32).astype(np.float64)[None, :]
    return v.astype(np.float32)


def int8_linear(x: np.ndarray, w: np.ndarray, bias=None) -> np.ndarray:
    """Full W8A8 linear in fp32 (pre-bf16-rounding)."""
    xq, sa = quantize_rows(x)
    wq, sw = quantize_rows(w)
    return dequant(int8_gemm_acc(xq, wq), sa, sw, bias)
