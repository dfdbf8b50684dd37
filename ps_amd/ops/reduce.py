"""Bucket / reduction ops: squared norm, clip factor, cast, axpy, N-way reduce, lerp."""
from __future__ import annotations

import torch

from ._ext import native, use_native


def sumsq(x: torch.Tensor, out: torch.Tensor | None = None, accumulate: bool = False) -> torch.Tensor:
    """Deterministic sum of squares of a flat buffer into ``out`` (float32[1])."""
    if out is None:
        out = torch.zeros(1, dtype=torch.float32, device=x.device)
    if use_native(x):
        native().sumsq(x.contiguous(), out, bool(accumulate))
        return out
    v = x.float().pow(2).sum().reshape(1)
    if accumulate:
        out.add_(v)
    else:
        out.copy_(v)
    return out


def clip_factor(sq: torch.Tensor, max_norm: float, factor: torch.Tensor | None = None) -> torch.Tensor:
    if factor is None:
        factor = torch.empty(1, dtype=torch.float32, device=sq.device)
    if use_native(sq):
        native().clip_factor(sq, float(max_norm), factor)
        return factor
    factor.copy_(torch.clamp(max_norm / (torch.sqrt(sq) + 1e-6), max=1.0))
    return factor


def cast_(x: torch.Tensor, y: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    """y = scale * x with dtype conversion (bf16 <-> fp32)."""
    if use_native(x, y):
        native().cast_(x, y, float(scale))
        return y
    y.copy_((x.float() * scale).reshape(y.shape))
    return y


def axpy_(a: float, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """y += a * x (bucket accumulate; reference KVStore.sum, store/KVStore.java:192-200)."""
    if use_native(x, y):
        native().axpy_(float(a), x, y)
        return y
    y.copy_((y.float() + a * x.float().reshape(y.shape)).to(y.dtype))
    return y


def reduce_n(x: torch.Tensor, y: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    """y = scale * sum_k x[k]  for x of shape [k, n] (server N-way reduce, fixed order)."""
    if use_native(x, y):
        native().reduce_n(x, y, float(scale))
        return y
    acc = torch.zeros(x.shape[1], dtype=torch.float32, device=x.device)
    for k in range(x.shape[0]):
        acc += x[k].float()
    y.copy_((acc * scale).reshape(y.shape))
    return y


def lerp(w0: torch.Tensor, w: torch.Tensor, s: float, out: torch.Tensor) -> torch.Tensor:
    """out = s*w0 + (1-s)*w (loss-surface interpolation, store/KVStore.java:153-155)."""
    if use_native(w0, w):
        native().lerp(w0, w, float(s), out)
        return out
    out.copy_((s * w0 + (1 - s) * w).reshape(out.shape))
    return out
