"""Bias-free linear layer whose weight gradient lands straight in the parameter server's gradient
bucket.

``ColocatedPS`` (parallel/colocated.py) gathers every step's gradients into flat per-bucket slots
that the push reads.  With ``nn.Linear`` the weight-gradient GEMM writes a fresh tensor, autograd
adopts it as ``p.grad`` and the bucket landing copies it into the slot: for Llama-3-8B that is
16 GB of bf16 gradients re-copied per step (~12 ms of multi-tensor copies on the compute stream,
profiles/r5_llama_grad_direct_ab.txt).  Here the weight-gradient GEMM writes into the slot view
itself (``torch.mm(..., out=view)``); autograd adopts the view (a fresh Tensor object, so it is
stolen, not cloned), and the landing sees ``p.grad`` already in place.

The destination is published per step by ``ColocatedPS._bind`` as ``weight._ps_gdst`` (the flat
buffer, offset and shape -- never a view Tensor, whose extra reference would make autograd clone).
Only the first gradient contribution of a step claims it; a second use of the same weight in one
graph, or gradient accumulation, falls back to the ordinary path, where autograd adds into the
already-landed view.

Reference: the reference computes the same product in its FC layer's backward
(layer/FcLayer.java: weight gradient = delta^T x) and sends it to the server as a separate copy.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import knobs

__all__ = ["GradDst", "PsLinear", "ps_linear"]


class GradDst:
    """Where this step's gradient of one parameter lives: ``buf[off:off + numel].view(shape)``."""

    __slots__ = ("buf", "off", "numel", "shape", "claimed")

    def __init__(self, buf: torch.Tensor, off: int, numel: int, shape):
        self.buf, self.off, self.numel, self.shape, self.claimed = buf, off, numel, tuple(shape), False


def _claim(w: torch.Tensor) -> Optional[torch.Tensor]:
    if knobs.disabled("ps_linear"):  # the ordinary weight gradient
        return None
    d = getattr(w, "_ps_gdst", None)
    if d is None or d.claimed or w.grad is not None or d.buf.dtype != w.dtype or d.buf.device != w.device:
        return None
    d.claimed = True
    return d.buf[d.off:d.off + d.numel].view(d.shape)


class _PsLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return F.linear(x, w)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gx = g.matmul(w)
        if ctx.needs_input_grad[1]:
            g2, x2 = g.reshape(-1, g.shape[-1]), x.reshape(-1, x.shape[-1])
            dst = _claim(w)
            if dst is not None:
                gw = torch.mm(g2.t(), x2, out=dst)
            else:
                gw = g2.t().mm(x2)
        return gx, gw


def ps_linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """y = x w^T, with the weight gradient written into the bound gradient slot when there is one."""
    return _PsLinearFn.apply(x, w)


class PsLinear(nn.Linear):
    """``nn.Linear`` (bias-free forward through ``ps_linear``; with a bias, plain ``F.linear``)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.bias is None and torch.is_grad_enabled():
            return ps_linear(x, self.weight)
        return F.linear(x, self.weight, self.bias)
