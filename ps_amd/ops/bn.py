"""Fused BatchNorm (+ residual add) + ReLU for channels_last bf16 activations.

GPU path: csrc/kernels/bn_act.hip (stats + apply forward, reduce + apply backward -- two
passes over HBM each way instead of MIOpen BN + separate add / ReLU / ReLU' kernels).
CPU path (and any non-NHWC / non-bf16 input): plain torch ``F.batch_norm`` + add + relu,
which is also the numerics oracle in tests/test_bn_gpu.py.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._ext import native

ACT = {"none": 0, "relu": 1}


def _as_rows(x: torch.Tensor) -> torch.Tensor:
    """NCHW channels_last tensor -> [N*H*W, C] view (no copy)."""
    n, c, h, w = x.shape
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    return x.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _from_rows(y2: torch.Tensor, shape) -> torch.Tensor:
    n, c, h, w = shape
    return y2.view(n, h, w, c).permute(0, 3, 1, 2)


class _BnActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, gamma, beta, rmean, rvar, training, momentum, eps, act):
        shape = x.shape
        x2 = _as_rows(x)
        r2 = _as_rows(res) if res is not None else None
        y2, mean, invstd, coef = native().bn_act_fwd(x2, r2, gamma, beta, rmean, rvar, bool(training),
                                                    float(momentum), float(eps), int(act))
        if act and res is None:
            # relu mask recomputed from x * scale + shift in backward: y is not re-read
            ctx.save_for_backward(x2, None, gamma, mean, invstd, coef)
        else:
            ctx.save_for_backward(x2, y2 if act else None, gamma, mean, invstd, None)
        ctx.act, ctx.has_res, ctx.shape = act, res is not None, shape
        ctx.affine = gamma is not None
        return _from_rows(y2, shape)

    @staticmethod
    def backward(ctx, dy):
        x2, y2, gamma, mean, invstd, coef = ctx.saved_tensors
        dy2 = _as_rows(dy)
        dx2, dres2, dg, db = native().bn_act_bwd(dy2, y2, x2, gamma, mean, invstd, int(ctx.act), ctx.has_res,
                                                 ctx.affine, coef)
        dx = _from_rows(dx2, ctx.shape)
        dres = _from_rows(dres2, ctx.shape) if ctx.has_res else None
        return dx, dres, (dg if ctx.affine else None), (db if ctx.affine else None), None, None, None, None, None, \
            None


def bn_act(x: torch.Tensor, weight, bias, running_mean, running_var, training: bool, momentum: float, eps: float,
           act: str = "relu", residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    use_hip = (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0
               and (weight is None or weight.dtype == torch.float32)
               and (running_mean is None or running_mean.dtype == torch.float32)
               and (residual is None or residual.dtype == torch.bfloat16))
    if use_hip:
        return _BnActFn.apply(x, residual, weight, bias, running_mean, running_var, training, momentum, eps, ACT[act])
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return torch.relu(y) if act == "relu" else y


class BatchNormAct2d(nn.BatchNorm2d):
    """nn.BatchNorm2d (same parameter / buffer names) with the activation and an optional
    residual add fused in: ``forward(x, residual=None)``."""

    def __init__(self, num_features: int, act: str = "relu", eps: float = 1e-5, momentum: float = 0.1):
        super().__init__(num_features, eps=eps, momentum=momentum)
        self.act = act

    def forward(self, x, residual=None):
        training = self.training or not self.track_running_stats
        if self.training and self.track_running_stats:
            self.num_batches_tracked.add_(1)
        return bn_act(x, self.weight, self.bias, self.running_mean if not training or self.track_running_stats
                      else None, self.running_var if not training or self.track_running_stats else None,
                      training, self.momentum if self.momentum is not None else 0.1, self.eps, self.act, residual)
