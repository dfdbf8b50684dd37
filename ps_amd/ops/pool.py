"""NHWC max pooling (csrc/kernels/pool.hip) and the fused ResNet stem tail
``BN -> ReLU -> maxpool`` whose BN output never touches HBM.

Reference counterpart: layer/PoolingLayer.java:62-134 (max pool with recorded argmax and a
scatter backward).  GPU tensors (bf16, channels_last, C % 8 == 0) take the HIP path; other
inputs use ``F.max_pool2d`` -- the numerics oracle in tests/test_pool_gpu.py.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._ext import native


def _nhwc(x: torch.Tensor) -> torch.Tensor:
    """NCHW channels_last tensor -> its [N, H, W, C] contiguous view."""
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    return x.permute(0, 2, 3, 1)


def _hip_ok(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0


class _MaxPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, idx = native().maxpool_nhwc_fwd(_nhwc(x), None, k, s, p)
        ctx.save_for_backward(idx)
        ctx.geo = (x.shape[2], x.shape[3], k, s, p)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        h, w, k, s, p = ctx.geo
        dx = native().maxpool_nhwc_bwd(_nhwc(dy).contiguous(), idx, h, w, k, s, p)
        return dx.permute(0, 3, 1, 2), None, None, None


def max_pool2d(x: torch.Tensor, k: int, s: int, p: int = 0) -> torch.Tensor:
    if _hip_ok(x):
        return _MaxPoolNHWC.apply(x, int(k), int(s), int(p))
    return F.max_pool2d(x, k, s, p)


class MaxPool2d(nn.MaxPool2d):
    """nn.MaxPool2d that runs the NHWC HIP kernel on channels_last bf16 GPU tensors."""

    def forward(self, x):
        if _hip_ok(x) and self.dilation in (1, (1, 1)) and not self.ceil_mode and not self.return_indices:
            k = self.kernel_size if isinstance(self.kernel_size, int) else self.kernel_size[0]
            s = self.stride if isinstance(self.stride, int) else self.stride[0]
            p = self.padding if isinstance(self.padding, int) else self.padding[0]
            return max_pool2d(x, k, s, p)
        return super().forward(x)


class _BnReluMaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, rmean, rvar, momentum, eps, k, s, p):
        xn = _nhwc(x)
        x2 = xn.reshape(-1, x.shape[1])
        mean, invstd, coef = native().bn_stats(x2, gamma, beta, rmean, rvar, True, float(momentum), float(eps))
        y, idx = native().maxpool_nhwc_fwd(xn, coef, k, s, p)
        ctx.save_for_backward(x2, gamma, mean, invstd, coef, idx)
        ctx.geo = (x.shape, k, s, p)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x2, gamma, mean, invstd, coef, idx = ctx.saved_tensors
        shape, k, s, p = ctx.geo
        n, c, h, w = shape
        dz = native().maxpool_nhwc_bwd(_nhwc(dy).contiguous(), idx, h, w, k, s, p)
        dx2, _, dg, db = native().bn_act_bwd(dz.reshape(-1, c), None, x2, gamma, mean, invstd, 1, False,
                                             gamma is not None, coef)
        dx = dx2.view(n, h, w, c).permute(0, 3, 1, 2)
        return dx, dg, db, None, None, None, None, None, None, None


def bn_relu_maxpool(x: torch.Tensor, bn: nn.BatchNorm2d, k: int, s: int, p: int) -> torch.Tensor:
    """maxpool(relu(bn(x))) in two HIP passes over x (statistics, then BN-apply + ReLU + pool);
    training-mode HIP path only, anything else composes the unfused modules."""
    if (_hip_ok(x) and bn.training and bn.track_running_stats and bn.weight is not None
            and bn.weight.dtype == torch.float32 and bn.running_mean.dtype == torch.float32):
        bn.num_batches_tracked.add_(1)
        mom = bn.momentum if bn.momentum is not None else 0.1
        return _BnReluMaxPool.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, mom, bn.eps, k, s, p)
    y = bn(x)
    if getattr(bn, "act", "relu") == "none" or type(bn) is nn.BatchNorm2d:
        y = torch.relu(y)
    return max_pool2d(y, k, s, p)


class _GlobalAvgPoolNHWC(torch.autograd.Function):
    """[N, C, H, W] channels_last -> [N, C] mean.  The backward writes the broadcast gradient
    straight in NHWC order (one vectorised expand-copy), instead of the NCHW-shaped adaptive-pool
    gradient plus a channels_last transpose in its consumer."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        return F.adaptive_avg_pool2d(x, 1).flatten(1)

    @staticmethod
    def backward(ctx, g):
        n, c, h, w = ctx.shape
        gx = (g * (1.0 / (h * w))).to(g.dtype)[:, None, None, :].expand(n, h, w, c).contiguous()
        return gx.permute(0, 3, 1, 2)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """AdaptiveAvgPool2d(1) + flatten; channels_last GPU tensors get the NHWC backward."""
    if x.is_cuda and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        return _GlobalAvgPoolNHWC.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
