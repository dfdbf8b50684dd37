"""1x1 stride-1 convolution on channels_last bf16 activations, routed per direction to the
faster backend measured on MI355X (scripts/probe_convs.py, profiles/r1_conv_probe_b512.jsonl).

A 1x1 conv over NHWC is a plain GEMM on the [N*H*W, C] view.  At ResNet-50 shapes (batch
512) hipBLASLt beats MIOpen's solvers for the forward when C_in >= 1024 (e.g. 14x14
1024->256: 56 vs 80 us) and for the data gradient when C_in >= 256 (e.g. 56x56 256->64:
261 vs 364 us), while MIOpen wins the small-channel layer1 shapes and every weight
gradient (hipBLASLt has no split-K for K = N*H*W).  The GEMM routes also skip MIOpen's
zero-fill / cast side kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

FWD_GEMM_MIN_CIN = 1024
BWD_DATA_GEMM_MIN_CIN = 256


def _rows(x: torch.Tensor) -> torch.Tensor:
    n, c, h, w = x.shape
    return x.permute(0, 2, 3, 1).reshape(n * h * w, c)


class _Conv1x1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        n, ci, h, wd = x.shape
        co = w.shape[0]
        w2 = w.view(co, ci)
        if ci >= FWD_GEMM_MIN_CIN:
            y = (_rows(x) @ w2.t()).view(n, h, wd, co).permute(0, 3, 1, 2)
        else:
            y = F.conv2d(x, w)
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        n, ci, h, wd = x.shape
        co = w.shape[0]
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        gemm_data = ctx.needs_input_grad[0] and ci >= BWD_DATA_GEMM_MIN_CIN
        if gemm_data:
            dx = (_rows(dy) @ w.view(co, ci)).view(n, h, wd, ci).permute(0, 3, 1, 2)
        mask = [ctx.needs_input_grad[0] and not gemm_data, ctx.needs_input_grad[1], False]
        if any(mask):
            gx, gw, _ = torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                            mask)
            if mask[0]:
                dx = gx
            dw = gw
        return dx, dw


class Conv1x1(nn.Conv2d):
    """nn.Conv2d(cin, cout, 1, bias=False) with per-direction backend routing on GPU bf16
    channels_last inputs (same parameters / state_dict as nn.Conv2d)."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__(in_channels, out_channels, 1, bias=False)

    def forward(self, x):
        if (x.is_cuda and x.dtype == torch.bfloat16 and self.weight.dtype == torch.bfloat16 and x.dim() == 4
                and x.is_contiguous(memory_format=torch.channels_last)
                and self.weight.is_contiguous(memory_format=torch.channels_last)):
            return _Conv1x1.apply(x, self.weight)
        return super().forward(x)
