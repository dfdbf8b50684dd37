"""1x1 stride-1 convolution on channels_last bf16 activations, routed per direction to the
faster backend measured on MI355X (scripts/probe_convs.py, profiles/archive/r1_conv_probe_b512.jsonl).

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

from .. import knobs

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


# ------------------------------------------------------------------------------ ResNet stem
def pack_stem_weight(w: torch.Tensor) -> torch.Tensor:
    """[64, C<=4, 7, 7] -> [64, 224] bf16 with k' = kh*32 + kw*4 + c (csrc/kernels/stem.hip);
    the kw = 7 and c >= C slots are zero."""
    wp = torch.zeros(64, 7, 8, 4, dtype=torch.bfloat16, device=w.device)
    wp[:, :, :7, :w.shape[1]] = w.permute(0, 2, 3, 1).to(torch.bfloat16)
    return wp.view(64, 224)


def unpack_stem_grad(dwp: torch.Tensor, cin: int) -> torch.Tensor:
    return dwp.view(64, 7, 8, 4)[:, :, :7, :cin].permute(0, 3, 1, 2).contiguous()


def nhwc_in(x: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] (C = 3 or 4) -> contiguous [N, H, W, C] bf16 -- a view for channels_last
    bf16 input; the kernel reads 3-channel pixels directly (no padding copy)."""
    xn = x.to(torch.bfloat16).permute(0, 2, 3, 1)
    return xn if xn.is_contiguous() else xn.contiguous()


class _StemConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        from ._ext import native

        x4 = nhwc_in(x)
        z = native().stem_conv_fwd(x4, pack_stem_weight(w))[0]
        ctx.save_for_backward(x4, w)
        ctx.xshape = x.shape
        return z.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dz):
        from ._ext import native

        x4, w = ctx.saved_tensors
        dzn = dz.permute(0, 2, 3, 1)
        if not dzn.is_contiguous():
            dzn = dzn.contiguous()
        dw = unpack_stem_grad(native().stem_conv_wrw(x4, dzn), w.shape[1]).to(w.dtype) \
            if ctx.needs_input_grad[1] else None
        dx = None
        if ctx.needs_input_grad[0]:  # the stem input normally needs no gradient
            x = x4[..., :ctx.xshape[1]].permute(0, 3, 1, 2)
            dx = torch.ops.aten.convolution_backward(dz, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                                     [True, False, False])[0]
        return dx, dw


class StemConv(nn.Conv2d):
    """nn.Conv2d(cin<=4, 64, 7, stride 2, pad 3, bias=False); on GPU bf16 it runs the MFMA stem
    kernels (csrc/kernels/stem.hip), elsewhere plain conv2d.  Inputs may carry a 4th zero
    channel (NHWC4) for the fast path; the CPU path ignores it."""

    def __init__(self, in_channels: int = 3):
        super().__init__(in_channels, 64, 7, stride=2, padding=3, bias=False)

    def forward(self, x):
        if (x.is_cuda and x.dtype == torch.bfloat16 and self.weight.dtype == torch.bfloat16 and x.shape[3] <= 256
                and x.shape[1] in (3, 4)):
            return _StemConv.apply(x, self.weight)
        if x.shape[1] != self.in_channels:
            x = x[:, :self.in_channels]
        return super().forward(x)


class _StemBnReluMaxPool(torch.autograd.Function):
    """conv7x7/2 -> BN (batch stats) -> ReLU -> maxpool 3x3/2 in three HIP kernels:
    (1) MFMA stem conv with the BN partial sums in its epilogue, (2) BN finalize (+ running
    stats), (3) BN-apply + ReLU + max pool with a 1-byte argmax.  Backward: pool scatter ->
    BN backward (ReLU mask recomputed from z) -> MFMA weight gradient."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, rmean, rvar, momentum, eps):
        from ._ext import native

        xin = nhwc_in(x)
        kshift = rmean.detach().clone()  # shift for the partial sums (~ the batch mean)
        z, part = native().stem_conv_fwd(xin, pack_stem_weight(w), kshift)
        n, oh, ow, c = z.shape
        mean, invstd, coef = native().bn_finalize_sums(part, kshift, n * oh * ow, gamma, beta, rmean, rvar,
                                                       float(momentum), float(eps))
        y, idx = native().maxpool_nhwc_fwd(z, coef, 3, 2, 1)
        ctx.save_for_backward(xin, w, z, gamma, mean, invstd, coef, idx)
        ctx.cin = x.shape[1]
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        from ._ext import native

        xin, w, z, gamma, mean, invstd, coef, idx = ctx.saved_tensors
        n, oh, ow, c = z.shape
        dyn = dy.permute(0, 2, 3, 1)
        dyn = dyn if dyn.is_contiguous() else dyn.contiguous()
        fusable = oh % 2 == 0 and ow % 2 == 0 and 256 % (c // 8) == 0 and knobs.enabled("pool_bn_bwd")
        if fusable and c == 64 and knobs.enabled("stem_bwd_fused"):
            # statistics pass, then the weight gradient computing each dz row itself from the
            # pooled gradient (csrc/kernels/stem.hip FUSED): dz is never written
            dwp, dg, db = native().stem_bwd_fused(xin, dyn, idx, z, coef, gamma, mean, invstd)
            return None, unpack_stem_grad(dwp, w.shape[1]).to(w.dtype), dg, db, None, None, None, None
        if fusable:
            # pool scatter fused into both BN-backward passes: the full-resolution pool gradient
            # is never written (csrc/kernels/pool.hip pool_bn_bwd_kernel)
            dz, dg, db = native().pool_bn_bwd(dyn, idx, z, coef, gamma, mean, invstd)
        else:
            dpool = native().maxpool_nhwc_bwd(dyn, idx, oh, ow, 3, 2, 1)
            dz, _, dg, db = native().bn_act_bwd(dpool.view(-1, c), None, z.view(-1, c), gamma, mean, invstd, 1, False,
                                                True, coef)
        dw = unpack_stem_grad(native().stem_conv_wrw(xin, dz.view(n, oh, ow, c)), w.shape[1]).to(w.dtype)
        return None, dw, dg, db, None, None, None, None


def stem_bn_relu_maxpool(x: torch.Tensor, conv: nn.Conv2d, bn: nn.BatchNorm2d) -> torch.Tensor:
    """maxpool3x3/2(relu(bn(conv(x)))) for the ResNet stem; fused HIP path for training-mode
    bf16 GPU input, the composed modules elsewhere."""
    if (isinstance(conv, StemConv) and x.is_cuda and x.dtype == torch.bfloat16 and conv.weight.dtype == torch.bfloat16
            and x.shape[1] in (3, 4) and x.shape[3] <= 256 and not x.requires_grad and bn.training
            and bn.track_running_stats and bn.weight is not None and bn.weight.dtype == torch.float32):
        bn.num_batches_tracked.add_(1)
        mom = bn.momentum if bn.momentum is not None else 0.1
        return _StemBnReluMaxPool.apply(x, conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var, mom,
                                        bn.eps)
    from .pool import bn_relu_maxpool

    return bn_relu_maxpool(conv(x), bn, 3, 2, 1)
