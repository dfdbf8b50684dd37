"""MFMA fused linear: y = act(x @ w^T + b) -- the reference FcLayer (layer/FcLayer.java:74-110).

Forward: ONE kernel, GEMM + bias + activation epilogue (bf16: csrc/kernels/dense.hip gemm_nt on
v_mfma_f32_16x16x32_bf16; fp32: csrc/kernels/fc.hip on v_mfma_f32_16x16x4_f32).
Backward (K2): two kernels (csrc/kernels/fc.hip) -- dW with the activation backward folded into
the prologue and db reduced from the same staged tile, dX with the same prologue; dy, y, x and
W are read in place (the transposes happen while staging into LDS).  CPU tensors use torch
(the numerics oracle).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from .. import knobs
from ._ext import native

ACT_NONE, ACT_RELU, ACT_LEAKY, ACT_SIGMOID = 0, 1, 2, 3


def _act_ref(z, act):
    if act == ACT_RELU:
        return torch.relu(z)
    if act == ACT_LEAKY:
        return F.leaky_relu(z, 0.01)
    if act == ACT_SIGMOID:
        return 0.001 + 0.998 * torch.sigmoid(z)
    return z


def gemm_nt(a: torch.Tensor, b: torch.Tensor, bias: Optional[torch.Tensor] = None, act: int = 0,
            out_dtype=torch.bfloat16) -> torch.Tensor:
    """act(a @ b^T + bias) with a [M,K], b [N,K] bf16 (HIP MFMA on GPU)."""
    if a.is_cuda:
        c = torch.empty(a.shape[0], b.shape[0], dtype=out_dtype, device=a.device)
        native().gemm_nt(a.contiguous(), b.contiguous(), c, bias, int(act), 1.0, False)
        return c
    z = a.float() @ b.float().t()
    if bias is not None:
        z = z + bias.float()
    return _act_ref(z, act).to(out_dtype)


class _LinearAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act):
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        if w.dtype == torch.float32:
            y = torch.empty(x2.shape[0], w.shape[0], dtype=torch.float32, device=x.device)
            native().fc_fwd_f32(x2, w.contiguous(), b.float().contiguous() if b is not None else None, y, int(act))
        else:
            y = gemm_nt(x2, w, b.float() if b is not None else None, act)
        ctx.save_for_backward(x2, w, y)
        ctx.act, ctx.has_b, ctx.xshape, ctx.bdtype = act, b is not None, x.shape, (b.dtype if b is not None else None)
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0]).contiguous().to(w.dtype)
        want_dx, want_dw = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        want_db = ctx.has_b and ctx.needs_input_grad[2]
        dx = torch.empty_like(x2) if want_dx else None
        dw = torch.empty_like(w) if (want_dw or want_db) else None
        db = torch.empty(w.shape[0], dtype=torch.float32, device=w.device) if want_db else None
        native().fc_bwd(dy2, y, x2, w.contiguous(), dw, db, dx, int(ctx.act))
        return ((dx.view(ctx.xshape) if dx is not None else None), (dw if want_dw else None),
                (db.to(ctx.bdtype) if db is not None else None), None)


def linear_act(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], act: int = 0) -> torch.Tensor:
    """act(x @ w^T + b); GPU fp32 / bf16 weights run the fused MFMA kernels (fwd + K2 bwd)."""
    if x.is_cuda and w.dtype in (torch.bfloat16, torch.float32):
        return _LinearAct.apply(x.to(w.dtype), w, b, int(act))
    z = F.linear(x.to(w.dtype), w, b)
    return _act_ref(z, act)


# ------------------------------------------------------------------------------ split-K weight gradient
def _wgrad_ok(x2: torch.Tensor, dy2: torch.Tensor) -> bool:
    """Long-reduction, small-output weight gradients (BERT: 32K tokens into a 768 x 2304 dW make
    27 output tiles of 256 x 256, which hipBLASLt runs on 27 of the 256 CUs at 200-500 TF/s) go
    to the split-M wide-tile kernel of csrc/kernels/convgemm.hip as a 1x1 "convolution"."""
    import os

    T, K = x2.shape
    N = dy2.shape[1]
    return (x2.is_cuda and x2.dtype == torch.bfloat16 and dy2.dtype == torch.bfloat16 and N % 128 == 0
            and K % 128 == 0 and (N % 256 == 0 or K % 256 == 0) and T >= 4096 and T < 2 ** 31
            and (N // 256 + 1) * (K // 256 + 1) < 256 and knobs.enabled("splitk_wgrad"))


def linear_wgrad(dy2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """dW [N, K] = dy2^T x2 (fp32 accumulation, fixed-order split reduction)."""
    if _wgrad_ok(x2, dy2):
        T = x2.shape[0]
        return native().conv_wgrad(dy2, x2, [T, 1, T, 1, 1, 1, 0])
    return dy2.t() @ x2


class _SplitKLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, relu=False):
        ctx.has_b = b is not None
        ctx.relu = relu
        if relu:  # bias + ReLU in the GEMM epilogue (hipBLASLt RELU_BIAS): no separate activation pass
            y = torch._addmm_activation(b, x.reshape(-1, x.shape[-1]), w.t()).view(*x.shape[:-1], w.shape[0])
            ctx.save_for_backward(x, w, y)
            return y
        ctx.save_for_backward(x, w)
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        if ctx.relu:
            x, w, y = ctx.saved_tensors
            dy = torch.ops.aten.threshold_backward(dy, y, 0)  # ReLU'(y), the pass nn.ReLU's backward was
        else:
            x, w = ctx.saved_tensors
        n, k = w.shape
        dy2 = dy.reshape(-1, n)
        dy2 = dy2 if dy2.is_contiguous() else dy2.contiguous()
        dx = (dy2 @ w).view(x.shape) if ctx.needs_input_grad[0] else None
        dw = db = None
        want_db = ctx.has_b and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, k)
            x2 = x2 if x2.is_contiguous() else x2.contiguous()
            if want_db and _wgrad_ok(x2, dy2):
                # bias gradient from the dz tiles the split-K kernel stages anyway (one pass over dy)
                dw, db = native().linear_wgrad_db(dy2, x2)
                db = db.to(w.dtype)
            else:
                dw = linear_wgrad(dy2, x2)
            dw = dw.to(w.dtype)
        if want_db and db is None:
            db = dy2.sum(0).to(w.dtype)
        return dx, dw, db, None


class _SplitKLinearFork(torch.autograd.Function):
    """(x W^T + b, x): the layer's input passed through as a second output, so a residual use of x
    hands its gradient to THIS backward, which folds it into the data-gradient GEMM
    (dx = dxr + dy W as one beta = 1 GEMM) -- autograd would otherwise sum the two branch gradients with a
    separate add pass over [tokens, D] (25 per BERT-base step)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return F.linear(x, w, b), x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dxr):
        x, w = ctx.saved_tensors
        n, k = w.shape
        dy2 = dy.reshape(-1, n)
        dy2 = dy2 if dy2.is_contiguous() else dy2.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if dxr is not None and dxr.is_contiguous() and dxr.dtype == dy2.dtype:
                # one GEMM with beta = 1 into a NEW buffer: the incoming residual gradient is not
                # guaranteed to be exclusively ours (hooks, retain_grad), so it is never written
                dx = torch.addmm(dxr.view(-1, k), dy2, w).view(x.shape)
            else:
                dx = (dy2 @ w).view(x.shape)
                if dxr is not None:
                    dx = dx + dxr
        want_db = ctx.has_b and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, k)
            x2 = x2 if x2.is_contiguous() else x2.contiguous()
            if want_db and _wgrad_ok(x2, dy2):
                dw, db = native().linear_wgrad_db(dy2, x2)
                db = db.to(w.dtype)
            else:
                dw = linear_wgrad(dy2, x2)
            dw = dw.to(w.dtype)
        if want_db and db is None:
            db = dy2.sum(0).to(w.dtype)
        return dx, dw, db


class SplitKLinear(torch.nn.Linear):
    """nn.Linear (same parameters / state_dict) whose weight gradient runs split-K on GPU bf16
    when the reduction (tokens) is long and the output small (``linear_wgrad``).  ``fuse_relu``:
    the layer applies ReLU itself, in the GEMM epilogue on GPU bf16 (``mlp`` sets it and puts a
    parameter-free ``nn.Identity`` where the ``nn.ReLU`` was, so state_dict keys do not move)."""

    fuse_relu = False

    def fork(self, x):
        """(self(x), x) where the second output's gradient is added inside this layer's data-gradient
        GEMM -- for an input that also feeds a residual (BertLayer)."""
        if (knobs.enabled("linear_fork") and not self.fuse_relu and x.is_cuda and x.dtype == torch.bfloat16
                and self.weight.dtype == torch.bfloat16 and torch.is_grad_enabled()):
            return _SplitKLinearFork.apply(x, self.weight, self.bias)
        return self(x), x

    def forward(self, x):
        if x.is_cuda and x.dtype == torch.bfloat16 and self.weight.dtype == torch.bfloat16 and torch.is_grad_enabled():
            relu = self.fuse_relu and self.bias is not None and knobs.enabled("fused_relu")
            y = _SplitKLinear.apply(x, self.weight, self.bias, relu)
            return torch.relu(y) if self.fuse_relu and not relu else y
        y = super().forward(x)
        return torch.relu(y) if self.fuse_relu else y


# ------------------------------------------------------------------------------ DLRM interaction
def _interact_ref(x: torch.Tensor, e: torch.Tensor) -> torch.Tensor:
    z = torch.cat([x.unsqueeze(1), e], dim=1)
    n = z.shape[1]
    iu = torch.triu_indices(n, n, offset=1, device=z.device)
    dots = torch.bmm(z, z.transpose(1, 2))
    return torch.cat([x, dots[:, iu[0], iu[1]]], dim=1)


class _Interact(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, e):
        x, e = x.contiguous(), e.contiguous()
        ctx.save_for_backward(x, e)
        return native().dlrm_interact_fwd(x, e)

    @staticmethod
    def backward(ctx, dout):
        x, e = ctx.saved_tensors
        dx, de = native().dlrm_interact_bwd(x, e, dout.contiguous().to(torch.bfloat16))
        return dx, de


def dlrm_interact(x: torch.Tensor, e: torch.Tensor) -> torch.Tensor:
    """[x | triu_{i<j}(z_i . z_j)] with z = [x; e] (DLRM dot interaction, torch.triu_indices order).
    x [B, D], e [B, T, D]; bf16 GPU tensors with T + 1 <= 32 and D % 32 == 0 run the MFMA kernel
    (csrc/kernels/dense.hip), anything else the torch composition."""
    if (x.is_cuda and x.dtype == torch.bfloat16 and e.dtype == torch.bfloat16 and e.shape[1] + 1 <= 32
            and x.shape[1] % 32 == 0 and x.shape[1] <= 224):
        return _Interact.apply(x, e)
    return _interact_ref(x, e)
