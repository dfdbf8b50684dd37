"""Reference-model ops: temperature softmax, losses, max-pool with argmax, im2col/col2im,
philox dropout, uniform init.  HIP on GPU; torch on CPU."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._ext import native, use_native


def softmax_temp_bwd(p: torch.Tensor, dy: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    """scale * p * (dy - sum(dy * p)) per row (activations/Softmax.java:45-67; scale 1 = the
    reference, which drops the 1/T, Q15)."""
    p, dy = p.contiguous().float(), dy.contiguous().float()
    if use_native(p):
        dx = torch.empty_like(p)
        native().softmax_temp_bwd(p, dy, dx, float(scale))
        return dx
    return scale * p * (dy - (dy * p).sum(dim=1, keepdim=True))


def softmax_temp(x: torch.Tensor, temp: float = 10000.0, clamp_lo: float = 0.001, clamp_hi: float = 0.999):
    """Row softmax of x/temp with the reference's 0->0.001 / 1->0.999 clamps
    (activations/Softmax.java:11-40)."""
    x = x.contiguous().float()
    y = torch.empty_like(x)
    if use_native(x):
        native().softmax_temp_fwd(x, y, float(temp), float(clamp_lo), float(clamp_hi))
        return y
    p = torch.softmax(x / temp, dim=1)
    if clamp_lo > 0:
        p = torch.where(p <= 0, torch.full_like(p, clamp_lo), p)
    if clamp_hi < 1:
        p = torch.where(p >= 1, torch.full_like(p, clamp_hi), p)
    return p


def softmax_xent(p: torch.Tensor, labels: torch.Tensor, want_grad: bool = True):
    """(-mean log p[label], dL/dp) for SoftmaxLoss (loss/SoftmaxLoss.java:9-28)."""
    p = p.contiguous().float()
    loss = torch.zeros(1, dtype=torch.float32, device=p.device)
    grad = torch.empty_like(p) if want_grad else None
    if use_native(p):
        native().softmax_xent(p, labels.contiguous(), loss, grad)
        return loss, grad
    b = p.shape[0]
    hot = p.gather(1, labels.view(-1, 1)).view(-1)
    loss.copy_(-(hot.log()).mean().reshape(1))
    if grad is not None:
        grad.zero_()
        grad.scatter_(1, labels.view(-1, 1), (-1.0 / hot / b).view(-1, 1))
    return loss, grad


def bce(p: torch.Tensor, y: torch.Tensor, want_grad: bool = True):
    """(mean BCE, dL/dp) (loss/CrossEntropy.java:10-28)."""
    p = p.contiguous().float()
    y = y.contiguous().float()
    loss = torch.zeros(1, dtype=torch.float32, device=p.device)
    grad = torch.empty_like(p) if want_grad else None
    if use_native(p):
        native().bce(p, y, loss, grad)
        return loss, grad
    loss.copy_((-(y * p.log() + (1 - y) * (1 - p).log())).mean().reshape(1))
    if grad is not None:
        grad.copy_((p - y) / (p * (1 - p)) / p.numel())
    return loss, grad


def maxpool2d_fwd(x: torch.Tensor, k: int, stride: int, pad: int = 0):
    n, c, h, w = x.shape
    oh, ow = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
    y = torch.empty(n, c, oh, ow, dtype=x.dtype, device=x.device)
    arg = torch.empty(n, c, oh, ow, dtype=torch.int32, device=x.device)
    if use_native(x):
        native().maxpool2d_fwd(x.contiguous(), k, stride, pad, y, arg)
        return y, arg
    yy, idx = F.max_pool2d(x.float(), k, stride, pad, return_indices=True)
    y.copy_(yy.to(x.dtype))
    arg.copy_(idx.to(torch.int32))
    return y, arg


def maxpool2d_bwd(dy: torch.Tensor, arg: torch.Tensor, x_shape, k: int, stride: int, pad: int = 0):
    dx = torch.empty(x_shape, dtype=dy.dtype, device=dy.device)
    if use_native(dy):
        native().maxpool2d_bwd(dy.contiguous(), arg.contiguous(), k, stride, pad, dx)
        return dx
    n, c, h, w = x_shape
    flat = torch.zeros(n * c, h * w, dtype=torch.float32)
    flat.scatter_add_(1, arg.reshape(n * c, -1).long(), dy.reshape(n * c, -1).float())
    dx.copy_(flat.reshape(x_shape).to(dy.dtype))
    return dx


def im2col(x: torch.Tensor, k: int, stride: int, pad: int):
    """[N,C,H,W] -> [N*OH*OW, C*k*k] patches (layer/Conv2DLayer.java:94-127, row-major)."""
    n, c, h, w = x.shape
    oh, ow = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
    col = torch.empty(n * oh * ow, c * k * k, dtype=torch.float32, device=x.device)
    if use_native(x):
        native().im2col(x.contiguous().float(), k, stride, pad, col)
        return col
    u = F.unfold(x.float(), k, padding=pad, stride=stride)  # [N, C*k*k, L]
    col.copy_(u.transpose(1, 2).reshape(n * oh * ow, c * k * k))
    return col


def col2im(col: torch.Tensor, x_shape, k: int, stride: int, pad: int):
    n, c, h, w = x_shape
    oh, ow = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
    x = torch.empty(x_shape, dtype=torch.float32, device=col.device)
    if use_native(col):
        native().col2im(col.contiguous().float(), k, stride, pad, x)
        return x
    u = col.reshape(n, oh * ow, c * k * k).transpose(1, 2)
    x.copy_(F.fold(u, (h, w), k, padding=pad, stride=stride))
    return x


def dropout(x: torch.Tensor, p: float, seed: int, offset: int = 0) -> torch.Tensor:
    """Philox dropout (keep prob 1-p, scale 1/(1-p)); backward = same call on dy."""
    x = x.contiguous()
    y = torch.empty_like(x)
    if use_native(x):
        native().dropout(x, y, float(p), int(seed), int(offset))
        return y
    g = torch.Generator().manual_seed(int(seed) ^ (int(offset) << 16))
    keep = torch.rand(x.shape, generator=g) >= p
    y.copy_(torch.where(keep, x.float() / (1 - p), torch.zeros((), dtype=torch.float32)).to(x.dtype))
    return y


def uniform_init_(w: torch.Tensor, seed: int, lo: float, hi: float, offset: int = 0) -> torch.Tensor:
    if use_native(w):
        native().uniform_init(w, int(seed), int(offset), float(lo), float(hi))
        return w
    g = torch.Generator().manual_seed(int(seed) * 7919 + int(offset))
    w.copy_(lo + (hi - lo) * torch.rand(w.shape, generator=g))
    return w
