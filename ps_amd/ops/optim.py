"""Fused optimizer ops (HIP on GPU, torch reference on CPU).

Kinds mirror csrc/kernels/optim.hip: 0 sgd(+momentum/nesterov/wd), 1 adam(w), 2 adagrad,
3 ftrl.  The CPU path is the numerical oracle the GPU tests compare against.
"""
from __future__ import annotations

from typing import Optional

import torch

from ._ext import native, use_native

SGD, ADAM, ADAGRAD, FTRL = 0, 1, 2, 3


def _hp(kw):
    d = dict(lr=0.01, beta1=0.9, beta2=0.999, eps=1e-8, wd=0.0, momentum=0.0, dampening=0.0, nesterov=False,
             adamw=False, bc1=1.0, bc2=1.0, l1=0.0, l2=0.0, fbeta=1.0, ftrl_mode=0, gscale=1.0)
    unknown = set(kw) - set(d)
    if unknown:
        raise TypeError(f"unknown optimizer hyper-parameters {sorted(unknown)}")
    d.update(kw)
    return d


def _apply_ref(kind, w, s0, s1, g, h):
    """Vectorized torch version of opt_apply<KIND> (fp32)."""
    if kind == SGD:
        if h["wd"]:
            g = g + h["wd"] * w
        if h["momentum"]:
            s0.mul_(h["momentum"]).add_(g, alpha=1.0 - h["dampening"])
            g = g + h["momentum"] * s0 if h["nesterov"] else s0.clone()
        w.sub_(h["lr"] * g)
    elif kind == ADAM:
        if h["wd"] and not h["adamw"]:
            g = g + h["wd"] * w
        s0.mul_(h["beta1"]).add_(g, alpha=1.0 - h["beta1"])
        s1.mul_(h["beta2"]).add_(g * g, alpha=1.0 - h["beta2"])
        upd = (s0 * h["bc1"]) / (torch.sqrt(s1 * h["bc2"]) + h["eps"])
        if h["wd"] and h["adamw"]:
            upd = upd + h["wd"] * w
        w.sub_(h["lr"] * upd)
    elif kind == ADAGRAD:
        if h["wd"]:
            g = g + h["wd"] * w
        s0.add_(g * g)
        w.sub_(h["lr"] * g / (torch.sqrt(s0) + h["eps"]))
    elif kind == FTRL:
        z, n = s0, s1
        lr, l1, l2, fb = h["lr"], h["l1"], h["l2"], h["fbeta"]
        if h["ftrl_mode"] == 1:
            sgn = torch.where(z >= 0, 1.0, -1.0)
            wn = -(z - sgn * l1) / ((l2 + (fb + torch.sqrt(n))) / lr)
            wn = torch.where(z.abs() <= l1, torch.zeros_like(wn), wn)
            sigma = torch.sqrt(n + g * g) - torch.sqrt(n / lr)
            z.add_(g - sigma * wn)
            n.add_(g * g)
            w.copy_(wn)
        else:
            nn_ = n + g * g
            sigma = (torch.sqrt(nn_) - torch.sqrt(n)) / lr
            z.add_(g - sigma * w)
            n.copy_(nn_)
            sgn = torch.where(z >= 0, 1.0, -1.0)
            wn = -(z - sgn * l1) / ((fb + torch.sqrt(n)) / lr + l2)
            w.copy_(torch.where(z.abs() <= l1, torch.zeros_like(wn), wn))
    else:
        raise ValueError(kind)


def fused_opt(kind: int, w: torch.Tensor, st0: Optional[torch.Tensor], st1: Optional[torch.Tensor],
              g: torch.Tensor, wout: Optional[torch.Tensor] = None, gscale_t: Optional[torch.Tensor] = None,
              **hp) -> None:
    """In-place optimizer step on a flat fp32 shard ``w`` with gradient ``g`` (bf16/fp32).

    ``wout`` (optional) receives the updated weights (bf16 or fp32) -- the pull buffer.
    ``gscale_t`` (optional, device float[1]) multiplies the gradient (clip factor).
    """
    h = _hp(hp)
    if use_native(w, g):
        native().fused_opt(kind, w, st0, st1, g, wout, h["lr"], h["beta1"], h["beta2"], h["eps"], h["wd"],
                           h["momentum"], h["dampening"], bool(h["nesterov"]), bool(h["adamw"]), h["bc1"],
                           h["bc2"], h["l1"], h["l2"], h["fbeta"], int(h["ftrl_mode"]), h["gscale"], gscale_t)
        return
    gg = g.float().reshape(w.shape) * h["gscale"]
    if gscale_t is not None:
        gg = gg * gscale_t.float()
    s0 = st0 if st0 is not None else torch.zeros_like(w)
    s1 = st1 if st1 is not None else torch.zeros_like(w)
    _apply_ref(kind, w, s0, s1, gg, h)
    if wout is not None:
        wout.copy_(w.reshape(wout.shape))


def sparse_opt(kind: int, table: torch.Tensor, st0: Optional[torch.Tensor], st1: Optional[torch.Tensor],
               rows: torch.Tensor, grad: torch.Tensor, rowwise: bool = False, skip_zero: bool = False,
               perm: Optional[torch.Tensor] = None, ncount: Optional[torch.Tensor] = None, **hp) -> None:
    """Row-sparse optimizer step on ``table[rows]``.

    ``ncount`` (int32 [1], device): only ``rows[:ncount]`` are live -- a touched list whose length
    stays on the device (the row plane's accumulator), so the kernel stops there instead of
    walking the list's full capacity.

    ``perm is None``: ``rows`` unique, ``grad`` [len(rows), dim] row-aligned.
    ``perm`` given: ``rows`` SORTED with repeats, ``grad[perm[j]]`` belongs to ``rows[j]``; the
    gradient rows of every run are summed and ONE update is applied per distinct row (the
    owner-side merge of several workers' / micro-batches' pushes, no host sync).  Negative
    rows are skipped."""
    h = _hp(hp)
    if use_native(table, grad):
        native().sparse_opt(kind, table, st0, st1, rows, grad, bool(rowwise), bool(skip_zero), h["lr"], h["beta1"],
                            h["beta2"], h["eps"], h["wd"], h["momentum"], h["dampening"], bool(h["nesterov"]),
                            bool(h["adamw"]), h["bc1"], h["bc2"], h["l1"], h["l2"], h["fbeta"], int(h["ftrl_mode"]),
                            h["gscale"], perm, ncount)
        return
    if ncount is not None:
        rows = rows[:int(ncount.item())]
        perm = perm[:rows.numel()] if perm is not None else None
    if rows.numel() == 0:
        return
    dim = table.shape[1]
    g = grad.float().reshape(-1, dim)
    if perm is not None:
        g = g[perm]
        head = torch.ones(rows.numel(), dtype=torch.bool)
        head[1:] = rows[1:] != rows[:-1]
        seg = torch.cumsum(head.long(), 0) - 1
        nu = int(seg[-1]) + 1
        acc = torch.zeros(nu, dim, dtype=torch.float32)
        acc.index_add_(0, seg, g)
        rows, g = rows[head], acc
    g = g * h["gscale"]
    keep = rows >= 0
    if skip_zero:
        keep &= g[:, 0] != 0
    rows, g = rows[keep], g[keep]
    if kind == ADAGRAD and rowwise:
        ss = (g * g).mean(dim=1)
        st0[rows] += ss
        denom = torch.sqrt(st0[rows]) + h["eps"]
        table[rows] -= h["lr"] * g / denom[:, None]
        return
    w = table[rows].clone()
    a = st0[rows].clone() if st0 is not None else torch.zeros_like(w)
    b = st1[rows].clone() if st1 is not None else torch.zeros_like(w)
    _apply_ref(kind, w, a, b, g, h)
    table[rows] = w
    if st0 is not None:
        st0[rows] = a
    if st1 is not None:
        st1[rows] = b
