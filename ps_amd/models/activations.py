"""Activations with the reference's semantics (activations/*.java).

Layout note: the reference is column-major features x batch; ps_amd is batch-major
[batch, features] (PyTorch idiom), so "per column" in the reference is "per row" here.

  Relu          max(0, x); backward masks by y > 0                 Relu.java:7-19
  LeakyRelu     slope 0.01                                          LeakyRelu.java:7-19
  Sigmoid       y = 0.001 + 0.998*sigmoid(x); backward dy*y*(1-y)   Sigmoid.java:9-21
                (so with BCE the logit gradient is exactly p - y)
  Softmax       softmax(x / T), T = 10000 by default, then 0 -> 0.001 and 1 -> 0.999
                (Softmax.java:11-40).  ``reference_backward=True`` reproduces the reference
                Jacobian that ignores the 1/T factor (Q15); False gives the exact gradient.

All are differentiable torch Functions; on a GPU the forward of Softmax runs the
``softmax_temp_fwd`` HIP kernel.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops import nn_ops


class Activation(nn.Module):
    name = "identity"

    def forward(self, x):  # pragma: no cover - overridden
        return x


class Relu(Activation):
    name = "relu"

    def forward(self, x):
        return torch.relu(x)


class LeakyRelu(Activation):
    name = "leaky_relu"

    def __init__(self, slope: float = 0.01):
        super().__init__()
        self.slope = slope

    def forward(self, x):
        return torch.nn.functional.leaky_relu(x, self.slope)


class _ClippedSigmoid(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = 0.001 + 0.998 * torch.sigmoid(x)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return dy * y * (1 - y)


class Sigmoid(Activation):
    name = "sigmoid"

    def forward(self, x):
        return _ClippedSigmoid.apply(x)


class _TempSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, temp, ref_bwd):
        p = nn_ops.softmax_temp(x, temp)
        ctx.save_for_backward(p)
        ctx.temp, ctx.ref_bwd = temp, ref_bwd
        return p.to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        (p,) = ctx.saved_tensors
        g = nn_ops.softmax_temp_bwd(p, dy, 1.0 if ctx.ref_bwd else 1.0 / ctx.temp)  # HIP on GPU
        return g.to(dy.dtype), None, None


class Softmax(Activation):
    name = "softmax"

    def __init__(self, temp: float = 10000.0, reference_backward: bool = True):
        super().__init__()
        self.temp = float(temp)
        self.reference_backward = reference_backward

    def forward(self, x):
        return _TempSoftmax.apply(x, self.temp, self.reference_backward)


def get(name: str | None) -> Activation | None:
    if name is None or name == "none":
        return None
    return {"relu": Relu, "leaky_relu": LeakyRelu, "sigmoid": Sigmoid, "softmax": Softmax}[name]()
