"""Reference-parity layers (layer/*.java) as torch modules, batch-major.

Parameter names reproduce the reference PS keys: a module registered as ``fc0`` owns
``fc0.weights`` [out, in] and ``fc0.bias`` [out]; embedding fields are sparse tables named
``emF<i>`` (rows are keyed ``emF<i>.<id>`` in the reference); the wide part is the sparse
table ``wide.weights`` plus the dense key ``wide.bias``.

Dense layers are ordinary autograd modules -- their gradients flow into the co-located
PS buckets (parallel/colocated.py).  Sparse layers pull the rows touched by the batch from
their table, expose them as a leaf tensor that autograd accumulates into, and push
(unique ids, row gradients) back after backward (``push_sparse``).

Reference semantics kept behind switches:
  * EmbeddingField gradient = mean over a key's occurrences of the per-sample delta
    (EmbeddingField.java:86-104) -> ``grad_mode="reference"``; default ``"exact"`` is the
    true gradient of the mean loss.  (Q7's double backward is NOT reproduced.)
  * LRLayer: every touched wide id receives the batch-mean delta regardless of how often
    it occurs (Q14) -> ``grad_mode="reference"``; default exact per-occurrence gradient.
  * Pooling backward accumulates (Q9 fixed), padded positions never win the max.
  * Dropout keeps with probability 1-p and scales by 1/(1-p) (Q10 fixed).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import dense as _dense
from ..ops import nn_ops
from ..utils.matrix import xavier_bound
from . import activations as A


def _uniform_(t: torch.Tensor, bound: float, gen: Optional[torch.Generator] = None):
    with torch.no_grad():
        t.copy_((torch.rand(t.shape, generator=gen) * 2 - 1) * bound)
    return t


_FUSED_ACT = {A.Relu: 1, A.LeakyRelu: 2, A.Sigmoid: 3}


class InputLayer(nn.Module):
    """Holds the input batch (layer/InputLayer.java)."""

    def __init__(self, name: str, dims: int = 0):
        super().__init__()
        self.lname = name
        self.dims = dims

    def forward(self, x):
        return x


class FcLayer(nn.Module):
    """Z = A W^T + b, A = act(Z) (layer/FcLayer.java:74-91).  Init U(+-4*sqrt(6/(in+out))),
    bias U(+-4*sqrt(6/(in+1))) (:36-49)."""

    def __init__(self, name: str, input_dims: int, output_dims: int, activation: Optional[A.Activation] = None,
                 gen: Optional[torch.Generator] = None):
        super().__init__()
        self.lname = name
        self.input_dims, self.output_dims = input_dims, output_dims
        self.weights = nn.Parameter(_uniform_(torch.empty(output_dims, input_dims),
                                              xavier_bound(input_dims, output_dims), gen))
        self.bias = nn.Parameter(_uniform_(torch.empty(output_dims), xavier_bound(input_dims, 1), gen))
        self.activation = activation

    def set_activation(self, act):
        self.activation = act
        return self

    def forward(self, x):
        if x.is_cuda and self.weights.dtype == torch.bfloat16:
            # MFMA GEMM with bias + activation fused in the epilogue (ops/dense.py)
            code = _FUSED_ACT.get(type(self.activation), None) if self.activation is not None else 0
            if code is not None:
                return _dense.linear_act(x, self.weights, self.bias, code)
            return self.activation(_dense.linear_act(x, self.weights, self.bias, 0))
        z = F.linear(x.to(self.weights.dtype), self.weights, self.bias)
        return self.activation(z) if self.activation is not None else z

    @staticmethod
    def build(input_size: int, dims: Sequence[int], gen=None) -> List["FcLayer"]:
        """ReLU hidden layers, Sigmoid last (FcLayer.java:53-70)."""
        out = []
        for i, d in enumerate(dims):
            act = A.Sigmoid() if i == len(dims) - 1 else A.Relu()
            out.append(FcLayer(f"fc{i}", input_size, d, act, gen))
            input_size = d
        return out


class SparseLayerMixin:
    """Common pull -> leaf -> push protocol for sparse-table layers."""

    def _pull_leaf(self, table, ids: torch.Tensor):
        uniq, inv, counts = torch.unique(ids.reshape(-1), return_inverse=True, return_counts=True)
        rows = table.pull(uniq)
        leaf = rows.detach().clone().requires_grad_(self.training and torch.is_grad_enabled())
        self._pending.append((table, uniq, leaf, counts, ids.shape[0]))
        return leaf, inv.view(ids.shape)

    def _lookup(self, table, ids: torch.Tensor, out_dtype=None) -> torch.Tensor:
        """rows of ``ids`` ([..., dim], autograd to the pulled leaf).  GPU: one sort for the
        dedupe, HIP gather with the dtype cast fused, segment-sum backward (ops/sparse.py)."""
        if not ids.is_cuda:
            leaf, inv = self._pull_leaf(table, ids)
            out = leaf[inv]
            return out if out_dtype is None else out.to(out_dtype)
        from ..ops.sparse import gather_unique, unique_with_segments

        uniq, inv, counts, perm, seg_off = unique_with_segments(ids)
        rows = table.pull(uniq)
        leaf = rows.detach().clone().requires_grad_(self.training and torch.is_grad_enabled())
        self._pending.append((table, uniq, leaf, counts, ids.shape[0]))
        out = gather_unique(leaf, inv, perm, seg_off, out_dtype)
        return out.view(*ids.shape, leaf.shape[1])

    def push_sparse(self) -> int:
        """Push gradients of the rows touched since the last call; returns rows pushed."""
        n = 0
        for table, uniq, leaf, counts, batch in self._pending:
            if leaf.grad is None:
                continue
            g = self._scale_grad(leaf.grad, counts, batch)
            table.push(uniq, g)
            n += uniq.numel()
        self._pending = []
        return n

    def _scale_grad(self, g, counts, batch):
        return g

    def clear(self):
        self._pending = []


class EmbeddingField(SparseLayerMixin, nn.Module):
    """One categorical field: ids [N] -> act(rows) [N, dim] (layer/EmbeddingField.java:66-78).
    Rows init U(+-4*sqrt(6/(1+dim))) on first touch (:31-38), deterministic per (seed, row)."""

    def __init__(self, name: str, dim: int, table, activation: Optional[A.Activation] = None,
                 grad_mode: str = "exact"):
        super().__init__()
        self.lname, self.dim, self.table = name, dim, table
        self.activation = activation
        self.grad_mode = grad_mode
        self._pending = []

    def forward(self, ids):
        leaf, inv = self._pull_leaf(self.table, ids)
        out = leaf[inv]
        return self.activation(out) if self.activation is not None else out

    def _scale_grad(self, g, counts, batch):
        if self.grad_mode == "reference":
            # reference: per-key mean over occurrences of the per-sample delta (no 1/N)
            return g * (batch / counts.to(g.dtype)).unsqueeze(1)
        return g


class EmbeddingLayer(SparseLayerMixin, nn.Module):
    """All categorical fields, outputs stacked into one [N, fields*dim] slice
    (layer/EmbeddingLayer.java:25-48, build :50-57: fields ``emF<i>`` with ReLU)."""

    def __init__(self, name: str, fields: int, dim: int, tables: List, activation: str = "relu",
                 grad_mode: str = "exact"):
        super().__init__()
        self.lname, self.fields, self.dim = name, fields, dim
        self.tables = tables
        self.act_name = activation
        self.grad_mode = grad_mode
        self.embedding_fields = nn.ModuleList([EmbeddingField(f"emF{i}", dim, tables[i], A.get(activation),
                                                             grad_mode) for i in range(fields)])
        self._pending = []

    @property
    def output_dims(self):
        return self.fields * self.dim

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        """ids: [N, fields] int64."""
        outs = [f(ids[:, i]) for i, f in enumerate(self.embedding_fields)]
        return torch.cat(outs, dim=1)

    def push_sparse(self) -> int:
        return sum(f.push_sparse() for f in self.embedding_fields)

    def clear(self):
        for f in self.embedding_fields:
            f.clear()


class LRLayer(SparseLayerMixin, nn.Module):
    """Wide logistic part: z = sum_f w[id_f] + b (layer/LRLayer.java:62-98); weights are a
    1-column sparse table created zero-initialised on first touch; bias is dense."""

    def __init__(self, name: str, table, activation: Optional[A.Activation] = None, grad_mode: str = "exact"):
        super().__init__()
        self.lname = name
        self.table = table
        self.bias = nn.Parameter(torch.zeros(1))
        self.activation = activation
        self.grad_mode = grad_mode
        self._pending = []

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        leaf, inv = self._pull_leaf(self.table, ids)
        z = leaf[inv].reshape(ids.shape[0], -1).sum(dim=1, keepdim=True) + self.bias
        self.register_delta_hook(z)
        return self.activation(z) if self.activation is not None else z

    def _scale_grad(self, g, counts, batch):
        if self.grad_mode == "reference":
            # every touched id gets mean(delta) (batch mean); sum over occurrences of
            # delta/N == mean(delta) only if the id occurs in every sample -> rebuild it
            return self._mean_delta.expand_as(g).clone()
        return g

    def register_delta_hook(self, z: torch.Tensor):
        if self.grad_mode == "reference" and z.requires_grad:
            def hook(grad):
                self._mean_delta = grad.sum().reshape(1, 1)  # grad already carries 1/N
                return grad
            z.register_hook(hook)


class AddLayer(nn.Module):
    """act(left + right); delta passes through unchanged (layer/AddLayer.java:33-61)."""

    def __init__(self, name: str, activation: Optional[A.Activation] = None):
        super().__init__()
        self.lname, self.activation = name, activation

    def forward(self, left, right):
        z = left + right
        return self.activation(z) if self.activation is not None else z


class ConcatLayer(nn.Module):
    """Feature-wise concat (layer/ConcatLayer.java:30-37; its double embedding backward,
    Q7, is not reproduced)."""

    def __init__(self, name: str):
        super().__init__()
        self.lname = name

    def forward(self, *xs):
        return torch.cat([x.to(xs[0].dtype) for x in xs], dim=1)


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed, offset):
        ctx.p, ctx.seed, ctx.offset = p, seed, offset
        return nn_ops.dropout(x, p, seed, offset)

    @staticmethod
    def backward(ctx, dy):
        return nn_ops.dropout(dy, ctx.p, ctx.seed, ctx.offset), None, None, None


class DropoutLayer(nn.Module):
    """Philox dropout: the mask is regenerated from (seed, offset) in backward, never stored
    (layer/DropoutLayer.java:23-53).  Keep prob 1-p, scale 1/(1-p) when ``scale``."""

    def __init__(self, name: str, p: float = 0.5, scale: bool = True, seed: int = 0):
        super().__init__()
        self.lname, self.p, self.scale, self.seed = name, float(p), scale, int(seed)
        self._offset = 0

    def forward(self, x):
        if not self.training or self.p == 0.0:
            return x
        self._offset += (x.numel() + 3) // 4
        y = _Dropout.apply(x, self.p, self.seed, self._offset)
        if not self.scale:
            y = y * (1 - self.p)
        return y


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, arg = nn_ops.maxpool2d_fwd(x.contiguous(), k, s, p)
        ctx.save_for_backward(arg)
        ctx.shape, ctx.k, ctx.s, ctx.p = x.shape, k, s, p
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        return nn_ops.maxpool2d_bwd(dy.contiguous(), arg, ctx.shape, ctx.k, ctx.s, ctx.p), None, None, None


class PoolingLayer(nn.Module):
    """Max pooling with stored argmax (layer/PoolingLayer.java:62-134), NCHW."""

    def __init__(self, name: str, input_w: int, input_h: int, input_d: int, kernel_size: int, stride: int,
                 padding: int = 0):
        super().__init__()
        self.lname = name
        self.input_w, self.input_h, self.input_d = input_w, input_h, input_d
        self.kernel_size, self.stride, self.padding = kernel_size, stride, padding

    @property
    def output_w(self):
        return (self.input_w - self.kernel_size + 2 * self.padding) // self.stride + 1

    @property
    def output_h(self):
        return (self.input_h - self.kernel_size + 2 * self.padding) // self.stride + 1

    @property
    def k(self):
        return self.input_d

    @property
    def output_dims(self):
        return self.output_w * self.output_h * self.input_d

    def forward(self, x):
        return _MaxPool.apply(x, self.kernel_size, self.stride, self.padding)


class _Im2colConv(torch.autograd.Function):
    """Conv as im2col + GEMM (layer/Conv2DLayer.java:146-240) with the HIP im2col/col2im."""

    @staticmethod
    def forward(ctx, x, w, b, k, s, p):
        n, c, h, wd = x.shape
        oh, ow = (h + 2 * p - k) // s + 1, (wd + 2 * p - k) // s + 1
        col = nn_ops.im2col(x.float(), k, s, p)  # [N*OH*OW, C*k*k]
        z = col @ w.float().t() + b.float()  # [N*OH*OW, K]
        ctx.save_for_backward(col, w)
        ctx.meta = (x.shape, k, s, p, oh, ow)
        return z.view(n, oh, ow, -1).permute(0, 3, 1, 2).contiguous().to(x.dtype)

    @staticmethod
    def backward(ctx, dz):
        col, w = ctx.saved_tensors
        xshape, k, s, p, oh, ow = ctx.meta
        n = xshape[0]
        dz2 = dz.float().permute(0, 2, 3, 1).reshape(n * oh * ow, -1)
        dw = dz2.t() @ col
        db = dz2.sum(0)
        dcol = dz2 @ w.float()
        dx = nn_ops.col2im(dcol, xshape, k, s, p)
        return dx, dw.to(w.dtype), db, None, None, None


class Conv2DLayer(nn.Module):
    """Square-kernel conv + bias + activation (layer/Conv2DLayer.java).  Weights [K, C, k, k]
    init U(+-4*sqrt(6/(K + C*k*k))), bias U[0,1) (:64-76).  ``impl="miopen"`` (default on
    GPU) runs MIOpen; ``impl="im2col"`` reproduces the reference algorithm on the HIP
    im2col/col2im kernels (Q8's misaligned ReLU mask is not reproduced)."""

    def __init__(self, name: str, input_w: int, input_h: int, input_d: int, kernel_size: int, stride: int,
                 output_num: int, padding: int = 0, activation: Optional[A.Activation] = None, impl: str = "auto",
                 gen=None):
        super().__init__()
        if min(input_w, input_h, input_d) < 0:
            raise ValueError("negative input dims")
        self.lname = name
        self.input_w, self.input_h, self.input_d = input_w, input_h, input_d
        self.kernel_size, self.stride, self.padding, self.K = kernel_size, stride, padding, output_num
        fan = input_d * kernel_size * kernel_size
        self.weights = nn.Parameter(_uniform_(torch.empty(output_num, input_d, kernel_size, kernel_size),
                                              xavier_bound(output_num, fan), gen))
        with torch.no_grad():
            self.bias = nn.Parameter(torch.rand(output_num, generator=gen))
        self.activation = activation
        self.impl = impl

    def set_activation(self, act):
        self.activation = act
        return self

    @property
    def output_w(self):
        return (self.input_w - self.kernel_size + 2 * self.padding) // self.stride + 1

    @property
    def output_h(self):
        return (self.input_h - self.kernel_size + 2 * self.padding) // self.stride + 1

    @property
    def k(self):
        return self.K

    @property
    def output_dims(self):
        return self.output_w * self.output_h * self.K

    def forward(self, x):
        x = x.view(x.shape[0], self.input_d, self.input_h, self.input_w)
        if self.impl == "im2col" or (self.impl == "auto" and not x.is_cuda):
            w2 = self.weights.view(self.K, -1)
            z = _Im2colConv.apply(x, w2, self.bias, self.kernel_size, self.stride, self.padding)
        else:
            z = F.conv2d(x.to(self.weights.dtype), self.weights, self.bias, self.stride, self.padding)
        return self.activation(z) if self.activation is not None else z
