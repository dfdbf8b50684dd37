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
        if x.is_cuda and self.weights.dtype in (torch.bfloat16, torch.float32):
            # MFMA GEMM with bias + activation fused in the epilogue, K2 fused backward
            # (ops/dense.py; fp32 models on v_mfma_f32_16x16x4_f32)
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
    """Common lookup -> (autograd leaf) -> push protocol of sparse-table layers: every table
    looked up in a forward keeps the routing of that pull and pushes the rows' gradients back
    along it (parallel/sparse_table.py); ``push_sparse`` flushes what the backward hooks have
    not already pushed."""

    def _tables_used(self) -> list:
        if not hasattr(self, "_used"):
            self._used = []
        return self._used

    def _lookup(self, table, ids: torch.Tensor, out_dtype=None, grad_fn=None) -> torch.Tensor:
        """rows of ``ids`` ([..., dim]); autograd to the pulled rows of ``table``."""
        used = self._tables_used()
        if not any(t is table for t in used):
            used.append(table)
        return table.lookup(ids, out_dtype, grad_fn)

    def push_sparse(self) -> int:
        """Push gradients of the rows touched since the last call; returns rows pushed."""
        return sum(t.push_pending() for t in self._tables_used())

    def clear(self):
        for t in self._tables_used():
            t.drop_pending()


def _reference_mean_grad(g: torch.Tensor, plan) -> torch.Tensor:
    """EmbeddingField.java:86-104: per key, the MEAN over its occurrences of the per-sample
    delta (no 1/N): exact grad (which carries 1/N) * N / count."""
    return g * (plan.n / plan.counts.to(g.dtype)).unsqueeze(1)


class EmbeddingField(SparseLayerMixin, nn.Module):
    """One categorical field: ids [N] -> act(rows) [N, dim] (layer/EmbeddingField.java:66-78).
    Rows init U(+-4*sqrt(6/(1+dim))) on first touch (:31-38), deterministic per (seed, key)."""

    def __init__(self, name: str, dim: int, table, activation: Optional[A.Activation] = None,
                 grad_mode: str = "exact"):
        super().__init__()
        self.lname, self.dim, self.table = name, dim, table
        self.activation = activation
        self.grad_mode = grad_mode

    def forward(self, ids):
        out = self._lookup(self.table, ids, None, _reference_mean_grad if self.grad_mode == "reference" else None)
        return self.activation(out) if self.activation is not None else out


class EmbeddingLayer(SparseLayerMixin, nn.Module):
    """All categorical fields, outputs stacked into one [N, fields*dim] slice
    (layer/EmbeddingLayer.java:25-48, build :50-57: fields ``emF<i>`` with ReLU).

    The fields share ONE table (``table.fields == fields``; key = (field, id)), so a forward
    pulls every field's rows in one exchange -- the reference issues one getList per field
    (EmbeddingField.preForward, layer/EmbeddingField.java:57-64).  A list of per-field tables
    is accepted too (looked up one by one)."""

    def __init__(self, name: str, fields: int, dim: int, table, activation: str = "relu",
                 grad_mode: str = "exact"):
        super().__init__()
        self.lname, self.fields, self.dim = name, fields, dim
        self.per_field = isinstance(table, (list, tuple))
        self.tables = list(table) if self.per_field else [table]
        if not self.per_field and getattr(table, "fields", 1) != fields:
            raise ValueError(f"table has {table.fields} fields, layer needs {fields}")
        self.act_name = activation
        self.act = A.get(activation)
        self.grad_mode = grad_mode

    @property
    def table(self):
        return self.tables[0]

    @property
    def output_dims(self):
        return self.fields * self.dim

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        """ids: [N, fields] int64."""
        gfn = _reference_mean_grad if self.grad_mode == "reference" else None
        if self.per_field:
            e = torch.stack([self._lookup(t, ids[:, i], None, gfn) for i, t in enumerate(self.tables)], dim=1)
        else:
            e = self._lookup(self.tables[0], ids, None, gfn)  # [N, fields, dim]
        e = e.reshape(ids.shape[0], self.fields * self.dim)
        return self.act(e) if self.act is not None else e


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

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        gfn = self._reference_grad if self.grad_mode == "reference" else None
        w = self._lookup(self.table, ids.reshape(-1), None, gfn)  # [N*k, 1]
        z = w.reshape(ids.shape[0], -1).sum(dim=1, keepdim=True) + self.bias
        self.register_delta_hook(z)
        return self.activation(z) if self.activation is not None else z

    def _reference_grad(self, g, plan):
        # every touched id gets mean(delta) (the batch mean; LRLayer.java:110-117, Q14)
        return self._mean_delta.to(g.dtype).expand_as(g).clone()

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


class _Im2col(torch.autograd.Function):
    """[N, C, H, W] -> [N*OH*OW, C*k*k] patches with the HIP im2col; backward = HIP col2im
    (the gather formulation, K12 / K15)."""

    @staticmethod
    def forward(ctx, x, k, s, p):
        ctx.meta = (x.shape, k, s, p)
        return nn_ops.im2col(x.float(), k, s, p)

    @staticmethod
    def backward(ctx, dcol):
        xshape, k, s, p = ctx.meta
        return nn_ops.col2im(dcol, xshape, k, s, p), None, None, None


def conv_k12(x, w2, b, k: int, s: int, p: int, act: int = 0):
    """The reference conv on the in-house kernels (layer/Conv2DLayer.java:146-240):
    HIP im2col -> the fused MFMA linear (fc.hip: fp32 16x16x4 MFMA, bias + activation in the
    epilogue) -> [N, K, OH, OW]; backward = the fused K2 kernel (act' in the prologue, dW, db
    from the staged tile, dcol) -> HIP col2im."""
    n, _, h, wd = x.shape
    oh, ow = (h + 2 * p - k) // s + 1, (wd + 2 * p - k) // s + 1
    col = _Im2col.apply(x, k, s, p)  # [N*OH*OW, C*k*k]
    y2 = _dense.linear_act(col, w2, b, act)  # [N*OH*OW, K]
    return y2.view(n, oh, ow, -1).permute(0, 3, 1, 2).contiguous()


class Conv2DLayer(nn.Module):
    """Square-kernel conv + bias + activation (layer/Conv2DLayer.java).  Weights [K, C, k, k]
    init U(+-4*sqrt(6/(K + C*k*k))), bias U[0,1) (:64-76).

    ``impl``: ``"auto"`` (default) runs the reference im2col + GEMM algorithm -- on GPU through
    the in-house kernels (HIP im2col, the fp32 MFMA fused linear with the bias + ReLU / leaky /
    clipped-sigmoid epilogue, the fused K2 backward, HIP col2im: ``conv_k12``), on CPU through
    torch matmuls; ``"im2col"`` forces the torch-matmul form; ``"miopen"`` uses F.conv2d.
    Q8's misaligned ReLU mask is not reproduced."""

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
        if self.impl == "auto" and x.is_cuda and self.weights.dtype == torch.float32:
            code = _FUSED_ACT.get(type(self.activation), None) if self.activation is not None else 0
            w2 = self.weights.view(self.K, -1)
            z = conv_k12(x, w2, self.bias, self.kernel_size, self.stride, self.padding, code or 0)
            if code is not None:
                return z
            return self.activation(z)
        if self.impl == "im2col" or (self.impl == "auto" and not x.is_cuda):
            w2 = self.weights.view(self.K, -1)
            z = _Im2colConv.apply(x, w2, self.bias, self.kernel_size, self.stride, self.padding)
        else:
            z = F.conv2d(x.to(self.weights.dtype), self.weights, self.bias, self.stride, self.padding)
        return self.activation(z) if self.activation is not None else z
