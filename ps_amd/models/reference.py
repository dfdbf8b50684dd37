"""The reference's four models (model/*.java) on ps_amd layers.

  DNN.build_model(fields, dim, numeric, fc_dims)                  model/DNN.java:92-128
      E ids -> Embedding(ReLU) || X -> Concat -> FC...(ReLU) -> Sigmoid ; BCE ; Adam default
  WideDeepNN.build_model(fields, dim, numeric, fc_dims, wide)     model/WideDeepNN.java:105-161
      deep part (last FC linear) + LR wide part over W ids -> Add -> Sigmoid ;
      FTRL for wide.weights / wide.bias, Adam default
  FullConnectedNN.build_model(numeric, fc_dims)                   model/FullConnectedNN.java:86-110
      MLP, Softmax(T=10000) last, SoftmaxLoss ; Adam default
  CNN.build_model(w, h, d, fc_dims)                               model/CNN.java:28-71
      conv3x3(16,p1)+ReLU -> maxpool2 -> conv3x3(32,p1)+ReLU -> maxpool2 -> FC... softmax

Interface (model/Model.java:11-17): ``train(batch) -> loss`` (forward + backward + train
metrics, no optimizer step -- the PS applies it), ``predict(batch)``, ``pull_weights()``,
``get_updater()`` (key-prefix -> Updater).  Batches are dicts with the reference's keys:
``X`` numeric [N, numeric], ``E`` categorical ids [N, fields], ``W`` wide ids [N, k],
``Y`` labels.  Sparse tables come from ``table_factory(name, dim, rows, init, mode, fields)``
so the same model runs standalone (``local_table_factory``: SparseTable), on the co-located
PS ranks (``sharded_table_factory``: rows partitioned over the torchrun/RCCL ranks) or on
dedicated TCP servers (``tcp_table_factory``: rows in the native server's row tables).
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.nn as nn

from ..context import ctx
from ..eval.metrics import AUC, SoftmaxPrecision
from ..obs import metrics as _metrics
from ..parallel.sparse_table import ShardedSparseTable, SparseTable, TcpSparseTable, stable_seed
from ..parallel.updaters import AdamUpdater, FtrlUpdater, Updater
from . import activations as A
from . import layers as L
from .losses import CrossEntropy, Loss, SoftmaxLoss


def local_table_factory(device=None, seed: int = 0, id_mode: str = "map"):
    """Standalone tables (one process holds every row)."""
    def make(name, dim, rows, init, mode=None, fields=1):
        return SparseTable(name, dim, rows, init=init, id_mode=mode or id_mode, seed=stable_seed(name, seed),
                           device=device, fields=fields)

    return make


def sharded_table_factory(transport, device=None, seed: int = 0, id_mode: str = "map", overlap: bool = True,
                          exchange=None):
    """Rows partitioned over the co-located servers of ``transport`` (torchrun ranks); with
    ``overlap`` (GPU) row gradients are pushed from backward hooks on a side stream.
    ``exchange``: "plane" | "collective" | None (auto, see row_plane.plane_rows_wanted)."""
    def make(name, dim, rows, init, mode=None, fields=1):
        return ShardedSparseTable(name, dim, rows, transport, init=init, id_mode=mode or id_mode,
                                  seed=stable_seed(name, seed), device=device, fields=fields, overlap=overlap,
                                  exchange=exchange)

    return make


def tcp_table_factory(client, device=None, seed: int = 0, id_mode: str = "map"):
    """Rows on the dedicated TCP parameter servers (-Dmode=dist)."""
    def make(name, dim, rows, init, mode=None, fields=1):
        return TcpSparseTable(name, dim, rows, client, init=init, id_mode=mode or id_mode,
                              seed=stable_seed(name, seed), fields=fields, device=device)

    return make


class Model(nn.Module):
    loss: Loss

    def __init__(self):
        super().__init__()
        self.updater: Dict[str, Updater] = {}

    # -- reference interface ------------------------------------------------------------
    def get_updater(self) -> Dict[str, Updater]:
        return self.updater

    def pull_weights(self) -> None:
        """Weights are PS-owned replica views (bound by the engine); clear sparse caches."""
        for layer in self.sparse_layers():
            layer.clear()

    def predict(self, batch: Dict[str, torch.Tensor]) -> torch.Tensor:
        was = self.training
        self.eval()
        with torch.no_grad():
            out = self.forward(batch)
        self.train(was)
        return out

    def train_batch(self, batch: Dict[str, torch.Tensor], scale: float = 1.0) -> float:
        """forward + loss + backward (reference ``Model.train``); returns the loss value."""
        self.train(True)
        p = self.forward(batch)
        loss = self.loss(p, batch["Y"])
        lv = float(loss.detach())
        if ctx.step % max(1, ctx.cfg.n_term_dump) == 0:
            self.log_train_metric(p.detach(), batch["Y"])
        if lv <= CrossEntropy.slim or math.isnan(lv):
            ctx.finish = True
            if math.isnan(lv):
                return lv
        (loss * scale).backward()
        return lv

    def log_train_metric(self, p, y):
        pass

    def _set_fc(self, fcs):
        """Register FC layers as fc0, fc1, ... so parameter keys are ``fc0.weights``."""
        self._fc_names = []
        for i, f in enumerate(fcs):
            self.add_module(f"fc{i}", f)
            self._fc_names.append(f"fc{i}")

    @property
    def fc(self):
        return [getattr(self, n) for n in self._fc_names]

    # -- sparse plumbing ----------------------------------------------------------------
    def sparse_layers(self) -> List[L.SparseLayerMixin]:
        return [m for m in self.modules() if isinstance(m, (L.EmbeddingLayer, L.LRLayer))]

    def tables(self):
        """Sparse tables by PS key prefix: ``emF`` (all embedding fields; per-field tables are
        ``emF<i>``) and ``wide.weights``."""
        out = {}
        for m in self.modules():
            if isinstance(m, L.EmbeddingLayer):
                if m.per_field:
                    for i, t in enumerate(m.tables):
                        out[f"emF{i}"] = t
                else:
                    out["emF"] = m.table
            elif isinstance(m, L.LRLayer):
                out[f"{m.lname}.weights"] = m.table
        return out

    def set_accumulating(self, on: bool) -> None:
        """Micro-batch accumulation: owners keep pushed rows and step once per round."""
        for t in self.tables().values():
            t.accumulating = on

    def push_sparse(self) -> int:
        return sum(layer.push_sparse() for layer in self.sparse_layers())


def _scale_init(model: Model, scale: float) -> None:
    """``init_scale`` != 1 shrinks the reference's 4*xavier uniform init (FcLayer.java:39)
    -- at scale 1 a small synthetic problem needs the reference's 100 epochs to recover
    from saturated sigmoids / dead ReLUs."""
    if scale == 1.0:
        return
    with torch.no_grad():
        for p in model.parameters():
            p.mul_(scale)
    for t in model.tables().values():
        t.init = (t.init[0] * scale, t.init[1] * scale)


def _bind_table_updaters(model: Model):
    from ..parallel.updaters import resolve_updater

    for name, t in model.tables().items():
        t.set_updater(resolve_updater(name, model.updater))


class DNN(Model):
    def __init__(self, fields, dim, numeric, fc_dims, table_factory=None, gen=None, grad_mode="exact",
                 emb_rows: int = 100000, init_scale: float = 1.0):
        super().__init__()
        tf = table_factory or local_table_factory()
        bound = 4 * math.sqrt(6) / math.sqrt(1 + dim)
        self.embedding = L.EmbeddingLayer("embedding", fields, dim,
                                          tf("emF", dim, emb_rows, (-bound, bound), None, fields), "relu", grad_mode)
        self.concat = L.ConcatLayer("concat")
        self._set_fc(L.FcLayer.build(fields * dim + numeric, fc_dims, gen))  # keys fc0.weights, ...
        self.loss = CrossEntropy()
        self.updater["default"] = AdamUpdater(0.005, 0.9, 0.999, 1e-8, bias_correction="reference")
        _bind_table_updaters(self)
        _scale_init(self, init_scale)

    def forward(self, batch):
        e = self.embedding(batch["E"])
        x = self.concat(e, batch["X"].to(e.dtype))
        for f in self.fc:
            x = f(x)
        return x.reshape(-1)

    def log_train_metric(self, p, y):
        a = AUC(p.float().cpu().numpy(), y.float().cpu().numpy()).calculate()
        _metrics.plot("Train_AUC", a, ctx.step)

    @staticmethod
    def build_model(embedding_field_num: int, embedding_size: int, number_field_num: int,
                    fc_layer_dims: Sequence[int], **kw) -> "DNN":
        return DNN(embedding_field_num, embedding_size, number_field_num, fc_layer_dims, **kw)


class WideDeepNN(Model):
    def __init__(self, fields, dim, numeric, fc_dims, wide_size, table_factory=None, gen=None, grad_mode="exact",
                 emb_rows: int = 100000, init_scale: float = 1.0):
        super().__init__()
        tf = table_factory or local_table_factory()
        bound = 4 * math.sqrt(6) / math.sqrt(1 + dim)
        self.embedding = L.EmbeddingLayer("embedding", fields, dim,
                                          tf("emF", dim, emb_rows, (-bound, bound), None, fields), "relu", grad_mode)
        self.concat = L.ConcatLayer("concat")
        fcs = L.FcLayer.build(fields * dim + numeric, fc_dims, gen)
        fcs[-1].set_activation(None)
        self._set_fc(fcs)
        self.wide = L.LRLayer("wide", tf("wide.weights", 1, wide_size, (0.0, 0.0), "hash"), None, grad_mode)
        self.add = L.AddLayer("addWideDeep", A.Sigmoid())
        self.loss = CrossEntropy()
        ftrl = FtrlUpdater(0.005, 1.0, 0.001, 0.001, mode="reference" if grad_mode == "reference" else "canonical")
        self.updater["wide.weights"] = ftrl
        self.updater["wide.bias"] = ftrl
        self.updater["default"] = AdamUpdater(0.005, 0.9, 0.999, 1e-8, bias_correction="reference")
        _bind_table_updaters(self)
        _scale_init(self, init_scale)

    def forward(self, batch):
        e = self.embedding(batch["E"])
        x = self.concat(e, batch["X"].to(e.dtype))
        for f in self.fc:
            x = f(x)
        w = self.wide(batch["W"])
        return self.add(x, w.to(x.dtype)).reshape(-1)

    def log_train_metric(self, p, y):
        a = AUC(p.float().cpu().numpy(), y.float().cpu().numpy()).calculate()
        _metrics.plot("Train_AUC", a, ctx.step)

    @staticmethod
    def build_model(embedding_field_num, embedding_size, number_field_num, fc_layer_dims, wide_size, **kw):
        return WideDeepNN(embedding_field_num, embedding_size, number_field_num, fc_layer_dims, wide_size, **kw)


class FullConnectedNN(Model):
    def __init__(self, numeric, fc_dims, gen=None, softmax_temp: float = 10000.0, reference_backward: bool = True):
        super().__init__()
        fcs = L.FcLayer.build(numeric, fc_dims, gen)
        fcs[-1].set_activation(A.Softmax(softmax_temp, reference_backward))
        self._set_fc(fcs)
        self.loss = SoftmaxLoss()
        self.updater["default"] = AdamUpdater(0.005, 0.9, 0.999, 1e-8, bias_correction="reference")

    def forward(self, batch):
        x = batch["X"]
        for f in self.fc:
            x = f(x)
        return x

    def log_train_metric(self, p, y):
        _metrics.plot("Train_Precision", SoftmaxPrecision(y, p).calculate(), ctx.step)

    @staticmethod
    def build_model(number_field_num: int, fc_layer_dims: Sequence[int], **kw) -> "FullConnectedNN":
        return FullConnectedNN(number_field_num, fc_layer_dims, **kw)


class CNN(FullConnectedNN):
    def __init__(self, w, h, d, fc_dims, gen=None, conv_impl="auto", **kw):
        Model.__init__(self)
        self.conv1 = L.Conv2DLayer("conv1", w, h, d, 3, 1, 16, 1, A.Relu(), conv_impl, gen)
        self.pool1 = L.PoolingLayer("pool1", self.conv1.output_w, self.conv1.output_h, self.conv1.k, 2, 2)
        self.conv2 = L.Conv2DLayer("conv2", self.pool1.output_w, self.pool1.output_h, self.pool1.k, 3, 1, 32, 1,
                                   A.Relu(), conv_impl, gen)
        self.pool2 = L.PoolingLayer("pool2", self.conv2.output_w, self.conv2.output_h, self.conv2.k, 2, 2)
        fcs = L.FcLayer.build(self.pool2.output_dims, fc_dims, gen)
        fcs[-1].set_activation(A.Softmax(kw.get("softmax_temp", 10000.0), kw.get("reference_backward", True)))
        self._set_fc(fcs)
        self.loss = SoftmaxLoss()
        self.updater["default"] = AdamUpdater(0.005, 0.9, 0.999, 1e-8, bias_correction="reference")
        self.in_shape = (d, h, w)

    def forward(self, batch):
        x = batch["X"].reshape(-1, *self.in_shape)
        x = self.pool1(self.conv1(x))
        x = self.pool2(self.conv2(x))
        x = x.reshape(x.shape[0], -1)
        for f in self.fc:
            x = f(x)
        return x

    @staticmethod
    def build_model(w: int, h: int, d: int, fc_layer_dims: Sequence[int], **kw) -> "CNN":
        return CNN(w, h, d, fc_layer_dims, **kw)
