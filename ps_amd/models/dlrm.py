"""DLRM-style CTR model for the BASELINE.json sparse config ("sparse push/pull + server-side
Adagrad on 8 x MI355X").

  dense [B, 13] -> bottom MLP 13-512-256-128 (ReLU)
  26 categorical ids -> 26 embedding tables (dim 128), ALL held in ONE row-sharded table
      (per-table row offsets) so a step does one id exchange + one row exchange instead of
      26 -- the reference's one-RPC-per-row push at the other extreme;
      the row-gradient push leaves from a backward hook on a side stream (overlapped)
  interaction: pairwise dots of the 27 vectors (upper triangle, 351) ++ bottom output
  top MLP 479-1024-1024-512-256-1 -> sigmoid, BCE.

Dense MLP weights train on the co-located PS (fused HIP optimizer on fp32 masters); the
embedding rows live on their owner ranks and are updated there by the row-wise Adagrad HIP
kernel (sparse push), never replicated.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..parallel.sparse_table import ShardedSparseTable
from ..parallel.transport import Transport
from ..parallel.updaters import AdagradUpdater, Updater
from ..ops.dense import SplitKLinear, dlrm_interact
from .layers import SparseLayerMixin


def mlp(dims: Sequence[int], last_act: bool = True) -> nn.Sequential:
    layers: List[nn.Module] = []
    for i in range(len(dims) - 1):
        # nn.Linear with split-K weight gradients on GPU bf16 (batch-long reductions into small dW)
        layers.append(SplitKLinear(dims[i], dims[i + 1]))
        if i < len(dims) - 2 or last_act:
            # the ReLU runs inside the linear (bias + ReLU GEMM epilogue); the Identity keeps the
            # Sequential's indices, so state_dict keys are those of Linear / ReLU pairs
            layers[-1].fuse_relu = True
            layers.append(nn.Identity())
    return nn.Sequential(*layers)


class MultiTableEmbedding(SparseLayerMixin, nn.Module):
    """T tables of (rows_t, dim) as the fields of ONE (sharded) sparse table: key = row offset
    of table t + id, range-partitioned over the co-located servers; one id exchange + one row
    exchange per step for all T tables."""

    def __init__(self, rows: Sequence[int], dim: int, transport: Optional[Transport] = None,
                 updater: Optional[Updater] = None, device=None, seed: int = 0, overlap: bool = True):
        super().__init__()
        self.rows = list(rows)
        self.dim = dim
        bound = (1.0 / max(self.rows)) ** 0.5
        upd = updater or AdagradUpdater(0.01, 1e-8, rowwise=True)
        self.table = ShardedSparseTable("emb", dim, self.rows, transport, upd, init=(-bound, bound), seed=seed,
                                        device=device, fields=len(self.rows), overlap=overlap)
        self.out_dtype = None  # compute dtype of the looked-up rows (tables stay fp32)

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        """ids [B, T] (per-table row ids) -> [B, T, dim]."""
        return self._lookup(self.table, ids, self.out_dtype)


class DLRM(nn.Module):
    def __init__(self, dense_in: int = 13, table_rows: Sequence[int] = (100000,) * 26, dim: int = 128,
                 bottom: Sequence[int] = (512, 256), top: Sequence[int] = (1024, 1024, 512, 256),
                 transport: Optional[Transport] = None, device=None, sparse_updater: Optional[Updater] = None,
                 overlap: bool = True):
        super().__init__()
        self.bottom = mlp([dense_in, *bottom, dim])
        self.emb = MultiTableEmbedding(table_rows, dim, transport, sparse_updater, device, overlap=overlap)
        n = len(table_rows) + 1
        self.n_inter = n * (n - 1) // 2
        self.top = mlp([self.n_inter + dim, *top, 1], last_act=False)
        iu = torch.triu_indices(n, n, offset=1)
        self.register_buffer("iu0", iu[0], persistent=False)
        self.register_buffer("iu1", iu[1], persistent=False)

    def forward(self, dense: torch.Tensor, sparse: torch.Tensor) -> torch.Tensor:
        x = self.bottom(dense.to(self.bottom[0].weight.dtype))  # [B, dim]
        self.emb.out_dtype = x.dtype
        e = self.emb(sparse)  # [B, T, dim] in the compute dtype (cast fused into the gather)
        # [x | triu(z z^T)], z = [x; e]: one fused MFMA kernel on GPU bf16 (ops/dense.py)
        return self.top(dlrm_interact(x, e)).squeeze(1)

    def push_sparse(self) -> int:
        return self.emb.push_sparse()

    def prefetch(self, sparse: torch.Tensor) -> None:
        """Route the next batch's ids ahead of time (no host wait on its lookup at W > 1)."""
        self.emb.table.prefetch(sparse)

    def pull_weights(self) -> None:
        self.emb.clear()


def dlrm_batch(batch: int, table_rows: Sequence[int], dense_in: int = 13, seed: int = 0, device=None,
               zipf: float = 1.05):
    """Synthetic Criteo-shaped batch: log-normal dense features, power-law (hot-id) sparse ids."""
    g = torch.Generator().manual_seed(seed)
    dense = torch.log1p(torch.rand(batch, dense_in, generator=g) * 100)
    cols = []
    for r in table_rows:
        u = torch.rand(batch, generator=g)
        ids = (torch.pow(u, zipf * 3) * r).long().clamp_(0, r - 1)  # skewed towards small ids
        cols.append(ids)
    sparse = torch.stack(cols, dim=1)
    y = (torch.rand(batch, generator=g) < 0.25).float()
    if device is not None:
        dense, sparse, y = dense.to(device), sparse.to(device), y.to(device)
    return dense, sparse, y
