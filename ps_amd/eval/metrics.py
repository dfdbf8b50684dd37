"""Evaluation metrics (evaluate/AUC.java, evaluate/SoftmaxPrecision.java).

AUC: the reference sorts by score, walks from the top and sums a ROC staircase; with its
swapped tp/fp names the result is exactly the pairwise AUC with ties broken by input
order (not averaged).  ``AUC.calculate()`` reproduces that; ``auc_exact`` averages ties
(Mann-Whitney).  Both run on numpy (host) or torch (GPU, sort on device).
"""
from __future__ import annotations

import numpy as np
import torch


def _np(x):
    if isinstance(x, torch.Tensor):
        return x.detach().float().cpu().numpy().reshape(-1)
    return np.asarray(x, dtype=np.float64).reshape(-1)


class AUC:
    def __init__(self, p, y):
        self.p = _np(p).astype(np.float64)
        self.y = _np(y).astype(np.float64)
        self.pos_num = float((self.y > 0).sum())
        self.neg_num = float((self.y <= 0).sum())

    def calculate(self) -> float:
        """Reference algorithm (AUC.java:51-82): stable ascending sort, walk from the end."""
        if self.pos_num == 0 or self.neg_num == 0:
            return float("nan")
        order = np.argsort(self.p, kind="stable")[::-1]
        pos = (self.y[order] > 0).astype(np.float64)
        cum_pos = np.cumsum(pos)
        # each negative adds (1/P) * (positives seen so far / N)
        neg_mask = pos == 0
        return float(cum_pos[neg_mask].sum() / (self.pos_num * self.neg_num))


def auc_exact(p, y) -> float:
    """Tie-averaged AUC (probability a random positive outranks a random negative)."""
    p = _np(p).astype(np.float64)
    y = _np(y) > 0
    P, N = y.sum(), (~y).sum()
    if P == 0 or N == 0:
        return float("nan")
    order = np.argsort(p, kind="stable")
    ranks = np.empty(len(p), dtype=np.float64)
    sp = p[order]
    i = 0
    while i < len(sp):
        j = i
        while j + 1 < len(sp) and sp[j + 1] == sp[i]:
            j += 1
        ranks[order[i:j + 1]] = (i + j) / 2.0 + 1.0
        i = j + 1
    return float((ranks[y].sum() - P * (P + 1) / 2) / (P * N))


def auc_torch(p: torch.Tensor, y: torch.Tensor) -> float:
    """Device-side reference AUC (sort + cumsum on the GPU; K30)."""
    p = p.reshape(-1).float()
    y = (y.reshape(-1) > 0).float()
    P = y.sum()
    N = y.numel() - P
    order = torch.argsort(p, stable=True).flip(0)
    pos = y[order]
    cum = torch.cumsum(pos, 0)
    return float((cum * (1 - pos)).sum() / (P * N))


class SoftmaxPrecision:
    """argmax accuracy (SoftmaxPrecision.java:40-49; first max wins ties)."""

    def __init__(self, labels, probs):
        self.l = _np(labels).astype(np.int64)
        if isinstance(probs, torch.Tensor):
            probs = probs.detach().float().cpu().numpy()
        self.p = np.asarray(probs, dtype=np.float64).reshape(len(self.l), -1)

    def calculate(self) -> float:
        return float((self.p.argmax(axis=1) == self.l).mean())
