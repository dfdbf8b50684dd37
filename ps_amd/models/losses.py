"""Losses (loss/*.java).  All return the batch mean; autograd of the mean reproduces the
reference's per-sample delta followed by the 1/N of FcLayer's dW (FcLayer.java:105).

  CrossEntropy  binary CE on probabilities; ``slim`` = 0.01 early-stop threshold (:8)
  MSE           0.5 * (y - p)^2
  SoftmaxLoss   -log p[label] with the label as a class index (SoftmaxLoss.java:9-28)
"""
from __future__ import annotations

import torch


class Loss:
    def forward(self, p: torch.Tensor, y: torch.Tensor) -> torch.Tensor:  # pragma: no cover
        raise NotImplementedError

    __call__ = lambda self, p, y: self.forward(p, y)  # noqa: E731


class CrossEntropy(Loss):
    slim = 0.01

    def forward(self, p, y):
        p = p.float().reshape(-1)
        y = y.float().reshape(-1)
        return -(y * torch.log(p) + (1 - y) * torch.log(1 - p)).mean()


class MSE(Loss):
    def forward(self, p, y):
        p = p.float().reshape(-1)
        y = y.float().reshape(-1)
        return (0.5 * (y - p) ** 2).mean()


class SoftmaxLoss(Loss):
    def forward(self, p, y):
        hot = p.float().gather(1, y.long().view(-1, 1)).view(-1)
        return -torch.log(hot).mean()
