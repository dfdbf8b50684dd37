"""MNIST MLP demo (reference Mnist.java:75-155): FullConnectedNN(784, {150, 50, 10}),
Adam 0.005, batch 100 x ``-Dthread`` replicas (reference: 1000 x 4).

    python -m ps_amd.apps.mnist [-Dtrain=path.csv] [-Dtest=path.csv] [-Dthread=4] [--epochs 10]

The reference's training CSV is not shipped (.MISSING_LARGE_BLOBS); by default the bundled
1000-row mnist_test.csv is split 800/200.
"""
from __future__ import annotations

import argparse

import torch

from ..context import ctx
from ..data.dataset import load_reference_mnist
from ..eval.metrics import SoftmaxPrecision
from ..models.reference import FullConnectedNN
from ..obs import metrics
from .common import device, make_trainer, maybe_run_server, setup


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=50)
    ap.add_argument("--batch", type=int, default=100)
    a, rest = ap.parse_known_args(argv)
    cfg = setup(rest)
    if maybe_run_server(cfg):
        return
    dev = device()
    if cfg.train:
        tr_d = load_reference_mnist(cfg.train)
        te_d = load_reference_mnist(cfg.test or cfg.train)
    else:
        d = load_reference_mnist()
        tr_d = {k: v[:800] for k, v in d.items()}
        te_d = {k: v[800:] for k, v in d.items()}
    model = FullConnectedNN.build_model(784, [150, 50, 10], gen=torch.Generator().manual_seed(cfg.seed)).to(dev)
    trainer = make_trainer(cfg, model, dev)
    n = tr_d["X"].shape[0]
    g = torch.Generator().manual_seed(cfg.seed)
    k = max(1, cfg.thread)
    for epoch in range(a.epochs):
        perm = torch.randperm(n, generator=g)
        for i in range(0, n - a.batch * k + 1, a.batch * k):
            idx = perm[i:i + a.batch * k]
            trainer.train([{"X": tr_d["X"][idx[j * a.batch:(j + 1) * a.batch]],
                            "Y": tr_d["Y"][idx[j * a.batch:(j + 1) * a.batch]]} for j in range(k)])
            if ctx.finish:
                break
        p = trainer.predict([{"X": te_d["X"]}])[0]
        prec = SoftmaxPrecision(te_d["Y"], p.cpu()).calculate()
        metrics.plot("test_precision", prec, epoch)
        print(f"epoch {epoch} test precision {prec:.4f}", flush=True)
        if ctx.finish:
            break


if __name__ == "__main__":
    main()
