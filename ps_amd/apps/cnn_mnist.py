"""CNN MNIST demo (reference CnnMnist.java:66-95): CNN.buildModel(28, 28, 1, {150, 50, 10}),
batch 100, 1 thread.  ``python -m ps_amd.apps.cnn_mnist [--epochs N]``."""
from __future__ import annotations

import argparse

import torch

from ..context import ctx
from ..data.dataset import load_reference_mnist
from ..eval.metrics import SoftmaxPrecision
from ..models.reference import CNN
from ..obs import metrics
from .common import device, make_trainer, maybe_run_server, setup


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--batch", type=int, default=100)
    a, rest = ap.parse_known_args(argv)
    cfg = setup(rest)
    if maybe_run_server(cfg):
        return
    dev = device()
    d = load_reference_mnist(cfg.train or None)
    tr_d = {k: v[:800] for k, v in d.items()}
    te_d = {k: v[800:] for k, v in d.items()}
    model = CNN.build_model(28, 28, 1, [150, 50, 10], gen=torch.Generator().manual_seed(cfg.seed)).to(dev)
    trainer = make_trainer(cfg, model, dev)
    for epoch in range(a.epochs):
        for i in range(0, 800, a.batch):
            trainer.train([{"X": tr_d["X"][i:i + a.batch], "Y": tr_d["Y"][i:i + a.batch]}])
            if ctx.finish:
                break
        p = trainer.predict([{"X": te_d["X"]}])[0]
        prec = SoftmaxPrecision(te_d["Y"], p.cpu()).calculate()
        metrics.plot("test_precision", prec, epoch)
        print(f"epoch {epoch} test precision {prec:.4f}", flush=True)


if __name__ == "__main__":
    main()
