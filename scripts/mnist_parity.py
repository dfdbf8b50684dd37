"""Reference-quality parity on the bundled data.

Trains the reference's two MNIST models with the reference hyper-parameters on the 1000-row
``mnist_test.csv`` shipped with the reference (the only MNIST data it ships), split 800 train /
200 held out, and prints held-out accuracy per seed:

  MLP  FullConnectedNN.buildModel(784, {150, 50, 10}); Adam(0.005, 0.9, 0.999, 1e-8) with the
       reference's constant bias correction; 4 replicas per round (Mnist.java:77 Context.thread=4),
       batch 100 per replica (the reference's 1000 does not fit 800 rows x 4); softmax T=10000
       on RAW 0-255 pixels exactly as MnistParser feeds them (Mnist.java:44-70); 100 epochs or
       the reference's early stop (loss <= 0.01).
  CNN  CNN.buildModel(28, 28, 1, {150, 50, 10}); same Adam; 1 replica, batch 100
       (CnnMnist.java:68-86); 100 epochs or early stop.

    python scripts/mnist_parity.py [--seeds 0 1 2] [--epochs 100] [--model mlp|cnn|both] [--device cuda]

On ``--device cuda`` the models run the in-house GPU kernels (FC: fused MFMA linear + K2
backward; CNN convs: HIP im2col -> fp32 MFMA linear -> K2 -> HIP col2im; HIP max-pool,
softmax-T, fused Adam on the PS shard).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ps_amd.context import ctx  # noqa: E402
from ps_amd.data.dataset import load_reference_mnist  # noqa: E402
from ps_amd.eval.metrics import SoftmaxPrecision  # noqa: E402
from ps_amd.models.reference import CNN, FullConnectedNN  # noqa: E402
from ps_amd.train.trainer import CollectiveEngine, Trainer  # noqa: E402


def run(kind: str, seed: int, epochs: int, raw: bool = True, device: str = "cpu", train_rows: int = 800,
        temp: float = 10000.0) -> dict:
    d = load_reference_mnist()
    X = d["X"] * (255.0 if raw else 1.0)
    Y = d["Y"]
    ctx.init()
    torch.manual_seed(seed)
    gen = torch.Generator().manual_seed(seed)
    if kind == "mlp":
        model, k, bs = FullConnectedNN.build_model(784, [150, 50, 10], gen=gen, softmax_temp=temp), 4, 100
    else:
        model, k, bs = CNN.build_model(28, 28, 1, [150, 50, 10], gen=gen, softmax_temp=temp), 1, 100
    dev = torch.device(device)
    model.to(dev)
    tr = Trainer(model, CollectiveEngine(model), n_threads=k, device=dev if dev.type == "cuda" else None)
    n = train_rows  # rows 0 .. n-1 train (a learning curve below 800); rows 800-999 are always held out
    Xt, Yt = X[:n], Y[:n]
    bs = min(bs, n // k)
    t0 = time.time()
    ep = 0
    for ep in range(epochs):
        perm = torch.randperm(n, generator=gen)
        for i in range(0, n - bs * k + 1, bs * k):
            idx = perm[i:i + bs * k]
            tr.train([{"X": Xt[idx[j * bs:(j + 1) * bs]], "Y": Yt[idx[j * bs:(j + 1) * bs]]} for j in range(k)])
            if ctx.finish:
                break
        if ctx.finish:
            break
    p = tr.predict([{"X": X[800:]}])[0]
    acc = SoftmaxPrecision(Y[800:], p.cpu()).calculate()
    from ps_amd.models.losses import CrossEntropy

    return {"model": kind, "seed": seed, "train_rows": n, "softmax_temp": temp, "slim": CrossEntropy.slim,
            "epochs_run": ep + 1,
            "heldout_acc": round(float(acc), 4), "raw_pixels": raw, "device": device,
            "seconds": round(time.time() - t0, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--model", default="both", choices=["mlp", "cnn", "both"])
    ap.add_argument("--device", default="cpu", choices=["cpu", "cuda"])
    ap.add_argument("--train-rows", type=int, nargs="+", default=[800])
    ap.add_argument("--temp", type=float, default=10000.0, help="softmax temperature (reference: 10000)")
    ap.add_argument("--slim", type=float, default=None,
                    help="early-stop threshold on a batch's loss (reference CrossEntropy.slim = 0.01; 0 = off)")
    a = ap.parse_args()
    if a.slim is not None:
        from ps_amd.models.losses import CrossEntropy

        CrossEntropy.slim = a.slim if a.slim > 0 else -1.0
    torch.set_num_threads(4)
    kinds = ["mlp", "cnn"] if a.model == "both" else [a.model]
    for n in a.train_rows:
        for kind in kinds:
            for s in a.seeds:
                print(json.dumps(run(kind, s, a.epochs, device=a.device, train_rows=n, temp=a.temp)), flush=True)


if __name__ == "__main__":
    main()
