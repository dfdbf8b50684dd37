"""CTR demo (reference CTR.java:70-158): DNN.buildModel(23, 10, 45, {150, 10, 1}), Adam 0.005,
batch 1000, train -> test AUC -> loss surface each epoch.  ``--wide`` uses WideDeepNN
(FTRL wide part, hash space 100000).

The reference's CTR files (train.txt / test.txt) are not shipped; with no ``-Dtrain`` a
synthetic CTR stream with a known logistic optimum is used (ps_amd.data.synthetic_ctr).
With ``-Dtrain=file`` the native reader parses ``label|num,...|cat,...`` lines.
"""
from __future__ import annotations

import argparse

import torch

from ..context import ctx
from ..data.dataset import NativeBatchDataSet, synthetic_ctr
from ..eval.loss_surface import LossSurface
from ..eval.metrics import AUC
from ..models.reference import DNN, WideDeepNN
from ..obs import metrics
from .common import connect, device, make_trainer, maybe_run_server, setup, worker_rank


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--steps-per-epoch", type=int, default=50)
    ap.add_argument("--batch", type=int, default=1000)
    ap.add_argument("--wide", action="store_true")
    ap.add_argument("--init-scale", type=float, default=1.0)
    ap.add_argument("--loss-surface", action="store_true")
    ap.add_argument("--dump", default="", help="write final dense weights + probe rows (rank files) here")
    a, rest = ap.parse_known_args(argv)
    cfg = setup(rest)
    if maybe_run_server(cfg):
        return
    dev = device()
    conn, tables = connect(cfg, dev)  # embedding / wide rows live on the parameter server
    gen = torch.Generator().manual_seed(cfg.seed)
    if a.wide:
        model = WideDeepNN.build_model(23, 10, 45, [150, 10, 1], 100000, gen=gen, init_scale=a.init_scale,
                                       table_factory=tables)
    else:
        model = DNN.build_model(23, 10, 45, [150, 10, 1], gen=gen, init_scale=a.init_scale, table_factory=tables)
    model = model.to(dev)
    trainer = make_trainer(cfg, model, dev, conn)
    start = trainer.resume()  # newest committed checkpoint of -Dcheckpoint_dir (0 = fresh start)
    rank, world = worker_rank(cfg, conn)
    w0 = {n: p.detach().clone() for n, p in model.named_parameters()}
    test = synthetic_ctr(5000, wide_k=23 if a.wide else 0, seed=10 ** 6)
    gstep = 0
    for epoch in range(a.epochs):
        if cfg.train:
            ds = NativeBatchDataSet(cfg.train, "ctr", a.batch, dims=45, fields=23, offset=rank, step=world)
            batches = iter(ds)
        else:  # synthetic stream: global batch of step i, this rank trains its stride of it
            batches = ({k: v[rank::world] for k, v in
                        synthetic_ctr(a.batch, wide_k=23 if a.wide else 0, seed=epoch * 100000 + i).items()}
                       for i in range(a.steps_per_epoch))
        for b in batches:
            gstep += 1
            if gstep <= start:
                continue  # already in the checkpoint
            if "W" not in b and a.wide:
                b["W"] = b["E"] % 100000
            trainer.train([b])
        p = trainer.predict([test])[0]
        auc = AUC(p.cpu(), test["Y"]).calculate()
        metrics.plot("test_auc", auc, epoch)
        print(f"epoch {epoch} test auc {auc:.4f}", flush=True)
        if a.loss_surface:
            LossSurface({k: v.to(dev) for k, v in test.items()}, model, w0).plot()
    if trainer.ckpt is not None:
        trainer.ckpt.wait()
    if a.dump:
        trainer.engine.synchronize()
        probe = torch.arange(200).repeat(23, 1).t().contiguous()
        rows = model.tables()["emF"].pull(probe.to(dev))
        torch.save({"dense": {n: p.detach().cpu() for n, p in model.named_parameters()}, "rows": rows.cpu()},
                   f"{a.dump}.rank{rank}")


if __name__ == "__main__":
    main()
