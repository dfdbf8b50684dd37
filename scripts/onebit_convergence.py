"""1-bit compressed push: convergence vs full precision.

Tiny Llama (2 layers, hidden 64, vocab 512) trained with data parallelism over W = 2 gloo
processes on the co-located PS (AdamW 3e-3), on a learnable synthetic language (a fixed random
first-order Markov chain, entropy well below log(vocab)); each rank draws its own sequences.
Three runs: full-precision push, 1-bit push with error feedback from step 0, 1-bit after
``--warmup`` full-precision rounds.  Prints one JSON line with the loss curves (mean of every
10 steps) and the final gap to full precision.

    python scripts/onebit_convergence.py [--steps 300] [--warmup 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import dist_util  # noqa: E402


def markov_batch(g: torch.Generator, trans: torch.Tensor, b: int, s: int) -> torch.Tensor:
    v = trans.shape[0]
    ids = torch.empty(b, s, dtype=torch.long)
    ids[:, 0] = torch.randint(0, v, (b,), generator=g)
    for t in range(1, s):
        ids[:, t] = torch.multinomial(trans[ids[:, t - 1]], 1, generator=g).squeeze(1)
    return ids


def body(tp, compress, warmup, steps):
    from ps_amd.models.transformer import LlamaConfig, LlamaForCausalLM
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import AdamUpdater

    torch.manual_seed(0)
    cfg = LlamaConfig.tiny()
    m = LlamaForCausalLM(cfg)
    tg = torch.Generator().manual_seed(1234)  # the language: same on every rank
    logits = torch.randn(cfg.vocab, cfg.vocab, generator=tg) * 3.0
    trans = torch.softmax(logits, dim=1)
    ps = ColocatedPS(m, AdamUpdater(3e-3, 0.9, 0.95, 1e-8, bias_correction="step", weight_decay=0.01), tp,
                     bucket_mb=0.25, compress=compress, compress_warmup=warmup)
    g = torch.Generator().manual_seed(100 + tp.rank)
    losses = []
    for _ in range(steps):
        ids = markov_batch(g, trans, 16, 64)
        loss = m(ids, ids)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    ent = float(-(trans * trans.clamp_min(1e-12).log()).sum(1).mean())  # achievable loss floor
    return losses, ent


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=50)
    a = ap.parse_args()
    out = {"config": "tiny Llama (2x64, vocab 512), W=2 gloo, AdamW 3e-3, batch 16x64 per rank", "steps": a.steps}
    for name, comp, wu in [("full_precision", None, 0), ("onebit", "onebit", 0),
                           (f"onebit_warmup{a.warmup}", "onebit", a.warmup)]:
        res = dist_util.run(body, 2, (comp, wu, a.steps))
        losses, ent = res[0]
        curve = [round(sum(losses[i:i + 10]) / len(losses[i:i + 10]), 4) for i in range(0, len(losses), 10)]
        out[name] = {"curve_mean10": curve, "final_mean20": round(sum(losses[-20:]) / 20, 4)}
        out["entropy_floor"] = round(ent, 4)
        print(json.dumps({name: out[name]["final_mean20"]}), flush=True)
    fp = out["full_precision"]["final_mean20"]
    for k in list(out):
        if k.startswith("onebit"):
            out[k]["gap_vs_full_precision"] = round(out[k]["final_mean20"] - fp, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
