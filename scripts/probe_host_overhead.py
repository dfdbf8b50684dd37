"""Host-side cost of one ResNet-50 bench step: issue time of step() with the GPU kept ahead of
the host (tiny batch: the GPU finishes every kernel before the host issues the next), vs the
synced wall time at the bench batch.  If the host issue time approaches the GPU time at
bs256, the step is launch-bound there and the GPU idles between dispatches.

Usage: python scripts/probe_host_overhead.py [--batches 8,256] [--steps 20]
Prints one JSON line per batch: host_ms (mean step() issue time), wall_ms (synced), and the
per-phase host split (forward / backward / finish_step)."""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="8,256")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    from ps_amd.models.resnet import prepare_for_mi355x, resnet50
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.transport import init_distributed
    from ps_amd.parallel.updaters import MomentumUpdater

    torch.cuda.set_device(0)
    tp = init_distributed(backend="gloo")
    torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
    dev = torch.device("cuda", 0)
    for B in [int(b) for b in a.batches.split(",")]:
        torch.manual_seed(0)
        model = prepare_for_mi355x(resnet50(fused_bn=True).to(dev))
        ps = ColocatedPS(model, MomentumUpdater(lr=0.1, momentum=0.9, weight_decay=5e-5), tp, bucket_mb=25.0)
        x = torch.randn(B, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (B,), device=dev)
        ph = {"fwd": 0.0, "bwd": 0.0, "finish": 0.0}

        def step(rec):
            t0 = time.perf_counter()
            loss = F.cross_entropy(model(x).float(), y)
            t1 = time.perf_counter()
            loss.backward()
            t2 = time.perf_counter()
            ps.finish_step()
            t3 = time.perf_counter()
            if rec:
                ph["fwd"] += t1 - t0
                ph["bwd"] += t2 - t1
                ph["finish"] += t3 - t2

        for _ in range(5):
            step(False)
        torch.cuda.synchronize()
        # host issue time: sync before each step so the launch queue is empty and never blocks
        host = 0.0
        for _ in range(a.steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            step(True)
            host += time.perf_counter() - t0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step(False)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        n = a.steps
        print(json.dumps({"batch": B, "host_ms": round(host / n * 1e3, 3), "wall_ms": round(wall / n * 1e3, 3),
                          **{k + "_host_ms": round(v / n * 1e3, 3) for k, v in ph.items()}}), flush=True)
        del model, ps, x, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
