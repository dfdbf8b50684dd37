"""GPU idle at the ResNet-50 step boundary WITHOUT a profiler: device events recorded on the
compute stream at the end of step k (after finish_step) and at the start of step k + 1 (before the
forward); their elapsed time is how long the compute stream waited in between (for the optimizer
serve of the last bucket on the comm stream, or for the host).  Also the wall per step.
usage: python scripts/probe_step_gap.py [--batch-per-gpu N] [--steps K]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    extra = sys.argv[1:]
    if "--batch-per-gpu" not in extra:
        extra = ["--batch-per-gpu", "256"] + extra
    sys.argv = [sys.argv[0]] + extra
    import bench as B
    from ps_amd import bench_configs as BC
    from ps_amd.parallel.transport import init_distributed

    args = B.parse()
    torch.cuda.set_device(0)
    tp = init_distributed(backend="gloo")
    torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    bench = BC.SETUPS["resnet50"](args, tp, dev)
    step = bench.step
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    n = args.steps
    ends, starts = [], []
    t0 = time.perf_counter()
    for _ in range(n):
        s = torch.cuda.Event(enable_timing=True)
        s.record()
        starts.append(s)
        step()
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ends.append(e)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n * 1e3
    gaps = [ends[k].elapsed_time(starts[k + 1]) for k in range(n - 1)]
    body = [starts[k].elapsed_time(ends[k]) for k in range(n)]
    print(json.dumps({"batch": args.batch_per_gpu, "wall_ms": round(wall, 3),
                      "step_body_ms": round(sum(body) / n, 3),
                      "boundary_gap_ms_mean": round(sum(gaps) / len(gaps), 3),
                      "boundary_gap_ms": [round(g, 3) for g in gaps]}))


if __name__ == "__main__":
    main()
