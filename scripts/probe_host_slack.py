"""Host slack of the ResNet-50 bench step: how long the host waits in the run-ahead bound per step
(ColocatedPS._bound_run_ahead) vs the step time.  Slack near zero = the host's issue rate sets the
step (launch-bound); slack of several ms = the GPU does.
usage: python scripts/probe_host_slack.py [batch] [steps]"""
import os
import sys
import time
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from ps_amd import bench_configs as BC
    from ps_amd.parallel.transport import init_distributed

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    torch.cuda.set_device(0)
    tp = init_distributed(backend="gloo")
    args = types.SimpleNamespace(batch_per_gpu=B, image_size=224, fused_bn=1, bn_fp32=1, lr=0.1, bucket_mb=25.0,
                                 last_bucket_mb=2.0, staleness=0, plane="auto")
    torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
    b = BC.setup_resnet50(args, tp, torch.device("cuda", 0))
    eng = b.engine
    waits = []
    orig = eng._bound_run_ahead

    def timed_bound():
        t0 = time.perf_counter()
        orig()
        waits.append(time.perf_counter() - t0)

    eng._bound_run_ahead = timed_bound
    for _ in range(15):
        b.step()
    torch.cuda.synchronize()
    waits.clear()
    t0 = time.perf_counter()
    issue = []
    for _ in range(steps):
        s0 = time.perf_counter()
        b.step()
        issue.append(time.perf_counter() - s0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    w = sorted(waits)
    iss = sorted(issue)
    print(f"batch {B}: step {wall:.3f} ms; host time per step() median {iss[len(iss) // 2] * 1e3:.3f} ms; "
          f"run-ahead wait median {w[len(w) // 2] * 1e3:.3f} ms, min {w[0] * 1e3:.3f} ms "
          f"-> host issue ~{(iss[len(iss) // 2] - w[len(w) // 2]) * 1e3:.3f} ms per step", flush=True)


if __name__ == "__main__":
    main()
