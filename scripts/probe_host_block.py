"""Where the host waits in the ResNet-50 bench step (bs256 by default): the bench's own setup,
then per-step host time of forward / backward / finish_step with NO synchronisation (a host that
keeps ahead of the GPU returns from step() in its issue time; one that blocks returns in the GPU
time), and a torch.profiler CPU table of the runtime calls over 3 steps (synchronising calls show
up as long hipStreamSynchronize / hipEventSynchronize / hipMemcpy / aten::item entries).
usage: python scripts/probe_host_block.py [--batch-per-gpu N]  -> gpurun_out/host_block.txt"""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    sys.argv = [sys.argv[0]] + ["--batch-per-gpu", "256"] + sys.argv[1:]
    import bench as B
    from ps_amd import bench_configs as BC
    from ps_amd.parallel.transport import init_distributed

    args = B.parse()
    if args.batch_per_gpu == 0:
        args.batch_per_gpu = 256
    torch.cuda.set_device(0)
    tp = init_distributed(backend="gloo")
    torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    bench = BC.SETUPS["resnet50"](args, tp, dev)
    model_step = bench.step
    for _ in range(10):
        model_step()
    torch.cuda.synchronize()
    # split the step by hand (the bench step = forward + loss, backward, finish_step)
    ps = bench.engine
    model = ps.model if hasattr(ps, "model") else None
    lines = []
    t_prev = time.perf_counter()
    deltas = []
    for _ in range(20):
        model_step()
        t = time.perf_counter()
        deltas.append((t - t_prev) * 1e3)
        t_prev = t
    torch.cuda.synchronize()
    lines.append("host time between step() returns (ms, no sync): " + " ".join(f"{d:.2f}" for d in deltas))
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for _ in range(3):
            model_step()
        torch.cuda.synchronize()
    lines.append(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=40))
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/host_block.txt", "w") as f:
        f.write("\n".join(lines) + "\n")
    print(lines[0])


if __name__ == "__main__":
    main()
