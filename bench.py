#!/usr/bin/env python
"""Headline benchmark: ResNet-50 sync-BSP on the co-located parameter server.

BASELINE.json metric: "samples/sec (whole node) ResNet-50 sync-BSP at 1/2/4/8 MI355X
workers" -- one process per GPU (torchrun), every rank a worker + the server of its range
partition, push = RCCL reduce-scatter, server = fused HIP momentum-SGD on the fp32 master
shard, pull = RCCL all-gather, all overlapped with backward (ps_amd/parallel/colocated.py).

Weak scaling: ``--batch-per-gpu`` images per rank per step (default 256), synthetic
ImageNet-shaped data resident on the GPU, random-init weights, bf16 compute (channels_last),
full optimizer step inside the timed region.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; W untimed steps, then
exactly K timed steps bracketed by barrier + cuda.synchronize on both sides; the max
elapsed over ranks is used; rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

METRIC = "samples/sec (whole node) ResNet-50 sync-BSP at 1/2/4/8 MI355X workers"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-per-gpu", type=int, default=int(os.environ.get("PS_AMD_BENCH_BATCH", "256")))
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--bucket-mb", type=float, default=float(os.environ.get("PS_AMD_BUCKET_MB", "25")))
    ap.add_argument("--last-bucket-mb", type=float, default=2.0)
    ap.add_argument("--staleness", type=int, default=0)
    ap.add_argument("--bn-fp32", type=int, default=1)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--profile-steps", type=int, default=0, help="torch.profiler over N extra steps (rank 0)")
    ap.add_argument("--json-out", type=str, default="")
    return ap.parse_args()


def main():
    args = parse()
    from ps_amd.parallel.transport import init_distributed
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import MomentumUpdater
    from ps_amd.models.resnet import resnet50, prepare_for_mi355x
    import torch.distributed as dist

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world_env == 1:
        # re-launch ourselves under torchrun as a CHILD process (never exec from a GPU process)
        import subprocess

        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", "--master-port=29533", __file__] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    if not torch.cuda.is_available():
        print(json.dumps({"metric": METRIC, "value": None, "error": "no GPU visible"}))
        return 1
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    tp = init_distributed()
    rank, world = tp.rank, tp.world
    dev = torch.device("cuda", local)
    torch.backends.cudnn.benchmark = True
    torch.manual_seed(1234)

    model = prepare_for_mi355x(resnet50().to(dev), bn_fp32=bool(args.bn_fp32))
    upd = MomentumUpdater(lr=args.lr, momentum=0.9, weight_decay=5e-5)
    ps = ColocatedPS(model, upd, tp, bucket_mb=args.bucket_mb, last_bucket_mb=args.last_bucket_mb,
                     staleness=args.staleness)
    B, S = args.batch_per_gpu, args.image_size
    g = torch.Generator(device=dev).manual_seed(rank)
    x = torch.randn(B, 3, S, S, device=dev, generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), device=dev, generator=g)

    def step():
        out = model(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        ps.finish_step()
        return loss

    for _ in range(args.warmup):
        step()
    tp.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    tp.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    samples = B * world * args.steps
    value = samples / elapsed
    if args.profile_steps and rank == 0:
        from torch.profiler import profile, ProfilerActivity

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(args.profile_steps):
                step()
            torch.cuda.synchronize()
        os.makedirs("gpurun_out", exist_ok=True)
        with open("gpurun_out/torch_profile.txt", "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random ImageNet-shaped images + labels, GPU resident); random-init weights",
            "config": {
                "model": "ResNet-50",
                "global_batch": B * world,
                "seq_len": None,
                "image_size": S,
                "parallelism": f"ps-bsp-colocated-dp{world}",
                "optimizer": upd.name,
                "bucket_mb": args.bucket_mb,
                "staleness": args.staleness,
                "final_loss": round(float(loss.item()), 4),
            },
        }
        line = json.dumps(rec)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
