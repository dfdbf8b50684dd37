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
    ap.add_argument("--fused-bn", type=int, default=int(os.environ.get("PS_AMD_FUSED_BN", "1")),
                    help="HIP fused BatchNorm+residual+ReLU kernels (ops/bn.py) instead of MIOpen BN")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--graph", type=str, default=os.environ.get("PS_AMD_GRAPH", "0"),
                    help="capture the whole step in a HIP graph: 1/0/auto (measured slower on ROCm 7 for "
                         "ResNet-50: 40.8 vs 39.4 ms, profiles/r1_graph_vs_eager.txt)")
    ap.add_argument("--cudnn-benchmark", type=int, default=int(os.environ.get("PS_AMD_CONV_BENCHMARK", "1")),
                    help="MIOpen find (exhaustive) for each conv shape during warm-up")
    ap.add_argument("--profile-steps", type=int, default=0, help="torch.profiler over N extra steps (rank 0)")
    ap.add_argument("--json-out", type=str, default="")
    return ap.parse_args()


def setup_miopen_db():
    """Point MIOpen at a writable copy of the in-repo find/perf db (miopen_db/udb: conv
    algorithm choices for the ResNet-50 shapes, recorded by our own warm-up runs) so a
    fresh box skips most of the exhaustive search.  Naive reference solvers are excluded
    from find (they are never chosen and cost minutes to benchmark)."""
    import shutil
    import tempfile

    for k in ("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_BWD",
              "MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_WRW"):
        os.environ.setdefault(k, "0")
    if "MIOPEN_USER_DB_PATH" in os.environ:
        return
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "miopen_db")
    dst = os.path.join(tempfile.gettempdir(), f"ps_amd_miopen_{os.getuid()}_{os.environ.get('LOCAL_RANK', '0')}")
    try:
        for sub in ("udb", "cache"):
            os.makedirs(os.path.join(dst, sub), exist_ok=True)
            if os.path.isdir(os.path.join(src, sub)):
                for f in os.listdir(os.path.join(src, sub)):
                    if not os.path.exists(os.path.join(dst, sub, f)):
                        shutil.copy2(os.path.join(src, sub, f), os.path.join(dst, sub, f))
        os.environ["MIOPEN_USER_DB_PATH"] = os.path.join(dst, "udb")
        os.environ["MIOPEN_CUSTOM_CACHE_DIR"] = os.path.join(dst, "cache")
    except OSError:
        pass


def main():
    args = parse()
    setup_miopen_db()
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
    torch.backends.cudnn.benchmark = bool(args.cudnn_benchmark)
    torch.manual_seed(1234)

    model = prepare_for_mi355x(resnet50(fused_bn=bool(args.fused_bn)).to(dev), bn_fp32=bool(args.bn_fp32))
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

    use_graph = args.graph == "1" or (args.graph == "auto" and world == 1)
    tw0 = time.perf_counter()
    if use_graph:
        from ps_amd.train.graphs import GraphedStep

        # eager warm-up (MIOpen find) inside GraphedStep, then capture; W counts warm-up steps
        graphed = GraphedStep(step, warmup=max(1, args.warmup - 1))
        step = graphed
    else:
        for _ in range(args.warmup):
            step()
    torch.cuda.synchronize()
    if rank == 0:
        print(f"[bench] warmup {args.warmup} steps took {time.perf_counter() - tw0:.1f}s "
              f"(includes MIOpen find/compile for new conv shapes)", file=sys.stderr, flush=True)
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
                "hip_graph": bool(use_graph),
                "fused_bn": bool(args.fused_bn),
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
