#!/usr/bin/env python
"""Headline benchmark: ResNet-50 sync-BSP on the co-located parameter server.

BASELINE.json metric: "samples/sec (whole node) ResNet-50 sync-BSP at 1/2/4/8 MI355X
workers" -- one process per GPU (torchrun), every rank a worker + the server of its range
partition (ps_amd/parallel/colocated.py).  Data plane (``--plane``, default auto = xgmi on one
node): push = land the bucket in the rank's own IPC-mapped buffer, serve = ONE kernel per owner
reading its chunk from all W peers over xGMI, fp32 sum fused with the HIP momentum-SGD step,
pull = ONE kernel copying every other owner's fresh chunk (ps_amd/parallel/plane.py); or
``collective`` = RCCL reduce-scatter / all-gather.  Both overlap with backward.
BatchNorm+residual+ReLU run as fused HIP kernels (ps_amd/ops/bn.py).

Weak scaling: ``--batch-per-gpu`` images per rank per step (default 1024 -- sized for the
288 GB HBM: ~50 GB peak; measured 10.5K / 11.6K / 12.1K / 12.4K / 12.3K / 12.4K img/s at
256 / 512 / 768 / 1024 / 1536 / 2048 per GPU, profiles/r2_resnet50_batch_sweep.txt), synthetic ImageNet-shaped data resident on the GPU, random-init weights, bf16
compute (channels_last), full optimizer step inside the timed region.

Other BASELINE configs: ``--config bert-ssp | dlrm | llama-onebit | mlp-tcp`` (see
ps_amd/bench_configs.py).

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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=os.environ.get("PS_AMD_BENCH_CONFIG", "resnet50"),
                    choices=["resnet50", "bert-ssp", "dlrm", "llama-onebit", "mlp-tcp", "ctr-async"])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: contract dry run of the same code path on CPU tensors over gloo (tests only; "
                         "the fused HIP paths fall back to the torch module path)")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-per-gpu", type=int, default=0, help="0 = config default")
    ap.add_argument("--seq-len", type=int, default=0, help="0 = config default")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--bucket-mb", type=float, default=float(os.environ.get("PS_AMD_BUCKET_MB", "25")))
    ap.add_argument("--last-bucket-mb", type=float, default=2.0)
    ap.add_argument("--staleness", type=int, default=0)
    ap.add_argument("--async-ps", type=int, default=1,
                    help="bert: the asynchronous PS (one-sided pushes); 0: the pipelined collective SSP engine")
    ap.add_argument("--plane", default=os.environ.get("PS_AMD_PLANE", "auto"), choices=["auto", "xgmi", "collective"],
                    help="PS data plane at world > 1: one-sided xGMI plane (IPC) or RCCL collectives")
    ap.add_argument("--bn-fp32", type=int, default=1)
    ap.add_argument("--fused-bn", type=int, default=1,
                    help="HIP fused BatchNorm+residual+ReLU kernels (ops/bn.py) instead of MIOpen BN")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--dlrm-rows", type=int, default=1000000)
    ap.add_argument("--tiny", type=int, default=0, help="llama-onebit: tiny config (smoke only)")
    ap.add_argument("--profile-steps", type=int, default=0, help="torch.profiler over N extra steps (rank 0)")
    ap.add_argument("--json-out", type=str, default="")
    ap.add_argument("--comm-probe", type=int, default=1,
                    help="world > 1: after the timed region, measure RS / AG / AR bandwidth (ps_amd/parallel/"
                         "comm_probe.py) and report it in the JSON config")
    ap.add_argument("--compute-priority", choices=["auto", "high", "normal"], default="auto",
                    help="stream priority of forward / backward (auto: high for ResNet-50 with one rank per GPU)")
    ap.add_argument("--checkpoint-dir", type=str, default=os.environ.get("PS_AMD_CHECKPOINT_DIR", ""),
                    help="after the timed region: one sharded checkpoint of every rank's server shard (timed, "
                         "reported on stderr) -- utils/checkpoint.py")
    ap.add_argument("--sync-audit", type=int, default=-1,
                    help="after the timed region: N steps under torch.cuda.set_sync_debug_mode('warn'), "
                         "reporting the host-synchronising torch ops per step (default 2 for the sparse "
                         "configs, 0 otherwise)")
    ap.add_argument("--timing", type=int, default=0,
                    help="after the timed region: N more steps with per-phase device timing "
                         "(fwd+bwd / push / serve / pull / exposed comm) printed to stderr")
    return ap.parse_args()


def _stream_count(engine, prio: str, side: bool, cpu: bool) -> int:
    """HIP streams this rank issues work on in the timed steps: compute (the default or a
    high-priority one), the weight-gradient side stream, and the PS engine's comm streams."""
    if cpu:
        return 0
    n = 1 + int(side)
    if engine is None:
        return n
    if getattr(engine, "plane", None) is not None:
        return n + 2  # the xGMI plane engine's native serve and pull streams (csrc/plane.cpp)
    seen = {id(s) for s in (getattr(engine, a, None) for a in ("comm", "comm_pull", "pull_stream"))
            if s is not None}
    return n + len(seen)


def main():
    args = parse()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from ps_amd import bench_configs as BC

    if args.config == "mlp-tcp":  # CPU plumbing config: no GPU involved
        rec = BC.run_mlp_tcp(args.steps)
        rec["warmup"] = 2
        print(json.dumps(rec), flush=True)
        return 0
    d = BC.DEFAULTS[args.config]
    args.batch_per_gpu = args.batch_per_gpu or d["batch"]
    args.seq_len = args.seq_len or d["seq"]
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world_env == 1:
        # launch ourselves under torchrun as a CHILD process (never exec from a GPU process)
        import subprocess

        import socket

        with socket.socket() as so:  # a free rendezvous port (several benches may share a node)
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
        return subprocess.call(cmd)
    cpu = args.device == "cpu"
    if not cpu and not torch.cuda.is_available():
        print(json.dumps({"metric": args.config, "value": None, "error": "no GPU visible"}))
        return 1
    from ps_amd.parallel.transport import init_distributed
    import torch.distributed as dist

    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-GPU path on a one-GPU box: every rank on cuda:0, gloo for the
    # control plane (RCCL refuses two ranks on one device); the xGMI plane still runs its IPC path
    one_gpu = os.environ.get("PS_AMD_BENCH_ONE_GPU", "0") == "1"
    if one_gpu:
        local = 0
    if not cpu:
        torch.cuda.set_device(local)
    tp = init_distributed(backend="gloo" if (cpu or one_gpu) else None)
    rank, world = tp.rank, tp.world
    from ps_amd.ops import side_stream as _side
    from ps_amd.parallel.transport import ranks_per_device

    rpd = ranks_per_device()  # ranks computing on this rank's GPU (1 on a real node)
    prio = "normal"
    if not cpu:
        # forward / backward on a high-priority stream: the weight-gradient side stream and the
        # PS's comm streams (normal priority) then take the CUs the compute chain leaves idle.
        # Default: high for ResNet-50 when this rank owns its GPU -- the single-process case it was
        # measured on (bs1024 +0.15 %, three interleaved pairs, profiles/r4_wgrad_stream_policy.txt),
        # which a one-process-per-GPU node reproduces whatever WORLD_SIZE is; normal when ranks
        # share a GPU, and for the asynchronous configs, whose owner service threads launch on
        # normal-priority streams (--compute-priority forces it)
        prio = args.compute_priority
        if prio == "auto":
            prio = "high" if (rpd == 1 and args.config == "resnet50") else "normal"
        if prio == "high":
            torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
    dev = torch.device("cpu") if cpu else torch.device("cuda", local)

    def sync():
        if not cpu:
            torch.cuda.synchronize()

    torch.manual_seed(1234)
    bench = BC.SETUPS[args.config](args, tp, dev)
    step = bench.step

    tw0 = time.perf_counter()
    for _ in range(args.warmup):
        step()
    sync()
    if rank == 0:
        print(f"[bench] {args.config}: warmup {args.warmup} steps took {time.perf_counter() - tw0:.1f}s "
              f"(kernel warm-up, allocator growth, PS setup)", file=sys.stderr, flush=True)
    tp.barrier()
    sync()
    if bench.stats is not None:
        bench.stats()  # zero the counters at the start of the timed region
    seg0 = None if cpu else torch.cuda.memory_stats(dev).get("num_device_alloc", 0)
    res0 = None if cpu else torch.cuda.memory_reserved(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    tp.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev if tp.backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    timed_stats = bench.stats() if bench.stats is not None else None
    # allocator steady state: a timed step that hipMallocs new segments means the host ran ahead of
    # the GPU far enough that freed blocks still pending on another stream could not be reused --
    # the mechanism behind the multi-second stall of an unbounded run-ahead
    # (profiles/r6_stall_root_cause.txt); the engines' in-flight bound keeps this at 0
    alloc_timed = None if cpu else torch.cuda.memory_stats(dev).get("num_device_alloc", 0) - seg0
    grew_gb = None if cpu else (torch.cuda.memory_reserved(dev) - res0) / 2**30
    if grew_gb is not None and grew_gb > 8 and rank == 0:  # (a bounded run adds one step's pending blocks at most)
        print(f"[bench] WARNING: the allocator grew by {grew_gb:.1f} GB ({alloc_timed} segments) inside the timed "
              f"region: the host ran far ahead of the GPU (PS_AMD_MAX_INFLIGHT=0?)", file=sys.stderr, flush=True)
    value = bench.samples_per_step * world * args.steps / elapsed
    # after the timed region: per-phase PS timing (default 3 steps at world > 1, so the driver's
    # multi-GPU lines show how much of the push / pull the backward hides) and the collective
    # bandwidth curve of this node's RCCL / xGMI plane
    tsum = comm = None
    n_timing = args.timing if args.timing else (3 if world > 1 else 0)
    if n_timing and getattr(bench.engine, "timing_summary", None) is not None:
        eng = bench.engine
        try:
            eng.timing = True
            eng._mark("step0")
            for _ in range(n_timing):
                step()
            sync()
            tsum = {k: round(v, 3) for k, v in eng.timing_summary().items()}
            if getattr(eng, "plane", None) is not None:
                eng.plane_stats(reset=True)
                for _ in range(n_timing):
                    step()
                sync()
                tsum.update({"plane_" + k: round(float(v), 3) for k, v in eng.plane_stats(reset=True).items()})
        except Exception as e:  # diagnostics only: never lose the measured line
            print(f"[bench-timing] failed: {e!r}", file=sys.stderr, flush=True)
        eng.timing = False
        if rank == 0 and tsum:
            print("[bench-timing] " + json.dumps(tsum), file=sys.stderr, flush=True)
    audit = None
    n_audit = args.sync_audit if args.sync_audit >= 0 else (2 if args.config in ("dlrm", "ctr-async") else 0)
    if n_audit and not cpu:
        import warnings

        try:
            with warnings.catch_warnings(record=True) as ws:
                warnings.simplefilter("always")
                torch.cuda.set_sync_debug_mode("warn")
                for _ in range(n_audit):
                    step()
                torch.cuda.set_sync_debug_mode(0)
            sync()
            # (torch's one-time "Synchronization debug mode is a prototype feature" notice is not a sync)
            hits = [str(w.message).split("\n")[0][:80] for w in ws
                    if "synchroniz" in str(w.message) and "prototype feature" not in str(w.message)]
            audit = {"host_syncs_per_step": round(len(hits) / n_audit, 2), "sync_ops": sorted(set(hits))[:4]}
        except Exception as e:  # diagnostics only
            torch.cuda.set_sync_debug_mode(0)
            print(f"[bench-sync-audit] failed: {e!r}", file=sys.stderr, flush=True)
    if world > 1 and args.comm_probe:
        from ps_amd.parallel.comm_probe import probe

        try:
            comm = probe(dev)
        except Exception as e:
            print(f"[bench-comm-probe] failed: {e!r}", file=sys.stderr, flush=True)
    if args.checkpoint_dir and getattr(bench.engine, "shard_state", None) is not None:
        from ps_amd.utils.checkpoint import CheckpointManager

        tc = time.perf_counter()
        ck = CheckpointManager(args.checkpoint_dir, rank=rank, world=world)
        ck.save(args.warmup + args.steps, bench.engine, None, extra={"config": args.config}, blocking=True)
        if rank == 0:
            print(f"[bench-checkpoint] sharded save of step {args.warmup + args.steps} took "
                  f"{time.perf_counter() - tc:.2f}s (committed={ck.latest() is not None})", file=sys.stderr,
                  flush=True)
    if args.profile_steps and rank == 0:
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(args.profile_steps):
                step()
            sync()
        os.makedirs("gpurun_out", exist_ok=True)
        with open("gpurun_out/torch_profile.txt", "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
    if rank == 0:
        cfg = dict(bench.config)
        # the stream policy this run used (keyed on ranks sharing a GPU, not on WORLD_SIZE)
        images = bench.samples_per_step if args.config == "resnet50" else None
        cfg["ranks_per_device"] = rpd
        cfg["compute_priority"] = prio
        cfg["side_stream"] = bool(not cpu and images is not None and _side.enabled(images))
        cfg["streams_per_rank"] = _stream_count(bench.engine, prio, cfg["side_stream"], cpu)
        if getattr(bench.engine, "plane_kind", None) is not None:
            cfg["data_plane"] = bench.engine.plane_kind
        if getattr(getattr(bench.engine, "plane", None), "info", None) is not None:
            cfg["plane_info"] = dict(bench.engine.plane.info)
        cfg["final_loss"] = round(float(loss.item()), 4)
        cfg["peak_mem_gb"] = None if cpu else round(torch.cuda.max_memory_allocated(dev) / 2**30, 1)
        if not cpu:
            cfg["reserved_gb"] = round(torch.cuda.memory_reserved(dev) / 2**30, 1)
            cfg["device_allocs_timed"] = alloc_timed
            cfg["reserved_growth_timed_gb"] = round(grew_gb, 2)
        if timed_stats:
            cfg.update(timed_stats)
        if audit is not None:
            cfg["sync_audit"] = audit  # torch ops that synchronised the host, after the timed region
        if tsum:
            cfg["ps_phase_ms_per_step"] = tsum  # measured after the timed region
        if comm:
            cfg["rccl_probe"] = comm  # measured after the timed region
        rec = {
            "metric": bench.metric,
            "value": round(value, 2),
            "unit": bench.unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,  # the reference publishes no throughput number
            "dtype": bench.dtype,
            "data": f"synthetic: a pool of {BC.POOL if args.config != 'dlrm' else 4 * BC.POOL} distinct "
                    f"GPU-resident batches of the named shape, cycled; random-init weights",
            "config": cfg,
        }
        line = json.dumps(rec)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if getattr(bench.engine, "close", None) is not None:
        bench.engine.close()  # stops async-PS progress threads before the process tears down
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
