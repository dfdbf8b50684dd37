"""1-bit compressed push at Llama-3-8B WIDTH (VERDICT r4 Next #4) and full DEPTH (VERDICT r5 Next #5):
the 8B hidden size (4096), FFN (14336), heads (32 q / 8 kv) and vocab (128256) with ``--layers`` blocks
(2: the round-5 width probe; 32: the whole 8.03B model, with ``--ckpt 1`` activation checkpointing
so two processes fit on one GPU) -- trained by W = 2 ranks over the xGMI plane with 64 MB buckets,
``--compress onebit`` (sign bits + per-chunk scales + error feedback, decoded in the owner's serve)
or ``none``.  Prints one JSON line per step (loss averaged over ranks) and a final line with the
plane's per-phase statistics and the 1-bit pack cost per bucket.  Reference: net/PSClient.java:37
(every push compressed), SURVEY K26.

  PS_AMD_BENCH_ONE_GPU=1 python -m torch.distributed.run --nproc-per-node 2 \\
      --master-addr 127.0.0.1 scripts/llama_width_onebit.py --compress onebit
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--compress", default="onebit", choices=["onebit", "none"])
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--timed", type=int, default=8, help="last N steps with per-phase timing")
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--ckpt", type=int, default=0, help="activation checkpointing per block")
    ap.add_argument("--ef", default="fp32", choices=["fp32", "bf16"], help="error-feedback buffer dtype")
    ap.add_argument("--warmup", type=int, default=0, help="full-precision rounds before the 1-bit push")
    ap.add_argument("--adam1bit", type=int, default=0,
                    help="1-bit Adam: push the worker momentum, owners freeze the variance after --warmup")
    ap.add_argument("--refresh", type=int, default=0, help="1-bit Adam: every k-th round full precision (variance refresh)")
    a = ap.parse_args()
    import faulthandler

    faulthandler.dump_traceback_later(45, repeat=True)  # a stuck phase names itself on stderr
    from ps_amd.models.transformer import LlamaConfig, LlamaForCausalLM
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.transport import init_distributed
    from ps_amd.parallel.updaters import AdamUpdater, OneBitAdamUpdater
    import torch.distributed as dist

    torch.cuda.set_device(0)
    tp = init_distributed(backend="gloo")
    dev = torch.device("cuda", 0)
    cfg = LlamaConfig(layers=a.layers)  # 8B width, reduced depth
    torch.manual_seed(0)
    ts = time.time()

    def say(msg):
        print(f"[rank {tp.rank} +{time.time() - ts:.1f}s] {msg}", file=sys.stderr, flush=True)

    with torch.device(dev):
        model = LlamaForCausalLM(cfg, checkpointing=bool(a.ckpt)).to(torch.bfloat16)
    torch.cuda.synchronize()
    say(f"model built, {torch.cuda.memory_allocated(dev) / 2**30:.1f} GB")
    nparam = sum(p.numel() for p in model.parameters())
    if a.adam1bit:
        upd = OneBitAdamUpdater(a.lr, 0.9, 0.95, 1e-8, bias_correction="step", weight_decay=0.1, adamw=True,
                                warmup=a.warmup, refresh=a.refresh)
    else:
        upd = AdamUpdater(a.lr, 0.9, 0.95, 1e-8, bias_correction="step", weight_decay=0.1, adamw=True)
    ps = ColocatedPS(model, upd, tp, bucket_mb=64.0, last_bucket_mb=2.0,
                     compress=None if a.compress == "none" else "onebit", plane="xgmi",
                     ef_dtype=torch.bfloat16 if a.ef == "bf16" else torch.float32, compress_warmup=a.warmup,
                     onebit_momentum=0.9 if a.adam1bit else None)
    torch.cuda.synchronize()
    say(f"PS built ({len(ps.reg.buckets)} buckets, plane {ps.plane_kind}), {torch.cuda.memory_allocated(dev) / 2**30:.1f} GB")
    g = torch.Generator(device=dev).manual_seed(100 + tp.rank)
    pool = [torch.randint(0, cfg.vocab, (a.batch, a.seq), device=dev, generator=g) for _ in range(4)]
    t0 = time.time()
    tprev = time.time()
    for step in range(a.steps):
        if step == a.steps - a.timed:
            ps.timing = True
            ps._mark("step0")
            ps.plane_stats(reset=True)
        ids = pool[step % len(pool)]
        loss = model(ids, ids)
        loss.backward()
        ps.finish_step()
        lv = torch.tensor([float(loss.item())])
        dist.all_reduce(lv)
        now = time.time()
        if tp.rank == 0:
            print(json.dumps({"step": step, "loss": round(lv.item() / tp.world, 5), "compress": a.compress,
                              "ms": round((now - tprev) * 1e3, 1)}), flush=True)
        tprev = now
        say(f"step {step} done")
    torch.cuda.synchronize()
    tsum = ps.timing_summary()
    pst = ps.plane_stats(reset=True)
    peaks = [None] * tp.world
    dist.all_gather_object(peaks, (round(torch.cuda.max_memory_allocated(dev) / 2**30, 1),
                                   round(torch.cuda.memory_reserved(dev) / 2**30, 1)))
    if tp.rank == 0:
        nb = len(ps.reg.buckets)
        packs = tsum.get("packs", 0.0)
        out = {"final": True, "compress": a.compress, "layers": a.layers, "hidden": cfg.hidden, "ffn": cfg.ffn,
               "vocab": cfg.vocab, "params": nparam, "world": tp.world, "buckets": nb,
               "bucket_mb": 64.0, "tokens_per_rank_step": a.batch * a.seq, "seconds": round(time.time() - t0, 1),
               "phase_ms_per_step": {k: round(v, 3) for k, v in tsum.items()},
               "pack_ms_per_bucket": round(tsum.get("pack_ms", 0.0) / packs, 4) if packs else None,
               "plane": {k: round(float(v), 3) for k, v in pst.items()},
               "checkpointing": bool(a.ckpt), "ef_dtype": a.ef, "compress_warmup": a.warmup, "adam1bit": bool(a.adam1bit), "refresh": a.refresh,
               "peak_allocated_reserved_gb_per_rank": peaks,
               "device_free_total_gb": [round(v / 2**30, 1) for v in torch.cuda.mem_get_info(dev)]}
        print(json.dumps(out), flush=True)
    ps.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
