"""The BASELINE.json benchmark configs (bench.py ``--config``).

  resnet50      ResNet-50 sync-BSP, co-located PS, fused HIP momentum SGD     (headline)
  bert-ssp      BERT-base MLM, bounded staleness s=1 (SSP), fused HIP AdamW
  dlrm          DLRM-style: 26 sharded embedding tables, sparse push/pull, row-wise
                Adagrad on the owning server (HIP), dense MLPs on the co-located PS
  llama-onebit  Llama-3-8B bf16, 1-bit compressed gradient push with error feedback
  ctr-async     the reference CTR Wide&Deep (23 fields x 10, 45 numeric, FC 150-10-1, wide hash
                100000) on the asynchronous PS: dense keys through AsyncPS SSP(1), embedding and
                wide rows through the device-resident asynchronous row tables
  mlp-tcp       2-layer MLP, 1 dedicated server + 2 workers on CPU/TCP loopback (plumbing)

Each ``setup_*`` returns a Bench with ``step()`` (one full PS round: forward, backward,
push, server update, pull -- nothing skipped), the samples processed per step on THIS rank,
and the metric/config metadata.  Synthetic data of the named shape, random-init weights.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Callable, Dict, Optional

import torch
import torch.nn.functional as F


POOL = 8  # distinct GPU-resident synthetic batches cycled


def _cycle(pool):
    while True:
        yield from pool


@dataclass
class Bench:
    step: Callable[[], torch.Tensor]
    samples_per_step: int
    metric: str
    unit: str
    config: Dict = field(default_factory=dict)
    engine: object = None
    stats: Optional[Callable[[], Dict]] = None  # extra counters for the JSON line (read after timing)
    dtype: str = "bf16"  # compute dtype reported in the JSON line


def setup_resnet50(args, tp, dev) -> Bench:
    from .models.resnet import prepare_for_mi355x, resnet50
    from .parallel.colocated import ColocatedPS
    from .parallel.updaters import MomentumUpdater

    model = prepare_for_mi355x(resnet50(fused_bn=bool(args.fused_bn)).to(dev), bn_fp32=bool(args.bn_fp32))
    upd = MomentumUpdater(lr=args.lr, momentum=0.9, weight_decay=5e-5)
    ps = ColocatedPS(model, upd, tp, bucket_mb=args.bucket_mb, last_bucket_mb=args.last_bucket_mb,
                     staleness=args.staleness, plane=getattr(args, "plane", None))
    B, S = args.batch_per_gpu, args.image_size
    g = torch.Generator(device=dev).manual_seed(tp.rank)
    pool = [(torch.randn(B, 3, S, S, device=dev, generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last), torch.randint(0, 1000, (B,), device=dev, generator=g))
        for _ in range(POOL)]
    it = _cycle(pool)

    def step():
        x, y = next(it)
        loss = F.cross_entropy(model(x).float(), y)
        loss.backward()
        ps.finish_step()
        return loss

    return Bench(step, B, "samples/sec (whole node) ResNet-50 sync-BSP at 1/2/4/8 MI355X workers", "samples/s",
                 {"model": "ResNet-50", "global_batch": B * tp.world, "seq_len": None, "image_size": S,
                  "parallelism": f"ps-bsp-colocated-dp{tp.world}", "optimizer": upd.name,
                  "bucket_mb": args.bucket_mb, "staleness": args.staleness, "fused_bn": bool(args.fused_bn)}, ps)


def async_or_pipelined(model, upd, tp, stale: int, args, use_async: bool = True):
    """The SSP(stale) engine of a model: the asynchronous PS (one-sided pushes into the owners'
    mailboxes + native progress threads, async_ps.py) -- or, when its start-up remote-write probe
    fails on any rank (remote_probe.py; every rank sees the same outcome), the pipelined
    collective rounds of ColocatedPS with the same staleness.  -> (engine, async?, probe record)."""
    from .parallel.colocated import ColocatedPS

    probe = {}
    if use_async:
        from .parallel.async_ps import AsyncPS
        from .parallel.remote_probe import RemoteWriteUnavailable

        try:
            ps = AsyncPS(model, upd, tp, staleness=stale)
            probe = {k: v for k, v in ps.info.items() if k == "remote_write_probe"}
            return ps, True, probe
        except RemoteWriteUnavailable as e:
            probe = {"remote_write_probe": "failed", "engine_fallback": "pipelined-collective: " + str(e)[:300]}
            if tp.rank == 0:
                print(f"[bench] {e}; falling back to the pipelined collective SSP", flush=True,
                      file=__import__("sys").stderr)
    ps = ColocatedPS(model, upd, tp, bucket_mb=args.bucket_mb, last_bucket_mb=args.last_bucket_mb,
                     staleness=stale, clip_norm=None)
    return ps, False, probe


def setup_bert_ssp(args, tp, dev) -> Bench:
    from .models.transformer import BertForMLM, mlm_batch
    from .parallel.updaters import AdamUpdater

    torch.manual_seed(0)
    model = BertForMLM().to(dev).to(torch.bfloat16)
    upd = AdamUpdater(1e-4, 0.9, 0.999, 1e-6, bias_correction="step", weight_decay=0.01, adamw=True)
    stale = 1 if args.staleness == 0 else args.staleness
    ps, use_async, probe = async_or_pipelined(model, upd, tp, stale, args, bool(getattr(args, "async_ps", 1)))
    B, S = args.batch_per_gpu, args.seq_len
    pool = [mlm_batch(B, S, seed=tp.rank * 1000 + i, device=dev, with_positions=True) for i in range(POOL)]
    it = _cycle(pool)

    def step():
        ids, labels, positions = next(it)
        loss = model(ids, labels, positions)  # LM head on the masked positions only (BERT format)
        loss.backward()
        ps.finish_step()
        return loss

    return Bench(step, B, "sequences/sec (whole node) BERT-base MLM async bounded-staleness s=1", "sequences/s",
                 {"model": "BERT-base", "global_batch": B * tp.world, "seq_len": S,
                  "parallelism": f"ps-ssp{stale}-{'async' if use_async else 'pipelined'}-dp{tp.world}",
                  "optimizer": upd.name, **probe}, ps)


def setup_dlrm(args, tp, dev) -> Bench:
    from .models.dlrm import DLRM, dlrm_batch
    from .parallel.colocated import ColocatedPS
    from .parallel.updaters import AdagradUpdater

    torch.manual_seed(0)
    rows = [args.dlrm_rows] * 26
    model = DLRM(table_rows=rows, transport=tp, device=dev,
                 sparse_updater=AdagradUpdater(0.01, 1e-8, rowwise=True), overlap=True).to(dev)
    # bf16 compute for the MLPs + interaction (fp32 master weights live in the PS shards);
    # embedding tables and their Adagrad state stay fp32, rows are cast inside the gather
    model.bottom.to(torch.bfloat16)
    model.top.to(torch.bfloat16)
    ps = ColocatedPS(model, AdagradUpdater(0.01, 1e-8), tp, bucket_mb=args.bucket_mb,
                     last_bucket_mb=args.last_bucket_mb, plane=getattr(args, "plane", None))
    B = args.batch_per_gpu
    # 4x the usual pool: every step brings new ids, so dedupe, lazy row creation and the row
    # exchange are measured on fresh data rather than on one memorised batch
    pool = [dlrm_batch(B, rows, seed=tp.rank * 1000 + i, device=dev) for i in range(4 * POOL)]
    it = _cycle(pool)
    cur = [next(it)]

    def step():
        dense, sparse, y = cur[0]
        cur[0] = nxt = next(it)
        model.prefetch(nxt[1])  # next batch's id routing runs ahead: its lookup needs no host wait
        loss = F.binary_cross_entropy_with_logits(model(dense, sparse).float(), y)
        loss.backward()  # row gradients leave from the embedding leaf's hook (side stream)
        model.push_sparse()  # flush (no-op when the hook already pushed)
        ps.finish_step()
        return loss

    tbl = model.emb.table
    s0 = {"host_syncs": 0, "pulls": 0}

    def stats():  # host waits of the sparse exchange per timed step (0 = sync-free)
        st = tbl.stats
        d = {"sparse_host_syncs_per_pull": round((st["host_syncs"] - s0["host_syncs"]) / max(1, st["pulls"] - s0["pulls"]), 3)}
        s0.update(host_syncs=st["host_syncs"], pulls=st["pulls"])
        if tbl.plane is not None and tbl.plane.timing:  # row-plane stage table (PS_AMD_ROWPLANE_TIMING=1)
            d["row_plane_stages"] = tbl.plane.timing_summary()
        return d

    return Bench(step, B, "samples/sec (whole node) DLRM sparse push/pull + server row-wise Adagrad", "samples/s",
                 {"model": "DLRM-26x128", "global_batch": B * tp.world, "seq_len": None,
                  "table_rows": args.dlrm_rows, "parallelism": f"ps-bsp-sparse-sharded-dp{tp.world}",
                  "sparse_push_overlap": True,
                  # row exchange path at W > 1: "plane" (IPC arenas, parallel/row_plane.py) or
                  # "collective" (RCCL all-to-alls); "local" at W = 1
                  "sparse_exchange": tbl.exchange, **({"sparse_exchange_info": tbl.exchange_info}
                                                      if tbl.exchange_info else {})}, ps, stats)


def setup_llama_onebit(args, tp, dev) -> Bench:
    from .models.transformer import LlamaConfig, LlamaForCausalLM
    from .parallel.colocated import ColocatedPS
    from .parallel.updaters import AdamUpdater, OneBitAdamUpdater

    cfg = LlamaConfig.tiny() if args.tiny else LlamaConfig.llama3_8b()
    torch.manual_seed(0)
    with torch.device(dev):
        # no activation checkpointing: 4 x 4096 tokens of activations (~26 GB per sequence) +
        # weights/grads (32 GB) + fp32 master/Adam state (96 GB, 1/W of it per rank) fit the 288 GB
        # HBM -- recomputing the forward would cost ~25 % of the step
        model = LlamaForCausalLM(cfg, checkpointing=bool(int(os.environ.get("PS_AMD_LLAMA_CKPT", "0")))).to(
            torch.bfloat16)
    # W > 1: 1-bit Adam -- the workers push their error-compensated 1-bit momentum, the owners
    # freeze the variance after 10 full-precision rounds and refresh it every 4th round (at 8B depth
    # this tracks the uncompressed run; compressed gradients into a live-variance Adam do not:
    # profiles/r6_llama8b_onebit_adam.txt)
    onebit = tp.world > 1
    warm, refresh = 10, 4
    upd = (OneBitAdamUpdater(3e-4, 0.9, 0.95, 1e-8, bias_correction="step", weight_decay=0.1, adamw=True,
                             warmup=warm, refresh=refresh) if onebit
           else AdamUpdater(3e-4, 0.9, 0.95, 1e-8, bias_correction="step", weight_decay=0.1, adamw=True))
    # every bucket's serve overlapped with backward (serving after backward instead was the A/B
    # that priced the serve's HBM traffic stretching backward: profiles/r4_llama_serve_overlap.txt)
    ps = ColocatedPS(model, upd, tp, bucket_mb=max(args.bucket_mb, 64.0), last_bucket_mb=args.last_bucket_mb,
                     compress="onebit" if onebit else None, plane=getattr(args, "plane", None),
                     ef_dtype=torch.bfloat16,  # bf16 error feedback (and momentum): 16 GB each per rank at 8B
                     overlap=True, compress_warmup=warm if onebit else 0, onebit_momentum=0.9 if onebit else None)
    B, S = args.batch_per_gpu, args.seq_len
    g = torch.Generator(device=dev).manual_seed(tp.rank)
    pool = [torch.randint(0, cfg.vocab, (B, S), device=dev, generator=g) for _ in range(POOL)]
    it = _cycle(pool)

    def step():
        ids = next(it)
        loss = model(ids, ids)
        loss.backward()
        ps.finish_step()
        return loss

    return Bench(step, B * S, "tokens/sec (whole node) Llama-3-8B bf16 1-bit compressed push", "tokens/s",
                 {"model": "Llama-3-8B" if not args.tiny else "Llama-tiny", "global_batch": B * tp.world,
                  "seq_len": S, "parallelism": f"ps-bsp-onebit-colocated-dp{tp.world}",
                  "compression": (f"1-bit Adam: 1-bit momentum + error feedback, {warm} full-precision warm-up rounds, "
                                  f"variance refresh every {refresh}th round") if onebit
                  else "none (1 worker: nothing to push)"},
                 ps)


def setup_ctr_async(args, tp, dev) -> Bench:
    """CTR.java:91 / WideDeepNN.java:105-161 shapes on the asynchronous PS (SSP(1) unless
    --staleness says otherwise; rows: parallel/async_rows.py, dense: parallel/async_ps.py)."""
    from .context import ctx
    from .data.dataset import synthetic_ctr
    from .models.reference import WideDeepNN
    from .parallel.async_ps import AsyncPS
    from .parallel.async_rows import async_table_factory

    ctx.init()
    stale = args.staleness if args.staleness else 1
    tf = async_table_factory(tp, dev, seed=7, staleness=stale, capacity=max(1 << 15, args.batch_per_gpu * 24))
    gen = torch.Generator().manual_seed(0)
    model = WideDeepNN.build_model(23, 10, 45, [150, 10, 1], 100000, gen=gen, emb_rows=100000, table_factory=tf,
                                   init_scale=0.2).to(dev)
    ps = AsyncPS(model, model.get_updater(), tp, staleness=stale)  # (a failed remote-write probe raises here)
    B = args.batch_per_gpu
    pool = []
    for i in range(POOL):
        b = synthetic_ctr(B, fields=23, numeric=45, ids_per_field=100000, wide_k=23, wide_size=100000,
                          seed=tp.rank * 1000 + i)
        pool.append({k: v.to(dev) for k, v in b.items()})
    it = _cycle(pool)

    def step():
        b = next(it)
        loss = model.loss(model(b), b["Y"])
        loss.backward()
        model.push_sparse()
        ps.finish_step()
        model.pull_weights()
        return loss

    class _Engine:  # closes the row tables' services, then the dense async PS (collective)
        def close(self):
            for t in model.tables().values():
                t.close()
            ps.close()

    return Bench(step, B, "samples/sec (whole node) CTR Wide&Deep on the asynchronous PS (SSP rows + dense)",
                 "samples/s", {"model": "CTR-WideDeep-23x10", "global_batch": B * tp.world, "seq_len": None,
                               "parallelism": f"ps-ssp{stale}-async-rows-dp{tp.world}",
                               "row_tables": "device-resident (csrc/async_rows_gpu.cpp)" if dev.type == "cuda"
                               else "host callbacks",
                               **{k: v for k, v in ps.info.items() if k == "remote_write_probe"}},
                 _Engine(), dtype="fp32")


SETUPS = {"resnet50": setup_resnet50, "bert-ssp": setup_bert_ssp, "dlrm": setup_dlrm,
          "llama-onebit": setup_llama_onebit, "ctr-async": setup_ctr_async}

DEFAULTS = {  # per-config defaults for --batch-per-gpu / --seq-len when not given
    "resnet50": dict(batch=1024, seq=0),
    # per-GPU batches sized for the 288 GB HBM (weak scaling; profiles/r2_bert_dlrm_batch_sweep.txt):
    # BERT 1024 x 128 (8.41K vs 7.22K seq/s at 256, 45.7 GB peak); DLRM 65536 (12.3M vs 6.9M
    # samples/s at 16384: the per-step sparse exchange / row optimizer cost amortises)
    "bert-ssp": dict(batch=1024, seq=128),
    "dlrm": dict(batch=65536, seq=0),
    # 4 x 4096 tokens per GPU: 215.6 GB peak at world 1 (sized for the 288 GB HBM; the per-step
    # optimizer / PS cost amortises over 4x the tokens): 16.9K vs 15.7K (2 x 4096) and 14.0K tok/s
    # (1 x 4096), profiles/r2_llama_batch_sweep.txt
    "llama-onebit": dict(batch=4, seq=4096),
    "ctr-async": dict(batch=1000, seq=0),  # CTR.java:83-87 training batch
}


# ----------------------------------------------------------------------------- CPU plumbing
def _mlp_worker(wid, port, steps, batch, q):
    import time

    torch.set_num_threads(2)
    from .parallel.kvstore import KVStore
    from .parallel.tcp import PSClient
    from .parallel.updaters import SimpleUpdater

    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(784, 256), torch.nn.ReLU(), torch.nn.Linear(256, 10))
    kv = KVStore(PSClient("127.0.0.1", port), worker_id=wid)
    upd = {"default": SimpleUpdater(0.05)}
    g = torch.Generator().manual_seed(wid)
    x = torch.randn(batch, 784, generator=g)
    y = torch.randint(0, 10, (batch,), generator=g)
    for i in range(steps + 2):
        if i == 2:
            t0 = time.perf_counter()
        kv.pull_into(m)
        m.zero_grad()
        F.cross_entropy(m(x), y).backward()
        kv.sum_from(m)
        kv.update(upd)
        kv.clear()
    q.put((wid, time.perf_counter() - t0))


def run_mlp_tcp(steps: int, batch: int = 128) -> Dict:
    import multiprocessing as mp

    from .parallel.tcp import PServer

    srv = PServer(0, workers=2, mode="bsp").start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_mlp_worker, args=(w, srv.port, steps, batch, q)) for w in range(2)]
    [p.start() for p in ps]
    res = [q.get(timeout=600) for _ in ps]
    [p.join() for p in ps]
    srv.stop()
    el = max(t for _, t in res)
    return {"metric": "samples/sec 2-layer MLP, 1 server + 2 workers on CPU/TCP loopback (plumbing)",
            "value": round(2 * batch * steps / el, 2), "unit": "samples/s", "n_gpus": 0, "steps": steps,
            "ms_per_step": round(el / steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"model": "MLP-784-256-10", "global_batch": 2 * batch, "seq_len": None,
                       "parallelism": "ps-tcp-1server-2workers-bsp"}}
