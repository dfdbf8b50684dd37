"""Collective bandwidth probe over the job's own process group (RCCL over xGMI on MI355X).

Measures the three collectives the co-located PS issues -- reduce-scatter (push), all-gather
(pull) and all-reduce (clip norm / dense fallback) -- at PS-bucket-like sizes, plus the DIRECT
one-shot forms of the first two (all-to-all over every peer link at once, owner-side sum: the
ring-vs-direct comparison SURVEY §2.4 asks for on 7 point-to-point xGMI links), and reports
nccl-tests style algorithm / bus bandwidth (busbw = algbw * (n-1)/n for RS / AG, 2(n-1)/n for
AR) with the time taken as the MAX over ranks.  bench.py runs it after the timed region at
world > 1 so the driver's multi-GPU runs carry a measured xGMI collective curve next to the
throughput number (bucket size is chosen against this curve: 7 point-to-point
links per GPU make ring collectives per-link bound, so small buckets sit on the latency floor).

    from ps_amd.parallel.comm_probe import probe
    probe(device, sizes_mb=(4, 25, 100))  -> {"reduce_scatter": {"25MB": {"algbw_GBps": ..}}, ...}
"""
from __future__ import annotations

import time
from typing import Dict, Sequence

import torch
import torch.distributed as dist


def _sync(dev: torch.device) -> None:
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _timed(fn, iters: int, dev: torch.device) -> float:
    fn()
    _sync(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    _sync(dev)
    el = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64, device=dev)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return float(el.item())


def probe(dev: torch.device, sizes_mb: Sequence[float] = (4, 25, 100), iters: int = 10,
          dtype: torch.dtype = torch.bfloat16) -> Dict[str, Dict[str, Dict[str, float]]]:
    """Per collective and size (MB of the full tensor): time in us, algbw and busbw in GB/s."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return {}
    n = dist.get_world_size()
    es = torch.tensor([], dtype=dtype).element_size()
    out: Dict[str, Dict[str, Dict[str, float]]] = {"reduce_scatter": {}, "all_gather": {}, "all_reduce": {},
                                                   "reduce_scatter_direct": {}, "all_gather_direct": {}}
    for mb in sizes_mb:
        numel = int(mb * 2**20 / es) // n * n
        full = torch.zeros(numel, dtype=dtype, device=dev)
        shard = torch.empty(numel // n, dtype=dtype, device=dev)
        recv = torch.empty(n, numel // n, dtype=dtype, device=dev)
        rep = torch.zeros(n, numel // n, dtype=dtype, device=dev)
        nbytes = numel * es

        def rs_direct():  # one-shot: slice j straight to owner j over its own link, owner sums W slices
            dist.all_to_all_single(recv.view(-1), full)
            torch.sum(recv, dim=0, out=shard)

        def ag_direct():  # one-shot: the owned slice to every peer at once
            dist.all_to_all_single(full, rep.view(-1))

        cases = {
            "reduce_scatter": (lambda: dist.reduce_scatter_tensor(shard, full), (n - 1) / n),
            "all_gather": (lambda: dist.all_gather_into_tensor(full, shard), (n - 1) / n),
            "all_reduce": (lambda: dist.all_reduce(full), 2 * (n - 1) / n),
            "reduce_scatter_direct": (rs_direct, (n - 1) / n),
            "all_gather_direct": (ag_direct, (n - 1) / n),
        }
        for name, (fn, fac) in cases.items():
            t = _timed(fn, iters, dev)
            algbw = nbytes / t / 1e9
            out[name][f"{mb:g}MB"] = {"us": round(t * 1e6, 1), "algbw_GBps": round(algbw, 1),
                                      "busbw_GBps": round(algbw * fac, 1)}
        del full, shard, recv, rep
    return out
