"""Shared launcher logic for the demo apps: the reference's -D flag semantics
(Context.java:60-88) mapped onto ps_amd engines.

  -Dmode=stand (default)       standalone: one process, local co-located PS
  torchrun (WORLD_SIZE > 1)    co-located PS over RCCL (GPU) / gloo (CPU), BSP or SSP
  -Dmode=dist -Dps=1           dedicated TCP parameter server (native), waits for workers
  -Dmode=dist                  TCP worker of the servers in -DpsAddrs (BSP/SSP/ASP)
"""
from __future__ import annotations

import logging
import os
import sys

import torch

from ..config import Config
from ..context import ctx
from ..parallel.kvstore import KVStore
from ..parallel.tcp import PServer, PSRouterClient
from ..parallel.transport import init_distributed
from ..train.trainer import CollectiveEngine, KVEngine, Trainer

log = logging.getLogger("ps_amd.app")


def setup(argv=None) -> Config:
    cfg = Config.from_args(sys.argv[1:] if argv is None else argv)
    ctx.init(cfg)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(message)s")
    if cfg.metrics_path:
        os.environ["PS_AMD_METRICS_PATH"] = cfg.metrics_path
    if cfg.fault:  # -Dfault=... reaches the engines' FaultInjector (utils/fault.py)
        os.environ["PS_AMD_FAULT"] = cfg.fault
    return cfg


def maybe_run_server(cfg: Config) -> bool:
    """Reference PS branch (CTR.java:73-82): -Dmode=dist -Dps=1 runs a TCP server and blocks."""
    if not (ctx.is_distributed() and cfg.ps):
        return False
    mode = "asp" if cfg.ps_async else cfg.consistency
    srv = PServer(cfg.ps_port, cfg.worker_num, mode, cfg.staleness, bind_any=True).start()
    log.info("PServer on port %d mode=%s workers=%d", srv.port, mode, cfg.worker_num)
    srv.wait()
    srv.stop()
    return True


def connect(cfg: Config, device=None):
    """The parameter-server connection of this process and the matching sparse-table factory:

      -Dmode=dist (TCP workers)      PSRouterClient, rows in the servers' row tables
      torchrun (WORLD_SIZE > 1)      Transport (RCCL / gloo), rows sharded over the ranks
      standalone                     None, rows in local tables

    Models with embedding / wide rows must be built with the returned factory so that their
    rows live on the parameter server (reference: every row is a PS key,
    layer/EmbeddingField.java:57-104, layer/LRLayer.java:62-120)."""
    from ..models.reference import local_table_factory, sharded_table_factory, tcp_table_factory

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if ctx.is_distributed() and world == 1:
        client = PSRouterClient(cfg.ps_addr_list)
        return client, tcp_table_factory(client, device, seed=cfg.seed)
    if world > 1:
        tp = init_distributed(_backend(cfg))
        cons = cfg.effective_consistency
        if cons in ("asp", "ssp"):  # rows reached one-sidedly, no lockstep all-to-alls
            from ..parallel.async_rows import async_table_factory

            return tp, async_table_factory(tp, device, seed=cfg.seed,
                                           staleness=None if cons == "asp" else int(cfg.staleness))
        return tp, sharded_table_factory(tp, device, seed=cfg.seed, overlap=device is not None and
                                         torch.device(device).type == "cuda")
    return None, local_table_factory(device, seed=cfg.seed)


def make_trainer(cfg: Config, model, device=None, conn=None) -> Trainer:
    """Engine for ``model`` over ``conn`` (from ``connect``; created here when omitted)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if ctx.is_distributed() and world == 1:
        client = conn if conn is not None else PSRouterClient(cfg.ps_addr_list)
        wid = int(os.environ.get("PS_AMD_WORKER_ID", os.environ.get("RANK", "0")))
        cons = "asp" if cfg.ps_async else cfg.consistency
        engine = KVEngine(model, KVStore(client, worker_id=wid, consistency=cons))
    else:
        tp = conn if conn is not None else (init_distributed(_backend(cfg)) if world > 1 else None)
        engine = CollectiveEngine(model, tp, bucket_mb=cfg.bucket_mb, staleness=cfg.staleness,
                                  clip_norm=cfg.clip_norm or None, compress=cfg.compress or None,
                                  consistency=cfg.effective_consistency, compress_warmup=cfg.compress_warmup)
        if tp is not None:
            # heartbeat + watchdog on every rank (Config.heartbeat_s): a dead peer ends the job
            # with EXIT_PEER_LOST instead of a hang; ps_amd.launch then restarts it
            from ..utils.fault import start_failure_detection

            start_failure_detection(cfg.heartbeat_s, tp.rank, tp.world)
    return Trainer(model, engine, n_threads=cfg.thread, device=device, checkpoint_dir=cfg.checkpoint_dir,
                   checkpoint_every=cfg.checkpoint_every)


def _backend(cfg: Config):
    """Config.backend: auto (RCCL when a GPU is visible, else gloo) | nccl | gloo."""
    b = (cfg.backend or "auto").lower()
    return None if b in ("auto", "tcp") else b


def worker_rank(cfg: Config, conn=None):
    """(rank, world) of this worker for data sharding (reference Q11: DataSource offset/step are
    never set, so every reference worker reads the same data): torchrun ranks, or the TCP worker
    id (PS_AMD_WORKER_ID / RANK) among -DworkerNum workers."""
    if conn is not None and hasattr(conn, "world"):
        return conn.rank, conn.world
    if ctx.is_distributed():
        wid = int(os.environ.get("PS_AMD_WORKER_ID", os.environ.get("RANK", "0")))
        return wid, max(1, cfg.worker_num)
    return 0, 1


def device() -> torch.device:
    if torch.cuda.is_available():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        return torch.device("cuda", local)
    return torch.device("cpu")
