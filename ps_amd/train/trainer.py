"""Training runtime (train/Trainer.java, TrainerThread.java, PredictThread.java).

The reference runs ``nThreads`` model replicas on a CPU thread pool, averages their
gradients in the shared KVStore and applies one optimizer step per round
(Trainer.java:70-101).  On a GPU the replicas become micro-batches accumulated into the
same gradient buckets (identical math: the average of the replica gradients), followed by
ONE parameter-server round.  Engines:

  CollectiveEngine  co-located PS over RCCL/gloo collectives (colocated.py) for dense keys
                    + sharded sparse tables; BSP or SSP(s).  The MI355X path.
  KVEngine          the reference KVStore API: standalone in-process store, or a worker of
                    dedicated TCP servers (tcp.py) -- pull before the step, sum + push +
                    barrier/clock after it.

``Trainer.train(batches)`` returns the mean loss; failures of a replica are counted as the
reference does (loss 0 + log) only when ``tolerate_failures`` is set -- by default they
raise.  Per-step timings (fwd+bwd, push/update, exposed wait) go to the metrics stream.

Checkpoint / resume: with ``checkpoint_dir`` every ``checkpoint_every`` rounds
each rank writes its server shard (dense master + optimizer state, sparse rows + id map) and
the step counter (utils/checkpoint.py, committed once all ranks are on disk); ``resume()``
restores the newest committed step.  The TCP topology asks the servers to save instead.
"""
from __future__ import annotations

import logging
import time
from typing import Dict, List, Optional, Sequence

import torch

from ..context import Stat, ctx
from ..obs import metrics as _metrics
from ..parallel.colocated import ColocatedPS
from ..parallel.kvstore import KVStore
from ..parallel.transport import Transport

log = logging.getLogger("ps_amd.trainer")


def _to(batch: Dict[str, torch.Tensor], device) -> Dict[str, torch.Tensor]:
    return {k: (v.to(device, non_blocking=True) if isinstance(v, torch.Tensor) else v) for k, v in batch.items()}


class CollectiveEngine:
    def __init__(self, model, transport: Optional[Transport] = None, *, bucket_mb: float = 25.0,
                 staleness: int = 0, clip_norm: Optional[float] = None, compress: Optional[str] = None,
                 overlap: bool = True, consistency: str = "bsp", compress_warmup: int = 0):
        """``consistency``: "bsp" (collective rounds; ``staleness`` > 0 pipelines them with the
        bound enforced by the collective), "ssp" / "asp" (parallel/async_ps.py: one-sided pushes
        into owner mailboxes, native progress threads, SSP(staleness) gate or none)."""
        self.model = model
        self.t = transport or Transport()
        dense = [p for p in model.parameters() if p.requires_grad]
        self.consistency = consistency
        if not dense:
            self.ps = None
        elif consistency in ("ssp", "asp"):
            from ..parallel.async_ps import AsyncPS

            self.ps = AsyncPS(model, model.get_updater(), self.t,
                              staleness=None if consistency == "asp" else int(staleness))
        else:
            self.ps = ColocatedPS(model, model.get_updater(), self.t, bucket_mb=bucket_mb, staleness=staleness,
                                  clip_norm=clip_norm, compress=compress, overlap=overlap,
                                  compress_warmup=compress_warmup)

    def accumulate(self, on: bool) -> None:
        if self.ps is not None:
            self.ps.accumulating = on
        if hasattr(self.model, "set_accumulating"):  # sparse rows: one owner step per round
            self.model.set_accumulating(on)

    def end_step(self) -> None:
        self.model.push_sparse()
        if self.ps is not None:
            self.ps.finish_step()

    def pull(self) -> None:
        self.model.pull_weights()

    def synchronize(self) -> None:
        if self.ps is not None:
            self.ps.synchronize()


class KVEngine:
    """The reference's per-step KVStore protocol (train/Trainer.java:70-101): pull the weights,
    train, ``sum`` every gradient, ``update`` (average + push + barrier), ``clear``.  ``store`` is
    the CPU ``KVStore`` (standalone or TCP worker) or the GPU engines' ``GpuKVStore``
    (parallel/gpu_kvstore.py), whose pulls bind the parameters to the replica and whose sums
    stay on the device."""

    def __init__(self, model, store=None):
        self.model = model
        self.kv = store or KVStore.ins()
        if getattr(self.kv, "umap", "n/a") is None:  # GpuKVStore without updaters yet
            self.kv.set_updaters(model.get_updater())

    @property
    def ps(self):
        return getattr(self.kv, "ps", None)

    @property
    def t(self):
        return getattr(self.kv, "t", None)

    @property
    def gpu_store(self) -> bool:
        return not isinstance(self.kv, KVStore)

    def accumulate(self, on: bool) -> None:
        pass

    def pull(self) -> None:
        self.model.pull_weights()
        self.kv.pull_into(self.model)

    def end_step(self) -> None:
        self.kv.sum_from(self.model)
        for p in self.model.parameters():
            p.grad = None
        self.model.push_sparse()
        self.kv.update(self.model.get_updater())
        self.kv.clear()

    def synchronize(self) -> None:
        if self.gpu_store:
            self.kv.synchronize()


class Trainer:
    def __init__(self, model, engine=None, n_threads: int = 1, device=None, tolerate_failures: bool = False,
                 checkpoint_dir: str = "", checkpoint_every: int = 0):
        self.model = model
        self.engine = engine or KVEngine(model)
        self.n_threads = max(1, int(n_threads))
        self.device = device
        self.tolerate_failures = tolerate_failures
        self.last_timing: Dict[str, float] = {}
        self.ckpt = None
        self.checkpoint_every = int(checkpoint_every)
        if checkpoint_dir:
            from ..utils.checkpoint import CheckpointManager

            t = getattr(self.engine, "t", None)
            rank, world = (t.rank, t.world) if t is not None else (0, 1)
            self.ckpt = CheckpointManager(checkpoint_dir, rank=rank, world=world)

    # ------------------------------------------------------------------ checkpoint
    def _tables(self) -> dict:
        return self.model.tables() if hasattr(self.model, "tables") else {}

    def save(self, step: int, extra: Optional[dict] = None, blocking: bool = False) -> None:
        if self.ckpt is None:
            return
        if isinstance(self.engine, KVEngine) and not self.engine.gpu_store:
            # dedicated TCP servers hold the whole model: worker 0 asks every server to write its
            # store, then marks the step COMMITTED (resume() only trusts committed steps)
            if self.engine.kv.client is not None and self.engine.kv.worker_id == 0:
                import os

                d = os.path.join(self.ckpt.dir, f"tcp_step{step:08d}")
                os.makedirs(d, exist_ok=True)
                self.engine.kv.client.save(os.path.join(d, "server"))
                with open(os.path.join(d, "COMMIT"), "w") as f:
                    f.write(str(step))
            return
        self.engine.synchronize()
        self.ckpt.save(step, getattr(self.engine, "ps", None), self._tables(), extra={"step": step, **(extra or {})},
                       blocking=blocking)

    def _tcp_latest(self) -> Optional[str]:
        import os

        if self.ckpt is None or not os.path.isdir(self.ckpt.dir):
            return None
        done = sorted(d for d in os.listdir(self.ckpt.dir)
                      if d.startswith("tcp_step") and os.path.exists(os.path.join(self.ckpt.dir, d, "COMMIT")))
        return os.path.join(self.ckpt.dir, done[-1]) if done else None

    def resume(self) -> int:
        """Restore the newest committed checkpoint (if any); returns the step to continue from.

        TCP topology: all workers rendezvous on the servers, worker 0 has every server reload its
        store from the newest committed ``tcp_step*`` directory, all rendezvous again, and every
        worker continues from that step."""
        if self.ckpt is None:
            return 0
        if isinstance(self.engine, KVEngine) and not self.engine.gpu_store:
            import os

            d = self._tcp_latest()
            if d is None:
                return 0
            client = self.engine.kv.client
            if client is not None:
                # every worker is present before worker 0 reloads and waits until the reload is
                # done: nobody pulls pre-restore weights or pushes a gradient the reload drops
                client.rendezvous(self.engine.kv.worker_id)
                if self.engine.kv.worker_id == 0:
                    client.load(os.path.join(d, "server"))
                client.rendezvous(self.engine.kv.worker_id)
            step = int(os.path.basename(d)[len("tcp_step"):])
            ctx.set_step(step)
            return step
        if self.ckpt.latest() is None:
            return 0
        st = self.ckpt.load(None, getattr(self.engine, "ps", None), self._tables())
        step = int(st.get("extra", {}).get("step", st["step"]))
        ctx.set_step(step)
        return step

    def _dev(self, b):
        return _to(b, self.device) if self.device is not None else b

    def train(self, batches: Sequence[Dict[str, torch.Tensor]]) -> float:
        """One PS round over up to ``n_threads`` micro-batches (Trainer.java:70-101)."""
        ctx.status = Stat.TRAINING
        batches = list(batches)[: self.n_threads] if self.n_threads > 1 else list(batches)[:1]
        if not batches:
            raise ValueError("no batches")
        t0 = time.perf_counter()
        self.engine.pull()
        losses = []
        for i, b in enumerate(batches):
            ctx.model_index = i
            self.engine.accumulate(i < len(batches) - 1)
            try:
                losses.append(self.model.train_batch(self._dev(b), scale=1.0 / len(batches)))
            except Exception:
                if not self.tolerate_failures:
                    raise
                log.exception("replica %d failed; counting loss 0 (reference TrainerThread.java:36-38)", i)
                losses.append(0.0)
        ctx.model_index = 0
        t1 = time.perf_counter()
        self.engine.end_step()
        t2 = time.perf_counter()
        loss = sum(losses) / len(losses)
        step = ctx.incr_step()
        _metrics.plot("loss", loss, step)
        self.last_timing = {"fwd_bwd_ms": (t1 - t0) * 1e3, "ps_round_ms": (t2 - t1) * 1e3}
        _metrics.log_step(step=step, loss=loss, **self.last_timing)
        if self.ckpt is not None and self.checkpoint_every and step % self.checkpoint_every == 0:
            self.save(step)
        return loss

    def predict(self, batches: Sequence[Dict[str, torch.Tensor]]) -> List[torch.Tensor]:
        """Forward only (Trainer.java:44-68 / PredictThread)."""
        prev = ctx.status
        if prev == Stat.TRAINING:
            ctx.status = Stat.PREDICTING
        self.engine.synchronize()
        out = []
        for b in batches:
            out.append(self.model.predict(self._dev(b)))
            self.model.pull_weights()  # drop sparse leaves created by the forward
        ctx.status = prev
        return out
