"""KVStore -- the reference's parameter-store API (store/KVStore.java), two backends.

* standalone (no client): the in-process parameter table.  ``get(key, init)`` creates a key
  lazily from its init callable (:136-159), ``sum(key, g)`` accumulates gradients with a count
  (:192-200), ``update(updaters)`` applies the AVERAGED gradient with the per-key updater
  resolved exact -> longest prefix -> "default" (:240-268), ``clear()`` drops the sums.
  In LOSS_SURFACE_EVAL status ``get`` returns s*w_init + (1-s)*w (:153-155).
* distributed worker (``client`` = PSClient / PSRouterClient over the native TCP server):
  ``get`` is a per-step cache in front of the servers; a missing key is created with
  upsert(replace=False) so the first writer wins (:168-190); ``async_get`` queues keys for a
  prefetch thread (started on first use, :54-68, 279-298) that fetches everything queued in
  ONE get_list + ONE upsert_list per shard while the caller goes on (:74-107), and
  ``async_wait`` blocks until every key queued so far is in the cache (:113-127); ``update`` pushes every summed key grouped by updater spec (one
  request per shard per spec instead of one RPC per key) and then meets the servers at the
  consistency point (BSP barrier / SSP clock / nothing for ASP); ``clear`` drops the cache.

The GPU engines have their own key-level store with the same API (gpu_kvstore.py: pulls
are replica views, sums stay on the device).
"""
from __future__ import annotations

import threading
from typing import Callable, Dict, Optional, Union

import torch

from ..context import Stat, ctx
from ..obs import trace as _trace
from .updaters import Updater, resolve_updater

Init = Callable[[], torch.Tensor]


class KVStore:
    _ins: Optional["KVStore"] = None

    @classmethod
    def ins(cls) -> "KVStore":
        if cls._ins is None:
            cls._ins = KVStore()
        return cls._ins

    @classmethod
    def reset(cls, store: Optional["KVStore"] = None) -> None:
        cls._ins = store

    def __init__(self, client=None, worker_id: int = 0, consistency: str = "bsp"):
        self.client = client
        self.worker_id = worker_id
        self.consistency = consistency
        self.store: Dict[str, torch.Tensor] = {}
        self.store_init: Dict[str, torch.Tensor] = {}
        self._sum: Dict[str, torch.Tensor] = {}
        self._cnt: Dict[str, int] = {}
        self._async: Dict[str, Init] = {}
        self._lock = threading.RLock()
        # prefetch thread (reference KVStore.run, :279-298): queued batches -> one batched fetch
        self._pf_cv = threading.Condition()
        self._pf_queue: list = []
        self._pf_done = 0
        self._pf_sent = 0
        self._gen = 0  # cache generation: clear() starts a new one; stale prefetches are dropped
        self._pf_err: Optional[BaseException] = None
        self._pf_thread: Optional[threading.Thread] = None
        self.prefetch_batches = 0
        self.clock = 0
        self.round = 0
        self._fault = None  # lazily built FaultInjector (PS_AMD_FAULT); False = none configured

    @property
    def distributed(self) -> bool:
        return self.client is not None

    # ------------------------------------------------------------------ get / create
    def get(self, key: str, init: Optional[Init] = None) -> Optional[torch.Tensor]:
        with self._lock:
            if key in self.store:
                w = self.store[key]
                if not self.distributed and ctx.status == Stat.LOSS_SURFACE_EVAL and key in self.store_init:
                    s = ctx.weights_scale
                    return self.store_init[key] * s + w * (1 - s)
                return w
            if self.distributed:
                m = self.client.get(key)
                if m is None and init is not None:
                    m = self.client.update(key, init(), replace=False)
                if m is not None:
                    self.store[key] = m.reshape(m.shape)
                return m
            if init is None:
                return None
            return self._create(key, init)

    def _create(self, key: str, init: Init) -> torch.Tensor:
        m = init().float()
        self.store[key] = m
        self.store_init[key] = m.clone()
        return m

    def put(self, key: str, val: torch.Tensor) -> None:
        if self.distributed:
            raise RuntimeError("KVStore.put is a server-side operation (reference :161-166)")
        with self._lock:
            self.store[key] = val

    # ------------------------------------------------------------------ batch prefetch
    def async_get(self, key: str, init: Init) -> None:
        """Queue ``key`` for the prefetch thread (store/KVStore.java:109-111); returns at once.
        Keys queued before the next ``async_wait`` go out as one batch."""
        with self._lock:
            if key not in self.store:
                self._async[key] = init

    def async_wait(self) -> None:
        """Hand the queued keys to the prefetch thread and wait until every key queued so far
        is in the cache (store/KVStore.java:113-127)."""
        with self._lock:
            pending = {k: f for k, f in self._async.items() if k not in self.store}
            self._async.clear()
        if pending and not self.distributed:
            with self._lock:
                for k, f in pending.items():
                    if k not in self.store:
                        self._create(k, f)
            return
        if pending:
            self.prefetch(pending)
        with self._pf_cv:
            target = self._pf_sent
            while self._pf_done < target and self._pf_err is None:
                self._pf_cv.wait(timeout=1.0)
            if self._pf_err is not None:
                err, self._pf_err = self._pf_err, None
                raise RuntimeError("KVStore prefetch failed") from err

    def prefetch(self, keys: Dict[str, Init]) -> None:
        """Start fetching ``keys`` (key -> init) on the prefetch thread without waiting."""
        if not self.distributed or not keys:
            return
        with self._pf_cv:
            if self._pf_thread is None:
                self._pf_thread = threading.Thread(target=self._prefetch_loop, name="kvstore-prefetch", daemon=True)
                self._pf_thread.start()
            self._pf_queue.append((self._gen, dict(keys)))
            self._pf_sent += 1
            self._pf_cv.notify_all()

    def _prefetch_loop(self) -> None:
        while True:
            with self._pf_cv:
                while not self._pf_queue:
                    self._pf_cv.wait()
                gen, batch = self._pf_queue.pop(0)
            try:
                with self._lock:
                    batch = {k: f for k, f in batch.items() if k not in self.store} if gen == self._gen else {}
                if batch:
                    got = self.client.get_list(list(batch))
                    missing = {k: batch[k]() for k, v in got.items() if v is None}
                    created = self.client.update_list(missing, replace=False) if missing else {}
                    with self._lock:
                        # a clear() since this batch was queued dropped the generation it belongs
                        # to: its values may predate the round that clear() ended -- never cache
                        # them (the next pull re-fetches post-barrier values)
                        if gen == self._gen:
                            for k, v in got.items():
                                self.store[k] = v if v is not None else created[k]
                self.prefetch_batches += 1
            except BaseException as e:  # noqa: BLE001 -- surfaced by async_wait
                with self._pf_cv:
                    self._pf_err = e
            with self._pf_cv:
                self._pf_done += 1
                self._pf_cv.notify_all()

    # ------------------------------------------------------------------ gradients
    def sum(self, key: str, g: torch.Tensor) -> None:
        g = g.detach().float()
        with self._lock:
            if key in self._sum:
                self._sum[key] += g.reshape(self._sum[key].shape)
                self._cnt[key] += 1
            else:
                self._sum[key] = g.clone()
                self._cnt[key] = 1

    def update(self, updaters: Union[Updater, Dict[str, Updater]]) -> None:
        """Apply (standalone) or push (distributed) every summed key, then the consistency
        point.  Gradients are averaged over the local contributions (reference :253)."""
        umap = updaters if isinstance(updaters, dict) else {"default": updaters}
        with self._lock:
            avg = {k: self._sum[k] / self._cnt[k] for k in self._sum}
        if not self.distributed:
            with self._lock:
                for k, g in avg.items():
                    resolve_updater(k, umap).update(k, self.store[k], g)
            self.round += 1
            return
        groups: Dict[str, Dict[str, torch.Tensor]] = {}
        for k, g in avg.items():
            groups.setdefault(resolve_updater(k, umap).name, {})[k] = g
        if self._fault is None:
            from ..utils.fault import FaultInjector

            fi = FaultInjector(rank=self.worker_id)
            self._fault = fi if fi.spec else False
        for spec, grads in groups.items():
            if self._fault:
                self._fault.before_push()
                if self.consistency == "asp" and self._fault.drop():  # lost push (ASP only)
                    continue
            self.client.push(grads, spec)
        if self._fault:
            self._fault.at_step(self.round)
        self.round += 1
        self.clock += 1
        with _trace.range(f"kv.{self.consistency}.wait"):
            if self.consistency == "bsp":
                self.client.barrier(self.worker_id)
            elif self.consistency == "ssp":
                self.client.clock(self.worker_id, self.clock)

    def barrier(self) -> None:
        if self.distributed:
            self.client.barrier(self.worker_id)

    def clear(self, prefetch: bool = True) -> None:
        """Drop the local sums and (worker) the per-step weight cache (store/KVStore.java:270-277).
        A worker then starts re-fetching the keys it just dropped on the prefetch thread, so the
        next step's pull finds them in flight or already cached (their values are post-barrier)."""
        with self._lock:
            self._sum.clear()
            self._cnt.clear()
            dropped = list(self.store) if self.distributed else []
            if self.distributed:
                self.store.clear()  # per-step worker cache: next step re-pulls (Q16)
                self._gen += 1  # in-flight prefetches of the previous generation are discarded
        if dropped and prefetch:
            self.prefetch({k: _no_init(k) for k in dropped})

    # ------------------------------------------------------------------ model helpers
    def pull_into(self, model: torch.nn.Module, init: Optional[Dict[str, Init]] = None) -> None:
        """Copy every parameter of ``model`` from the store (creating keys from the model's
        current values on first use -- the reference's init callables)."""
        params = dict(model.named_parameters())
        if self.distributed:
            for n, p in params.items():
                if n not in self.store:
                    self.async_get(n, (init or {}).get(n, (lambda t=p: t.detach().float().cpu().clone())))
            self.async_wait()
        with torch.no_grad():
            for n, p in params.items():
                w = self.get(n, (init or {}).get(n, (lambda t=p: t.detach().float().cpu().clone())))
                p.copy_(w.reshape(p.shape).to(p.device, p.dtype))

    def sum_from(self, model: torch.nn.Module) -> None:
        for n, p in model.named_parameters():
            if p.grad is not None:
                self.sum(n, p.grad.cpu())


def _no_init(key: str) -> Init:
    def f():
        raise KeyError(f"prefetched key {key!r} vanished from the servers")
    return f
