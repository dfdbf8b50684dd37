"""KVStore -- the reference's parameter-store API (store/KVStore.java), two backends.

* standalone (no client): the in-process parameter table.  ``get(key, init)`` creates a key
  lazily from its init callable (:136-159), ``sum(key, g)`` accumulates gradients with a count
  (:192-200), ``update(updaters)`` applies the AVERAGED gradient with the per-key updater
  resolved exact -> longest prefix -> "default" (:240-268), ``clear()`` drops the sums.
  In LOSS_SURFACE_EVAL status ``get`` returns s*w_init + (1-s)*w (:153-155).
* distributed worker (``client`` = PSClient / PSRouterClient over the native TCP server):
  ``get`` is a per-step cache in front of the servers; a missing key is created with
  upsert(replace=False) so the first writer wins (:168-190); ``async_get``/``async_wait``
  batch-prefetch many keys in ONE get_list + ONE upsert_list per shard on a background
  thread (:74-127, 279-298); ``update`` pushes every summed key grouped by updater spec (one
  request per shard per spec instead of one RPC per key) and then meets the servers at the
  consistency point (BSP barrier / SSP clock / nothing for ASP); ``clear`` drops the cache.

The GPU hot path does not go through this class: it uses the co-located collective PS
(colocated.py) and sharded sparse tables (sparse_table.py).
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
        with self._lock:
            self._async[key] = init

    def async_wait(self) -> None:
        """Fetch every key registered with async_get in one batched round trip."""
        with self._lock:
            pending = {k: f for k, f in self._async.items() if k not in self.store}
            self._async.clear()
        if not pending:
            return
        if not self.distributed:
            with self._lock:
                for k, f in pending.items():
                    if k not in self.store:
                        self._create(k, f)
            return
        got = self.client.get_list(list(pending))
        missing = {k: pending[k]() for k, v in got.items() if v is None}
        created = self.client.update_list(missing, replace=False) if missing else {}
        with self._lock:
            for k, v in got.items():
                self.store[k] = v if v is not None else created[k]

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

    def clear(self) -> None:
        with self._lock:
            self._sum.clear()
            self._cnt.clear()
            if self.distributed:
                self.store.clear()  # per-step worker cache: next step re-pulls (Q16)

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
