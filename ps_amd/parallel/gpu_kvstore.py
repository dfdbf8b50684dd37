"""GpuKVStore -- the reference's key-level KVStore API on the MI355X parameter-server engines.

Reference (store/KVStore.java): the whole model layer talks to the store by key --
``get(key, init)`` creates-or-reads (:136-159), ``sum(key, g)`` accumulates a gradient with a
count (:192-200), ``update(Map<prefix, Updater>)`` averages, pushes and meets the servers at the
barrier (:240-268), ``clear()`` drops the per-step state (:270-277), ``asyncGet/asyncWait``
batch-prefetch many keys (:109-127, 279-298); rows of the sparse layers are keys too
(layer/EmbeddingField.java:57-104).  SURVEY §7.1 names the MI355X API
``init(keys) / pull(keys) / push(keys, grads) / pull_rows / push_rows / barrier()``.

Here the same API drives the GPU engines directly, with no ``nn.Module`` in between:

* ``init(specs)``  declares keys (name -> initial tensor, or (shape, dtype) for zeros, or a
  callable).  Declaration is collective and ends at the next data-plane call: the store then
  SEALS the pending keys as one KEY GROUP -- every rank checks that all ranks declared the same
  keys, rank 0's initial values are broadcast, and an engine lays the group out in its flat
  buckets (owner ranges, fp32 masters, optimizer state, plane arenas):
    consistency "bsp" (staleness s >= 0) -> ``ColocatedPS`` (xGMI plane on one node, RCCL
                                            collectives otherwise, gloo on CPU);
    consistency "ssp" / "asp"            -> ``AsyncPS`` (one-sided mailboxes + native owner
                                            threads).
  Keys are registered in declaration order and the engines lay them out in reverse (the
  order gradients become ready in a backward pass), so declare keys in forward order.
  Keys may appear at ANY round (the reference creates a key on its first ``get(key, init)``,
  store/KVStore.java:136-190): keys declared after a group was sealed form the next group, sealed
  by the next data-plane call -- a new engine beside the first, on the same ranks, whose rounds
  ``barrier`` advances together with the others (groups in creation order on every rank).
* ``pull(keys)``   the replica views of the current weight slot (device tensors; valid until
  the next ``barrier``, clone to keep them).  After ``barrier`` the compute stream already
  waits for the round the next forward may see (BSP: the one just pushed; SSP: t - s), so a
  pull costs no host sync and no copy.
* ``push(keys, grads)``  lands each gradient like the engines' backward hooks do: the bucket of
  a key leaves (push -> owner serve -> pull, on the engines' own streams) as soon as its last
  key arrived, so pushes overlap whatever the caller does next.  A key pushed twice in one
  round is summed while its bucket has not left.
* ``barrier()``    ends the round (buckets with keys that were not pushed leave with zeros for
  them, as for parameters that got no gradient) -- ``finish_step`` of the engine.
* ``get(key, init)`` / ``sum`` / ``update`` / ``clear`` / ``async_get`` / ``async_wait`` keep
  the reference semantics on top (``update`` = average the local sums, push, barrier); in
  LOSS_SURFACE_EVAL status ``get`` returns ``s * w_init + (1 - s) * w`` (:153-155).
* ``add_table / pull_rows / push_rows``: row-sparse tables on the same ranks (sparse_table.py
  for BSP, async_rows.py for SSP/ASP).
* ``pull_into(model)`` / ``sum_from(model)``: the model helpers ``train.trainer.KVEngine``
  uses, so the reference apps run on the GPU engines through this API.  Gradients stay on the
  device (no host copies).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Mapping, Optional, Sequence, Tuple, Union

import torch

from ..context import Stat, ctx
from .transport import Transport
from .updaters import Updater

Spec = Union[torch.Tensor, Tuple[Sequence[int], torch.dtype], Callable[[], torch.Tensor]]


class _KeyBank:
    """The engines' view of the declared keys: ``named_parameters()`` in declaration order,
    with the store's key strings (dots included) as names -- per-key-prefix updaters resolve
    on them exactly as on the reference's keys."""

    def __init__(self, params: Dict[str, torch.nn.Parameter]):
        self._p = params

    def named_parameters(self):
        return iter(self._p.items())

    def parameters(self):
        return iter(self._p.values())


class GpuKVStore:
    client = None  # not a TCP worker (Trainer / KVEngine test this)

    def __init__(self, transport: Optional[Transport] = None,
                 updaters: Optional[Union[Updater, Dict[str, Updater]]] = None, *, consistency: str = "bsp",
                 staleness: int = 0, device=None, bucket_mb: float = 25.0, last_bucket_mb: float = 4.0,
                 clip_norm: Optional[float] = None, compress: Optional[str] = None, compress_warmup: int = 0,
                 plane: Optional[str] = None, timeout_s: float = 600.0, average: bool = True):
        if consistency not in ("bsp", "ssp", "asp"):
            raise ValueError(f"unknown consistency {consistency!r}")
        self.t = transport or Transport()
        self.world, self.rank = self.t.world, self.t.rank
        self.consistency = consistency
        self.staleness = int(staleness)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.ps = None  # the first group's engine, once sealed
        self.engines: List[object] = []  # one engine per key group, in creation order
        self._key_engine: Dict[str, object] = {}
        self.umap: Optional[Dict[str, Updater]] = None
        if updaters is not None:
            self.set_updaters(updaters)
        self._kw = dict(bucket_mb=bucket_mb, last_bucket_mb=last_bucket_mb, clip_norm=clip_norm, compress=compress,
                        compress_warmup=compress_warmup, plane=plane, timeout_s=timeout_s, average=average)
        self._decl: Dict[str, torch.Tensor] = {}  # declared initial values (declaration order)
        self._init_host: Dict[str, torch.Tensor] = {}  # w_init for the loss-surface mode
        self.params: Dict[str, torch.nn.Parameter] = {}
        self._sum: Dict[str, torch.Tensor] = {}
        self._cnt: Dict[str, int] = {}
        self._async: List[str] = []
        self.tables: Dict[str, object] = {}
        self.round = 0

    # ------------------------------------------------------------------ configuration
    def set_updaters(self, updaters: Union[Updater, Dict[str, Updater]]) -> None:
        """Per-key-prefix updaters (exact key -> longest prefix -> "default",
        store/KVStore.java:242-252).  Fixed once the store is sealed: the owners' optimizer
        state is laid out per updater segment."""
        umap = dict(updaters) if isinstance(updaters, Mapping) else {"default": updaters}
        if self.ps is not None:
            old = {k: u.name for k, u in self.umap.items()}
            new = {k: u.name for k, u in umap.items()}
            if old != new:
                raise ValueError(f"updaters are fixed once the store is sealed: {old} != {new}")
            return
        self.umap = umap

    @property
    def sealed(self) -> bool:
        return self.ps is not None

    def keys(self) -> List[str]:
        return list(self.params) + [k for k in self._decl if k not in self.params]

    def __contains__(self, key: str) -> bool:
        return key in self.params or key in self._decl

    # ------------------------------------------------------------------ declaration
    def init(self, specs: Mapping[str, Spec]) -> None:
        """Declare keys (collective: every rank declares the same keys, in the same order).
        A key declared again with the same shape and dtype keeps its first value (the
        reference's upsert with replace=false: the first writer wins).  After the first seal,
        new keys wait as the next key group until the next pull / push / barrier seals it."""
        for k, v in specs.items():
            t = self._materialize(v)
            if k in self._decl or k in self.params:
                have = self._decl[k] if k in self._decl else self.params[k]
                if tuple(have.shape) != tuple(t.shape) or have.dtype != t.dtype:
                    raise ValueError(f"key {k!r} re-declared as {tuple(t.shape)} {t.dtype}, "
                                     f"was {tuple(have.shape)} {have.dtype}")
                continue
            self._decl[k] = t

    def _materialize(self, v: Spec) -> torch.Tensor:
        if callable(v) and not isinstance(v, torch.Tensor):
            v = v()
        if isinstance(v, tuple):
            shape, dt = v
            v = torch.zeros(tuple(shape), dtype=dt)
        if not isinstance(v, torch.Tensor):
            raise TypeError("a key spec is a tensor, (shape, dtype) or a callable returning a tensor")
        return v.detach().to(self.device).clone()

    def _seal(self) -> None:
        """Seal the pending keys (collective): the first call builds the first key group's
        engine; keys declared later become further groups, each with an engine of its own."""
        if self.ps is not None and not self._decl:
            return
        if not self._decl:
            raise RuntimeError("GpuKVStore: no keys declared (call init() first)")
        if self.umap is None:
            raise RuntimeError("GpuKVStore: no updaters (pass updaters= or call set_updaters())")
        sig = [(k, tuple(v.shape), str(v.dtype)) for k, v in self._decl.items()]
        sigs = self.t.all_gather_object(sig)
        if any(s != sigs[0] for s in sigs):
            bad = [r for r, s in enumerate(sigs) if s != sigs[0]]
            raise RuntimeError(f"GpuKVStore: ranks {bad} declared different keys than rank 0")
        group = {k: torch.nn.Parameter(v, requires_grad=True) for k, v in self._decl.items()}
        for k, v in self._decl.items():
            self._init_host[k] = v.detach().float().cpu()
        self._decl = {}
        bank = _KeyBank(group)
        kw = self._kw
        if self.consistency == "bsp":
            from .colocated import ColocatedPS

            eng = ColocatedPS(bank, self.umap, self.t, bucket_mb=kw["bucket_mb"],
                              last_bucket_mb=kw["last_bucket_mb"], staleness=self.staleness,
                              clip_norm=kw["clip_norm"], compress=kw["compress"],
                              compress_warmup=kw["compress_warmup"], average=kw["average"], overlap=True,
                              plane=kw["plane"], timeout_s=kw["timeout_s"])
        else:
            from .async_ps import AsyncPS

            if kw["clip_norm"] is not None or kw["compress"] is not None:
                raise ValueError("clipping / compression are BSP-engine options")
            eng = AsyncPS(bank, self.umap, self.t, staleness=None if self.consistency == "asp" else self.staleness,
                          timeout_s=kw["timeout_s"], bucket_mb=kw["bucket_mb"],
                          gscale=None if kw["average"] else 1.0)
        self.engines.append(eng)
        if self.ps is None:
            self.ps = eng
        self.params.update(group)
        for k in group:
            self._key_engine[k] = eng
        # the broadcast of rank 0's values happened inside the engine; the initial values the
        # loss surface interpolates from are the ones every rank now holds
        if self.world > 1:
            for k in group:
                self._init_host[k] = eng.weight(k).detach().float().cpu()

    # ------------------------------------------------------------------ dense keys
    def pull(self, keys: Union[str, Sequence[str]]) -> Union[torch.Tensor, List[torch.Tensor]]:
        """Current weights of ``keys`` (views of this rank's replica; no copy, no host sync)."""
        self._seal()
        if isinstance(keys, str):
            return self.weight(keys)
        return [self.weight(k) for k in keys]

    def weight(self, key: str) -> torch.Tensor:
        if key not in self.params:
            raise KeyError(f"unknown key {key!r}")
        return self._key_engine[key].weight(key)

    def push(self, keys: Union[str, Sequence[str]], grads: Union[torch.Tensor, Sequence[torch.Tensor]]) -> None:
        """Hand gradients of ``keys`` to the engine; a bucket leaves once its last key arrived."""
        self._seal()
        if isinstance(keys, str):
            keys, grads = [keys], [grads]
        if len(keys) != len(grads):
            raise ValueError("push: one gradient per key")
        for k, g in zip(keys, grads):
            if k not in self.params:
                raise KeyError(f"unknown key {k!r}")
            self._key_engine[k].push_key(k, g)

    def barrier(self) -> None:
        """End of the round: every bucket leaves, the PS clock advances and the next pull sees
        the round the consistency mode allows (store/KVStore.java:265, net/PServer.java:238-283)."""
        self._seal()
        for eng in self.engines:  # creation order on every rank: the collectives line up
            eng.finish_step()
        self.round += 1

    def get(self, key: str, init: Optional[Spec] = None) -> Optional[torch.Tensor]:
        """``get(key)``: the current weights or None for an unknown key; ``get(key, init)``
        creates the key first (store/KVStore.java:136-159 -> create :168-190), at any round:
        collective, like ``init`` -- every rank gets the same new key at the same point."""
        if init is not None and key not in self.params and key not in self._decl:
            self.init({key: init})
        if key not in self.params and key not in self._decl:
            return None
        self._seal()
        w = self.weight(key)
        if ctx.status == Stat.LOSS_SURFACE_EVAL:
            s = ctx.weights_scale
            return (self._init_host[key].to(w.device) * s + w.float() * (1 - s)).to(w.dtype)
        return w

    # ---------------------------------------------------------- batched prefetch (reference)
    def async_get(self, key: str, init: Optional[Spec] = None) -> None:
        """Queue a key for ``async_wait`` (store/KVStore.java:109-111).  On the GPU engines a
        pull is already asynchronous -- the replica is written by the engines' pull kernels on
        their own streams and the compute stream waits on them -- so no prefetch thread is
        needed: ``async_wait`` returns the views at once.  ``async_get(key, init)`` creates an
        unknown key at any round, like ``get(key, init)`` (store/KVStore.java:109 -> create)."""
        if init is not None and key not in self.params and key not in self._decl:
            self.init({key: init})
        self._async.append(key)

    def async_wait(self) -> Dict[str, torch.Tensor]:
        keys, self._async = self._async, []
        return {k: self.get(k) for k in keys}

    # ------------------------------------------------------------ local sums (reference)
    def sum(self, key: str, g: torch.Tensor) -> None:
        """Accumulate a local gradient contribution (summed in fp32 on the device, counted)."""
        g = g.detach().to(self.device, torch.float32)
        if key in self._sum:
            self._sum[key].add_(g.reshape(self._sum[key].shape))
            self._cnt[key] += 1
        else:
            self._sum[key] = g.clone()
            self._cnt[key] = 1

    def update(self, updaters: Optional[Union[Updater, Dict[str, Updater]]] = None) -> None:
        """Push the average of every summed key and end the round (store/KVStore.java:240-268)."""
        if updaters is not None:
            self.set_updaters(updaters)
        self._seal()
        sums, cnts = self._sum, self._cnt
        self._sum, self._cnt = {}, {}
        keys = [k for k in sums if k in self.params]
        self.push(keys, [sums[k].div_(cnts[k]) for k in keys])
        self.barrier()

    def clear(self) -> None:
        """Drop local sums and queued prefetches (store/KVStore.java:270-277)."""
        self._sum.clear()
        self._cnt.clear()
        self._async = []

    # ------------------------------------------------------------------ sparse rows
    def add_table(self, name: str, dim: int, rows: Union[int, Sequence[int]], updater: Optional[Updater] = None, *,
                  init: Tuple[float, float] = (0.0, 0.0), id_mode: str = "map", seed: int = 0, fields: int = 1):
        """A row-sparse table on the same ranks (collective).  Rows are created lazily on first
        pull with a deterministic init keyed by the global row key."""
        if name in self.tables:
            raise KeyError(f"table {name!r} exists")
        from .sparse_table import stable_seed

        if self.consistency == "bsp":
            from .sparse_table import ShardedSparseTable

            tab = ShardedSparseTable(name, dim, rows, self.t, updater, init=init, id_mode=id_mode,
                                     seed=stable_seed(name, seed), device=self.device, fields=fields)
        else:
            from .async_rows import AsyncRowTable

            tab = AsyncRowTable(name, dim, rows, self.t, updater, init=init, id_mode=id_mode,
                                seed=stable_seed(name, seed), device=self.device, fields=fields,
                                staleness=None if self.consistency == "asp" else self.staleness)
        self.tables[name] = tab
        return tab

    def pull_rows(self, table: str, ids: torch.Tensor) -> torch.Tensor:
        """Rows of ``ids`` from their owners ([n, dim]; [..., fields, dim] for multi-field)."""
        return self.tables[table].pull(ids)

    def push_rows(self, table: str, ids: torch.Tensor, grads: torch.Tensor) -> None:
        """Per-id gradient rows to their owners (duplicates summed, one update per row)."""
        self.tables[table].push(ids, grads)

    # ------------------------------------------------------------------ model helpers
    def pull_into(self, model: torch.nn.Module, init: Optional[Dict[str, Spec]] = None) -> None:
        """Bind every trainable parameter of ``model`` to its key's replica view (declaring the
        keys from the model's current values -- or ``init`` -- on first use)."""
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        if not self.sealed:
            self.init({n: (init[n] if init and n in init else p.detach()) for n, p in named})
        self._seal()
        with torch.no_grad():
            for n, p in named:
                w = self.weight(n)
                if w.shape == p.shape and w.dtype == p.dtype and w.device == p.device:
                    p.data = w
                else:
                    p.data = w.detach().to(p.device, p.dtype).reshape(p.shape).clone()

    def sum_from(self, model: torch.nn.Module) -> None:
        for n, p in model.named_parameters():
            if p.grad is not None:
                self.sum(n, p.grad)

    # ------------------------------------------------------------------ lifecycle
    def synchronize(self, collective: bool = False) -> None:
        """Drain every engine.  ``collective=True`` (every rank calls it, e.g. before reading the
        final weights): the asynchronous engine's replicas then also hold every OTHER worker's
        pushes, not just this rank's."""
        for eng in self.engines:
            if collective and getattr(eng, "info", {}).get("engine") == "AsyncPS":
                eng.synchronize(collective=True)
            else:
                eng.synchronize()
        for t in self.tables.values():
            t.synchronize()

    def shard_state(self) -> dict:
        """This rank's server state: the engine's for one key group, ``{"groups": [...]}`` for more."""
        if len(self.engines) == 1:
            return self.ps.shard_state()
        return {"groups": [e.shard_state() for e in self.engines]}

    def load_shard_state(self, st: dict) -> None:
        self._seal()
        if "groups" in st:
            if len(st["groups"]) != len(self.engines):
                raise ValueError(f"checkpoint has {len(st['groups'])} key groups, the store {len(self.engines)}")
            for e, s in zip(self.engines, st["groups"]):
                e.load_shard_state(s)
        else:
            self.ps.load_shard_state(st)

    def stats(self) -> dict:
        d = {"round": self.round, "keys": len(self.keys()), "engine": type(self.ps).__name__ if self.ps else None,
             "groups": len(self.engines)}
        if self.ps is not None and hasattr(self.ps, "plane_stats"):
            d["plane"] = self.ps.plane_stats()
            d["plane_kind"] = self.ps.plane_kind
        return d

    def close(self) -> None:
        for t in self.tables.values():
            if hasattr(t, "close"):
                t.close()
        self.tables = {}
        for eng in self.engines:
            eng.close()
        self.engines = []
        self._key_engine = {}
        self.ps = None
