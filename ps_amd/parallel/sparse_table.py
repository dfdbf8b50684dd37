"""Row-sparse parameter tables: embeddings and wide (LR) weights.

Reference: one PS key per row -- ``"<field>.<id>"`` embedding rows (layer/EmbeddingField.java)
and ``"wide.weights.<id>"`` 1x1 wide weights (layer/LRLayer.java) -- pulled with getList
fan-out (store/KVStore.java:74-127), created lazily on first touch by an
upsert(replace=false) round trip (net/PServer.java:143-162) and pushed one RPC per row
(store/KVStore.java:259).

Here a table is a dense fp32 [rows, dim] array (plus per-row "initialised" flags and
optimizer state) held by the server that owns those rows:

* ``SparseTable``          one owner (standalone, or the local shard of a sharded table).
* ``ShardedSparseTable``   rows partitioned over W co-located servers.  pull: dedupe ->
  all_to_all(ids) -> owner gathers (lazy-init HIP kernel) -> all_to_all(rows).  push:
  dedupe + segment-reduce (HIP) -> all_to_all(ids, grads) -> owner reduces duplicates from
  different workers -> fused row-sparse optimizer (HIP).  Sizes move in a count exchange
  first (all_to_all of W int64s).

Id modes: ``direct`` (ids are row numbers, DLRM-style), ``hash`` (id mod rows, the wide
hashing of util/MatrixUtil.java:27-33), ``map`` (exact id -> slot assignment on first
touch through the native IdMap -- the reference's unbounded string keys, Q17 fixed by int64
ids).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from ..ops import sparse as _sp
from .transport import Transport
from .updaters import Updater


def _mix64(x: torch.Tensor) -> torch.Tensor:
    """splitmix-style avalanche on int64 (works on CPU and GPU; wraps like uint64)."""
    x = x.long()
    x = (x ^ (x >> 31)) * 0x7FB5D329728EA185
    x = (x ^ (x >> 27)) * -0x7E25210B43D22E0B  # 0x81DADEF4BC2DD44D as signed
    return x ^ (x >> 33)


class IdMap:
    """Exact id -> slot map with lazy slot allocation (host side)."""

    def __init__(self, capacity: int):
        self.capacity = capacity
        try:
            from .. import _native  # type: ignore

            self._m = _native.IdMap(capacity)
        except Exception:
            self._m = None
            self._d = {}

    def lookup(self, ids: torch.Tensor, insert: bool = True) -> torch.Tensor:
        ids_c = ids.detach().cpu().long().contiguous()
        if self._m is not None:
            out = torch.from_numpy(self._m.lookup(ids_c.numpy(), insert))
        else:
            res = []
            for v in ids_c.tolist():
                s = self._d.get(v)
                if s is None:
                    if not insert or len(self._d) >= self.capacity:
                        s = -1
                    else:
                        s = len(self._d)
                        self._d[v] = s
                res.append(s)
            out = torch.tensor(res, dtype=torch.int64)
        if (out < 0).any():
            raise RuntimeError(f"IdMap capacity {self.capacity} exhausted")
        return out.to(ids.device)

    def __len__(self):
        return self._m.size() if self._m is not None else len(self._d)


class SparseTable:
    def __init__(self, name: str, dim: int, rows: int, updater: Optional[Updater] = None, *,
                 init: Tuple[float, float] = (0.0, 0.0), id_mode: str = "direct", seed: int = 0,
                 row_base: int = 0, device=None):
        self.name, self.dim, self.rows = name, int(dim), int(rows)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.table = torch.zeros(self.rows, self.dim, dtype=torch.float32, device=self.device)
        self.flags = torch.zeros(self.rows, dtype=torch.uint8, device=self.device)
        self.init = init
        self.seed = int(seed)
        self.row_base = int(row_base)
        if id_mode not in ("direct", "hash", "map"):
            raise ValueError(id_mode)
        self.id_mode = id_mode
        self.idmap = IdMap(self.rows) if id_mode == "map" else None
        self.updater = updater
        self.states: List[torch.Tensor] = []
        if updater is not None:
            self._alloc_states()
        self.round = 0

    def _alloc_states(self):
        u = self.updater
        rowwise = getattr(u, "rowwise", False)
        if rowwise:
            self.states = [torch.zeros(self.rows, dtype=torch.float32, device=self.device)]
        else:
            self.states = [torch.zeros_like(self.table) for _ in range(u.n_state)]

    def set_updater(self, u: Updater):
        self.updater = u
        self._alloc_states()

    # ------------------------------------------------------------------ id -> slot
    def slots(self, ids: torch.Tensor, insert: bool = True) -> torch.Tensor:
        if self.id_mode == "direct":
            s = ids.long()
            if s.numel() and (int(s.min()) < 0 or int(s.max()) >= self.rows):
                raise IndexError(f"{self.name}: id out of range [0, {self.rows})")
            return s
        if self.id_mode == "hash":
            return torch.remainder(ids.long(), self.rows)
        return self.idmap.lookup(ids, insert)

    # ------------------------------------------------------------------ pull / push
    def pull_slots(self, slots: torch.Tensor) -> torch.Tensor:
        """Rows for (unique) local slots; lazily initialises untouched rows."""
        slots = slots.to(self.device)
        lo, hi = self.init
        if lo != 0.0 or hi != 0.0:
            _sp.lazy_init_rows(self.table, slots, self.flags, self.seed, self.row_base, lo, hi)
        else:
            self.flags[slots] = 1
        return _sp.gather_rows(self.table, slots)

    def pull(self, ids: torch.Tensor) -> torch.Tensor:
        return self.pull_slots(self.slots(ids))

    def push_slots(self, slots: torch.Tensor, grads: torch.Tensor, gscale: float = 1.0) -> None:
        """Apply the updater to unique local ``slots`` with ``grads`` [n, dim]."""
        if self.updater is None:
            raise RuntimeError(f"table {self.name} has no updater")
        if slots.numel() == 0:
            return
        u = self.updater
        skip = getattr(u, "mode", "") == "reference"  # FTRL reference skip of dw[0]==0 keys
        u.step_rows(self.table, self.states, slots.to(self.device), grads.to(self.device).contiguous(),
                    gscale=gscale, step=self.round + 1, rowwise=getattr(u, "rowwise", False), skip_zero=skip)

    def push(self, ids: torch.Tensor, grads: torch.Tensor, gscale: float = 1.0) -> None:
        self.push_slots(self.slots(ids, insert=True), grads, gscale)
        self.round += 1

    def state_dict(self) -> dict:
        return {"table": self.table.cpu(), "flags": self.flags.cpu(), "states": [s.cpu() for s in self.states],
                "round": self.round,
                "idmap": (None if self.idmap is None else self.idmap.lookup(torch.empty(0, dtype=torch.long)))}

    def load_state_dict(self, d: dict) -> None:
        self.table.copy_(d["table"])
        self.flags.copy_(d["flags"])
        for s, src in zip(self.states, d["states"]):
            s.copy_(src)
        self.round = int(d["round"])


class ShardedSparseTable:
    """Rows range/hash-partitioned over the co-located servers of ``transport``."""

    def __init__(self, name: str, dim: int, rows: int, transport: Transport, updater: Optional[Updater] = None, *,
                 init: Tuple[float, float] = (0.0, 0.0), id_mode: str = "direct", seed: int = 0, device=None):
        self.t = transport
        self.world, self.rank = transport.world, transport.rank
        self.name, self.dim, self.rows = name, int(dim), int(rows)
        self.id_mode = id_mode
        self.per_rank = (self.rows + self.world - 1) // self.world
        local_rows = self.per_rank if id_mode == "direct" else self.per_rank
        self.local = SparseTable(name, dim, local_rows, updater, init=init,
                                 id_mode=("direct" if id_mode == "direct" else id_mode), seed=seed,
                                 row_base=self.rank * self.per_rank, device=device)
        self.device = self.local.device
        self.round = 0

    def set_updater(self, u: Updater):
        self.local.set_updater(u)

    # ------------------------------------------------------------------ routing
    def _owner_local(self, ids: torch.Tensor):
        ids = ids.long()
        if self.id_mode == "direct":
            owner = torch.div(ids, self.per_rank, rounding_mode="floor")
            local = ids - owner * self.per_rank
            return owner, local
        owner = torch.remainder(_mix64(ids), self.world)
        return owner, ids  # owner maps the raw id (hash or exact map) itself

    def _exchange(self, owner: torch.Tensor, payloads: List[torch.Tensor]):
        """Send payload rows to their owners; returns (order, send_counts, recv_counts, received)."""
        order = torch.argsort(owner, stable=True)
        counts = torch.bincount(owner, minlength=self.world).to(torch.int64)
        send_counts = counts.to(self.device)
        recv_counts = torch.empty_like(send_counts)
        self.t.all_to_all(recv_counts, send_counts)
        sc = send_counts.cpu().tolist()
        rc = recv_counts.cpu().tolist()
        out = []
        for p in payloads:
            ps = p[order].contiguous()
            tail = tuple(ps.shape[1:])
            rbuf = torch.empty((sum(rc),) + tail, dtype=ps.dtype, device=ps.device)
            if tail:
                self.t.all_to_all(rbuf.view(sum(rc), -1), ps.view(ps.shape[0], -1), rc, sc)
            else:
                self.t.all_to_all(rbuf, ps, rc, sc)
            out.append(rbuf)
        return order, sc, rc, out

    def pull(self, ids: torch.Tensor) -> torch.Tensor:
        """Rows for unique global ``ids`` (any rank may ask for any rows)."""
        ids = ids.to(self.device).long()
        if self.world == 1:
            return self.local.pull(self._owner_local(ids)[1])
        owner, local = self._owner_local(ids)
        order, sc, rc, (rids,) = self._exchange(owner, [local])
        # serve: owner-side dedupe (several workers may ask for the same row)
        if rids.numel():
            u, inv = torch.unique(rids, return_inverse=True)
            rows_u = self.local.pull(u)
            rows = rows_u[inv]
        else:
            rows = torch.empty(0, self.dim, device=self.device)
        back = torch.empty(ids.numel(), self.dim, dtype=rows.dtype, device=self.device)
        self.t.all_to_all(back, rows.contiguous(), sc, rc)
        out = torch.empty_like(back)
        out[order] = back
        return out

    def push(self, ids: torch.Tensor, grads: torch.Tensor, average: bool = True) -> None:
        """Push per-row gradients for unique local ``ids``; owners sum duplicates across
        workers (divided by W when ``average``) and apply the row-sparse optimizer."""
        ids = ids.to(self.device).long()
        grads = grads.to(self.device).float().reshape(ids.numel(), self.dim)
        gscale = 1.0 / self.world if average else 1.0
        if self.world == 1:
            self.local.push(self._owner_local(ids)[1], grads, gscale)
            self.round += 1
            return
        owner, local = self._owner_local(ids)
        _, _, _, (rids, rgrads) = self._exchange(owner, [local, grads])
        if rids.numel():
            u, red = _sp.dedup_rows(rids, rgrads, mean=False, out_dtype=torch.float32)
            self.local.push(u, red, gscale)
        else:
            self.local.round += 1
        self.round += 1
