"""Row-sparse parameter tables: embeddings and wide (LR) weights on the parameter server.

Reference: one PS key per row -- ``"<field>.<id>"`` embedding rows (layer/EmbeddingField.java:57-104)
and ``"wide.weights.<id>"`` 1x1 wide weights (layer/LRLayer.java:62-120) -- batch-prefetched with
getList fan-out (store/KVStore.java:74-127, 279-298), created lazily on first touch by an
upsert(replace=false) round trip (net/PServer.java:143-162) and pushed one RPC per row
(store/KVStore.java:259).

Here a table is a set of row shards, one per co-located server rank (W >= 1).  All fields of a
layer share ONE table (keys carry the field), so a step moves every field's rows in one
exchange instead of one getList per field:

* key      direct: field_offset + id (range-partitioned rows, DLRM-style)
           hash:   field_offset + id mod rows (the wide hashing of util/MatrixUtil.java:27-33)
           map:    field << 44 | id, exact id -> slot on the owner (unbounded ids, Q17: int64)
* owner    direct/hash: key // ceil(total_rows / W);  map: mix64(key) mod W
* pull     (worker) sort keys by (owner, key) -> run heads = unique keys, per-owner counts
           -> count exchange -> async device->host copy of the W send + W receive counts ->
           all_to_all(keys) -> (owner) slot lookup (HIP hash map for map mode: no host round
           trip), deterministic lazy init keyed by the global key (HIP), gather ->
           all_to_all(rows) back.  The pulled rows are an autograd leaf; outputs gather
           through the inverse index (HIP), backward is a deterministic segment sum per unique
           key (HIP).  Host syncs: none at W = 1 on the GPU (every buffer is sized by the
           host-known n, pad keys -1 resolve to slot -1 = zero row / skipped update, the id
           range check is deferred to ``synchronize``); at W > 1 the split sizes must reach
           the host, and ``prefetch(next_ids)`` routes the next batch a step ahead so the
           copy has landed by the time its lookup runs (``stats["host_syncs"]`` counts waits).
* push     the leaf's gradient goes back along the SAME splits (no second count exchange);
           the owner sorts the received slots (several workers may push one row) and the
           HIP sparse optimizer sums each run and applies ONE update per row.  With
           ``overlap`` the push is launched from the leaf's post-accumulate-grad hook on a
           side stream, i.e. while the rest of backward still runs.
* micro-batches (Trainer n_threads > 1): while ``accumulating`` the owner keeps the received
  (slot, grad) pairs and applies once at the end of the round -- one optimizer step per row
  per round, the reference Trainer's single KVStore.update (train/Trainer.java:93).

``SparseTable`` is the W = 1 (standalone) table.  The TCP-server equivalent for the
dedicated-server topology is ``TcpSparseTable`` (rows live in the native server's row tables).
"""
from __future__ import annotations

import os
import zlib
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple, Union

import torch

from ..obs import trace as _trace
from ..ops import sparse as _sp
from .transport import Transport, side_stream
from .updaters import Updater

KEY_ID_BITS = 44
KEY_FIELD_BITS = 14
OWNER_SHIFT = KEY_ID_BITS + KEY_FIELD_BITS  # 58: keys stay below 2^58, owner in the top bits
KEY_MASK = (1 << OWNER_SHIFT) - 1


def stable_seed(name: str, seed: int = 0) -> int:
    """Per-table seed from a stable digest (Python's str hash is salted per process)."""
    return int(seed) + zlib.crc32(name.encode()) % 9973


def _mix64(x: torch.Tensor) -> torch.Tensor:
    """splitmix-style avalanche on int64 (works on CPU and GPU; wraps like uint64)."""
    x = x.long()
    x = (x ^ (x >> 31)) * 0x7FB5D329728EA185
    x = (x ^ (x >> 27)) * -0x7E25210B43D22E0B  # 0x81DADEF4BC2DD44D as signed
    return x ^ (x >> 33)


def _pow2(n: int) -> int:
    p = 1
    while p < n:
        p <<= 1
    return p


class _HostIdMap:
    """Exact id -> slot map on the host (CPU tables): native IdMap, dict fallback."""

    def __init__(self, capacity: int):
        self.capacity = capacity
        try:
            from .. import _native  # type: ignore

            self._m = _native.IdMap(capacity)
        except Exception:  # noqa: BLE001 -- pure-Python fallback
            self._m = None
            self._d = {}

    def lookup(self, ids: torch.Tensor, insert: bool = True) -> torch.Tensor:
        ids_c = ids.detach().cpu().long().contiguous()
        if self._m is not None:
            return torch.from_numpy(self._m.lookup(ids_c.numpy(), insert))
        res = []
        for v in ids_c.tolist():
            s = self._d.get(v)
            if s is None:
                s = -1
                if insert and len(self._d) < self.capacity:
                    s = len(self._d)
                    self._d[v] = s
            res.append(s)
        return torch.tensor(res, dtype=torch.int64)

    def items(self) -> torch.Tensor:
        """[n, 2] int64 (id, slot) pairs."""
        pairs = self._m.items() if self._m is not None else list(self._d.items())
        return torch.tensor(sorted(pairs), dtype=torch.int64).reshape(-1, 2)

    def restore(self, pairs: torch.Tensor) -> None:
        pairs = pairs.reshape(-1, 2)
        if self._m is not None:
            self._m = type(self._m)(self.capacity)
            if pairs.numel():
                self._m.restore(pairs[:, 0].contiguous().numpy(), pairs[:, 1].contiguous().numpy())
        else:
            self._d = {int(a): int(b) for a, b in pairs.tolist()}

    def __len__(self):
        return self._m.size() if self._m is not None else len(self._d)


class RowShard:
    """Owner-side storage of one table shard: fp32 rows, init flags, optimizer state, and
    (map mode) the key -> slot map -- a device hash map on the GPU, the native IdMap on CPU."""

    def __init__(self, dim: int, capacity: int, mode: str, row_base: int, seed: int, init: Tuple[float, float],
                 device, updater: Optional[Updater]):
        self.dim, self.mode, self.row_base, self.seed = int(dim), mode, int(row_base), int(seed)
        self.init = init
        self.device = device
        self.gpu = device.type == "cuda"
        if mode == "map" and self.gpu:
            capacity = _pow2(max(64, 2 * capacity))  # load factor <= 0.5 for linear probing
            self.hkeys = torch.full((capacity,), -1, dtype=torch.int64, device=device)
            self.idmap = None
        elif mode == "map":
            self.hkeys = None
            self.idmap = _HostIdMap(capacity)
        else:
            self.hkeys = self.idmap = None
        self.capacity = int(capacity)
        self.status = torch.zeros(1, dtype=torch.int32, device=device)  # map miss / overflow flag
        self.table = torch.zeros(self.capacity, self.dim, dtype=torch.float32, device=device)
        self.flags = torch.zeros(self.capacity, dtype=torch.uint8, device=device)
        self.updater = updater
        self.states: List[torch.Tensor] = []
        if updater is not None:
            self.alloc_states()

    def alloc_states(self) -> None:
        u = self.updater
        if getattr(u, "rowwise", False):
            self.states = [torch.zeros(self.capacity, dtype=torch.float32, device=self.device)]
        else:
            self.states = [torch.zeros_like(self.table) for _ in range(u.n_state)]

    def slots(self, keys: torch.Tensor, insert: bool = True) -> torch.Tensor:
        if self.mode != "map":
            return keys - self.row_base
        if self.gpu:
            return _sp.hash_slots(self.hkeys, keys, insert, self.status)
        s = self.idmap.lookup(keys, insert).to(keys.device)
        if insert and bool((s < 0).any()):
            raise RuntimeError(f"sparse table shard full ({self.capacity} rows)")
        return s

    def read(self, slots: torch.Tensor, keys: torch.Tensor) -> torch.Tensor:
        """Rows at ``slots`` (lazy deterministic init of untouched rows, RNG keyed by ``keys``)."""
        lo, hi = self.init
        if lo != 0.0 or hi != 0.0:  # zero-initialised tables (wide weights) need no first touch
            _sp.lazy_init_rows(self.table, slots, self.flags, self.seed, 0, lo, hi, keys=keys)
        return _sp.gather_rows(self.table, slots)

    def apply(self, slots: torch.Tensor, grads: torch.Tensor, gscale: float, step: int,
              sorted_runs: bool) -> None:
        u = self.updater
        if u is None:
            raise RuntimeError("sparse table has no updater")
        if slots.numel() == 0:
            return
        skip = getattr(u, "mode", "") == "reference"  # FTRL reference skip of dw[0]==0 keys
        perm = None
        if sorted_runs:
            slots, perm = torch.sort(slots)
        u.step_rows(self.table, self.states, slots, grads.contiguous(), gscale=gscale, step=step,
                    rowwise=getattr(u, "rowwise", False), skip_zero=skip, perm=perm)

    def check(self) -> None:
        """Raise if a map lookup missed / overflowed since the last check (GPU flag)."""
        if self.gpu and self.mode == "map" and int(self.status.item()):
            raise RuntimeError(f"sparse table shard full ({self.capacity} slots) or bad key")

    def state_dict(self) -> dict:
        snap = lambda t: t.detach().to("cpu", copy=True)  # noqa: E731 -- never alias live CPU state
        d = {"table": snap(self.table), "flags": snap(self.flags), "states": [snap(s) for s in self.states]}
        if self.hkeys is not None:
            d["hkeys"] = snap(self.hkeys)
        if self.idmap is not None:
            d["idmap"] = self.idmap.items()
        return d

    def load_state_dict(self, d: dict) -> None:
        self.table.copy_(d["table"])
        self.flags.copy_(d["flags"])
        for s, src in zip(self.states, d["states"]):
            s.copy_(src)
        if self.hkeys is not None and "hkeys" in d:
            self.hkeys.copy_(d["hkeys"])
        if self.idmap is not None and "idmap" in d:
            self.idmap.restore(d["idmap"])


@dataclass
class _Plan:
    """One pull's routing, reused by the matching push (no second count exchange)."""
    n: int
    nu: int
    inv: torch.Tensor          # [n] unique index of every looked-up position
    perm: torch.Tensor         # [n] positions in (owner, key) sorted order
    seg_off: torch.Tensor      # [nu + 1] runs of perm per unique key
    send: List[int]            # unique keys sent to each owner
    recv: List[int]            # keys received from each worker
    rslots: torch.Tensor       # owner-local slots of the received keys (push lands there)
    leaf: Optional[torch.Tensor] = None
    grad_fn: Optional[Callable] = None
    pushed: bool = False
    extra: dict = field(default_factory=dict)

    @property
    def counts(self) -> torch.Tensor:
        """Occurrences per unique key (>= 1; the empty pad segments of a sync-free plan read 1)."""
        return (self.seg_off[1:] - self.seg_off[:-1]).clamp(min=1)


@dataclass
class _Route:
    """Device-side routing of one lookup (sizes n / n + 1; nu and the splits live in ``counts``
    = [W send counts, #bad ids, W receive counts], copied to ``host`` asynchronously)."""
    n: int
    inv: torch.Tensor
    perm: torch.Tensor
    seg_full: torch.Tensor
    ubuf: torch.Tensor
    counts: torch.Tensor
    nbad: torch.Tensor
    host: Optional[torch.Tensor] = None
    event: Optional[object] = None


class ShardedSparseTable:
    """Rows partitioned over the co-located servers of ``transport`` (W = 1 without one).

    ``rows``: rows per field (int, or one int per field).  ``fields`` > 1 makes lookups take
    ids of shape [..., fields] (one table for all fields of a layer)."""

    def __init__(self, name: str, dim: int, rows: Union[int, Sequence[int]], transport: Optional[Transport] = None,
                 updater: Optional[Updater] = None, *, init: Tuple[float, float] = (0.0, 0.0),
                 id_mode: str = "direct", seed: int = 0, device=None, fields: int = 1, overlap: bool = False,
                 average: bool = True, exchange: Optional[str] = None):
        if id_mode not in ("direct", "hash", "map"):
            raise ValueError(id_mode)
        self.t = transport or Transport()
        self.world, self.rank = self.t.world, self.t.rank
        self.name, self.dim, self.id_mode = name, int(dim), id_mode
        if isinstance(rows, int):
            rows = [int(rows)] * int(fields)
        self.field_rows = [int(r) for r in rows]
        self.fields = len(self.field_rows)
        if self.fields >= (1 << KEY_FIELD_BITS):
            raise ValueError("too many fields")
        off = [0]
        for r in self.field_rows[:-1]:
            off.append(off[-1] + r)
        self.field_off = off
        self.rows = sum(self.field_rows)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.gpu = self.device.type == "cuda"
        self._foff = torch.tensor(off, dtype=torch.int64, device=self.device)
        self._frows = torch.tensor(self.field_rows, dtype=torch.int64, device=self.device)
        self.per_rank = (self.rows + self.world - 1) // self.world
        if id_mode == "map":
            cap = self.rows if self.world == 1 else int(self.per_rank * 1.25) + 64
            self.shard = RowShard(dim, cap, "map", 0, seed, init, self.device, updater)
        else:
            self.shard = RowShard(dim, self.per_rank, "direct", self.rank * self.per_rank, seed, init, self.device,
                                  updater)
        self.seed = int(seed)
        self.overlap = bool(overlap) and self.gpu
        self.average = average
        self.accumulating = False
        self.round = 0
        self._pending: List[_Plan] = []
        self._acc: List[Tuple[torch.Tensor, torch.Tensor]] = []
        self._push_done: Optional[torch.cuda.Event] = None
        self.stats = {"pulls": 0, "pushes": 0, "rows_pulled": 0, "rows_pushed": 0, "host_syncs": 0}
        self._pf: dict = {}  # ids signature -> (keys, route) of prefetched lookups
        self._nbad: Optional[torch.Tensor] = None  # deferred out-of-range id count (sync-free path)
        self._rows_dev = torch.zeros((), dtype=torch.int64, device=self.device)  # sync-free rows pulled
        # W > 1 on one node: the IPC / shared-memory row plane (row_plane.py) instead of all-to-alls
        # (``exchange`` "plane" | "collective"; default: PS_AMD_ROW_EXCHANGE, else auto)
        self.plane = None
        self._rowacc = None
        self.exchange_info: dict = {}  # row-plane probe record / fallback reason (bench JSON)
        if self.world > 1:
            from . import row_plane as _rp

            if exchange not in (None, "auto", "plane", "collective"):
                raise ValueError(exchange)
            if _rp.plane_rows_wanted(self.t, self.device, exchange):
                from .remote_probe import RemoteWriteUnavailable

                try:
                    self.plane = _rp.RowPlane(self.t, self.dim, self.device)
                    self._rowacc = _rp.RowAccumulator(self.shard)
                    self.exchange_info.update(self.plane.info)
                except RemoteWriteUnavailable as e:  # every rank: the collective all-to-alls instead
                    if exchange == "plane":
                        raise
                    self.exchange_info["fallback"] = str(e)
        self.exchange = "plane" if self.plane is not None else ("collective" if self.world > 1 else "local")

    # ------------------------------------------------------------------ compat accessors
    @property
    def table(self) -> torch.Tensor:
        return self.shard.table

    @property
    def states(self) -> List[torch.Tensor]:
        return self.shard.states

    @property
    def flags(self) -> torch.Tensor:
        return self.shard.flags

    @property
    def updater(self) -> Optional[Updater]:
        return self.shard.updater

    @property
    def init(self) -> Tuple[float, float]:
        return self.shard.init

    @init.setter
    def init(self, v: Tuple[float, float]) -> None:
        self.shard.init = v

    def set_updater(self, u: Updater) -> None:
        self.shard.updater = u
        self.shard.alloc_states()

    # ------------------------------------------------------------------ keys / routing
    def keys_of(self, ids: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(flat int64 keys, #invalid ids as a device scalar) for ids [..., fields]."""
        ids = ids.to(self.device).long()
        if self.fields > 1:
            if ids.shape[-1] != self.fields:
                raise ValueError(f"{self.name}: ids last dim {ids.shape[-1]} != fields {self.fields}")
            f = torch.arange(self.fields, device=self.device).expand_as(ids)
        else:
            f = torch.zeros_like(ids)
        ids, f = ids.reshape(-1), f.reshape(-1)
        if self.id_mode == "map":
            bad = (ids < 0) | (ids >= (1 << KEY_ID_BITS))
            keys = (f << KEY_ID_BITS) | ids.clamp(0, (1 << KEY_ID_BITS) - 1)
        else:
            rows_f = self._frows[f]
            if self.id_mode == "hash":
                ids = torch.remainder(ids, rows_f)
            bad = (ids < 0) | (ids >= rows_f)
            keys = self._foff[f] + ids.clamp(min=0).minimum(rows_f - 1)
        return keys, bad.sum()

    def _owner(self, keys: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return torch.zeros_like(keys)
        if self.id_mode == "map":
            return torch.remainder(_mix64(keys), self.world)
        return torch.div(keys, self.per_rank, rounding_mode="floor")

    def _wait_push(self) -> None:
        if self._push_done is not None:
            torch.cuda.current_stream(self.device).wait_event(self._push_done)
            self._push_done = None

    def _route(self, keys: torch.Tensor, nbad: torch.Tensor) -> "_Route":
        """Device half of the routing: dedupe + owner sort, per-owner unique counts and the count
        exchange, then (GPU) an ASYNC device->host copy of the counts.  No host sync here:
        ``_counts`` reads them when the key exchange needs its split sizes."""
        n = keys.numel()
        W = self.world
        owner = self._owner(keys)
        srt, perm = torch.sort((owner << OWNER_SHIFT) | keys)
        head = torch.ones(n, dtype=torch.bool, device=self.device)
        if n > 1:
            head[1:] = srt[1:] != srt[:-1]
        cum = torch.cumsum(head.long(), 0)
        uidx = cum - 1
        # outputs sized n / n + 1: unique key u < nu at ubuf[u], pad keys -1 behind it (no row);
        # segment u's occurrences at seg[u] .. seg[u + 1], empty pad segments [n, n)
        ubuf = torch.full((n,), -1, dtype=torch.int64, device=self.device)
        seg_full = torch.full((n + 1,), n, dtype=torch.int64, device=self.device)
        if n == 0:
            pass
        elif self.gpu:  # one HIP pass: unique keys + segment starts (no atomics, no host size)
            from ..ops._ext import native

            native().unique_runs(srt, uidx, KEY_MASK, ubuf, seg_full)
        else:
            ubuf.scatter_(0, uidx, srt & KEY_MASK)  # duplicates write identical values
            seg_full.scatter_reduce_(0, uidx, torch.arange(n, device=self.device), reduce="amin", include_self=True)
        # per-owner unique counts from the owner-major sort order (binary search, no atomics)
        bounds = torch.searchsorted(srt, torch.arange(W + 1, device=self.device, dtype=torch.int64) << OWNER_SHIFT)
        cum0 = torch.cat([torch.zeros(1, dtype=torch.int64, device=self.device), cum])
        meta = torch.empty(W + 1, dtype=torch.int64, device=self.device)
        meta[:W] = cum0[bounds[1:]] - cum0[bounds[:-1]]
        meta[W] = nbad
        if W > 1 and self.plane is None:
            recv = torch.empty(W, dtype=torch.int64, device=self.device)
            self.t.all_to_all(recv, meta[:W].contiguous())
            counts = torch.cat([meta, recv])
        else:
            counts = torch.cat([meta, meta[:1]])
        inv = torch.empty(n, dtype=torch.int64, device=self.device)
        inv[perm] = uidx
        r = _Route(n, inv, perm, seg_full, ubuf, counts, nbad)
        if self.gpu and self.plane is None:
            r.host = torch.empty(counts.numel(), dtype=torch.int64, pin_memory=True)
            r.host.copy_(counts, non_blocking=True)
            r.event = torch.cuda.Event()
            r.event.record()
        return r

    def _counts(self, r: "_Route") -> List[int]:
        """The route's counts on the host.  A host sync only if the copy has not landed yet --
        a route made by ``prefetch`` a step earlier has (stats["host_syncs"] counts the waits)."""
        if r.event is not None:
            if not r.event.query():
                self.stats["host_syncs"] += 1
                r.event.synchronize()
            return r.host.tolist()
        return r.counts.tolist()

    def prefetch(self, ids: torch.Tensor) -> None:
        """Route the NEXT batch's ids now (its device work and count exchange run ahead of this
        step's compute), so the lookup of ``ids`` finds its split sizes already on the host.
        Only useful at W > 1: at W = 1 the GPU lookup needs no counts at all."""
        if (self.world == 1 and self.gpu) or self.plane is not None:
            return  # no host-side sizes to wait for
        keys, nbad = self.keys_of(ids)
        if len(self._pf) >= 4:  # stale prefetches (ids never looked up): drop the oldest
            self._pf.pop(next(iter(self._pf)))
        self._pf[self._ids_sig(ids)] = (keys, self._route(keys, nbad))

    @staticmethod
    def _ids_sig(ids: torch.Tensor):
        return ids.data_ptr(), tuple(ids.shape), ids._version, ids.dtype

    def check_ids(self) -> None:
        """Raise if a sync-free (W = 1, GPU) lookup saw ids out of range since the last check."""
        if self._nbad is not None:
            nb = int(self._nbad.item())
            self._nbad = None
            if nb:
                raise IndexError(f"{self.name}: {nb} ids out of range for id_mode={self.id_mode!r}")

    def _serve_keys(self, ukeys: torch.Tensor, send: List[int], recv: List[int]):
        """Ship unique keys to their owners; owners resolve slots.  -> (received keys, slots)"""
        if self.world > 1:
            rkeys = torch.empty(sum(recv), dtype=torch.int64, device=self.device)
            self.t.all_to_all(rkeys, ukeys, recv, send)
        else:
            rkeys = ukeys
        return rkeys, self.shard.slots(rkeys, insert=True)

    def _rows_back(self, rows: torch.Tensor, nu: int, send: List[int], recv: List[int]) -> torch.Tensor:
        if self.world == 1:
            return rows
        back = torch.empty(nu, self.dim, dtype=rows.dtype, device=self.device)
        self.t.all_to_all(back, rows.contiguous(), send, recv)
        return back

    def _plan(self, keys: torch.Tensor, nbad: torch.Tensor, fetch: bool = True, route=None):
        with _trace.range(f"sparse.pull.{self.name}"):
            return self._plan_impl(keys, nbad, fetch, route)

    def _plan_impl(self, keys: torch.Tensor, nbad: torch.Tensor, fetch: bool, route=None):
        self._wait_push()
        r = route if route is not None else self._route(keys, nbad)
        n = r.n
        if self.plane is not None:
            # one-node IPC plane: counts stay on the device, the id check is deferred like W = 1
            self._nbad = r.nbad.clone() if self._nbad is None else self._nbad + r.nbad
            rows, st = self.plane.pull(r.ubuf, r.counts, n, self.shard, fetch)
            plan = _Plan(n, n, r.inv, r.perm, r.seg_full, [n], [n], None)
            plan.extra["plane"] = st
            if fetch:
                self.stats["pulls"] += 1
            return plan, (rows if fetch else None)
        if self.world == 1 and self.gpu:
            # sync-free: every buffer sized n (pad keys -1 -> slot -1 -> zero row, skipped by
            # the optimizer), the id check deferred to check_ids / synchronize
            self._nbad = r.nbad.clone() if self._nbad is None else self._nbad + r.nbad
            nu, send, recv = n, [n], [n]
            ukeys, seg_off = r.ubuf, r.seg_full
            self._rows_dev = self._rows_dev + r.counts[0]
        else:
            h = self._counts(r)
            W = self.world
            if h[W]:
                raise IndexError(f"{self.name}: {h[W]} ids out of range for id_mode={self.id_mode!r}")
            send, recv = h[:W], h[W + 1:]
            nu = sum(send)
            ukeys, seg_off = r.ubuf[:nu], r.seg_full[:nu + 1]
            self.stats["rows_pulled"] += nu
        rkeys, rslots = self._serve_keys(ukeys, send, recv)
        rows = None
        if fetch:
            rows = self._rows_back(self.shard.read(rslots, rkeys), nu, send, recv)
            self.stats["pulls"] += 1
        return _Plan(n, nu, r.inv, r.perm, seg_off, send, recv, rslots), rows

    def _take_prefetch(self, ids: torch.Tensor):
        if not self._pf:
            return None
        return self._pf.pop(self._ids_sig(ids), None)

    # ------------------------------------------------------------------ worker API
    def lookup(self, ids: torch.Tensor, out_dtype=None, grad_fn: Optional[Callable] = None) -> torch.Tensor:
        """Rows of ``ids`` -> [*ids.shape, dim] (ids [..., fields] when fields > 1).  Autograd
        flows to the pulled rows; their gradient is pushed by ``push_pending`` (or by the
        leaf hook when ``overlap``).  ``grad_fn(grad_unique, plan)`` may rewrite the pushed
        gradient (reference gradient modes)."""
        pf = self._take_prefetch(ids)
        if pf is not None:
            keys, route = pf
            plan, rows = self._plan(keys, route.nbad, route=route)
        else:
            keys, nbad = self.keys_of(ids)
            plan, rows = self._plan(keys, nbad)
        want_grad = torch.is_grad_enabled()
        leaf = rows.detach().requires_grad_(want_grad)
        out = _sp.gather_unique(leaf, plan.inv, plan.perm, plan.seg_off, out_dtype)
        if want_grad:
            plan.leaf, plan.grad_fn = leaf, grad_fn
            self._pending.append(plan)
            if self.overlap:
                leaf.register_post_accumulate_grad_hook(lambda _p, pl=plan: self._push_plan(pl, not self.accumulating))
        return out.view(*ids.shape, self.dim)

    def pull_keys(self, keys: torch.Tensor) -> torch.Tensor:
        keys = keys.to(self.device).long().reshape(-1)
        plan, rows = self._plan(keys, torch.zeros((), dtype=torch.int64, device=self.device))
        return rows[plan.inv]

    def pull(self, ids: torch.Tensor) -> torch.Tensor:
        """Rows for ``ids`` (no autograd): [n, dim] for flat ids, [..., fields, dim] otherwise."""
        keys, nbad = self.keys_of(ids)
        plan, rows = self._plan(keys, nbad)
        out = rows[plan.inv]
        return out if self.fields == 1 else out.view(*ids.shape, self.dim)

    def push(self, ids: torch.Tensor, grads: torch.Tensor, gscale: Optional[float] = None, *,
             average: Optional[bool] = None) -> None:
        """Direct push of per-id gradient rows (duplicates within a worker are summed)."""
        keys, nbad = self.keys_of(ids)
        plan, _ = self._plan(keys, nbad, fetch=False)
        grads = grads.to(self.device).float().reshape(plan.n, self.dim).contiguous()
        ug = torch.empty(plan.nu, self.dim, dtype=torch.float32, device=self.device)
        _sp.segment_reduce_rows(grads, plan.perm, plan.seg_off, ug, False)
        self._exchange_grads(plan, ug)
        self._apply_acc(gscale, average)

    def _exchange_grads(self, plan: _Plan, g: torch.Tensor) -> None:
        _trace.mark(f"sparse.push.{self.name}")
        if "plane" in plan.extra:
            self.plane.push(g, plan.nu, plan.extra.pop("plane"), self.shard, self._rowacc)
            plan.pushed = True
            self.stats["pushes"] += 1
            return
        if self.world > 1:
            rg = torch.empty(sum(plan.recv), self.dim, dtype=torch.float32, device=self.device)
            self.t.all_to_all(rg, g.contiguous(), plan.recv, plan.send)
        else:
            rg = g
        self._acc.append((plan.rslots, rg))
        plan.pushed = True
        self.stats["pushes"] += 1
        if not (self.world == 1 and self.gpu):
            self.stats["rows_pushed"] += plan.nu

    def _apply_acc(self, gscale: Optional[float] = None, average: Optional[bool] = None) -> None:
        avg = self.average if average is None else average
        gs = gscale if gscale is not None else (1.0 / self.world if avg else 1.0)
        if self._rowacc is not None and self._rowacc.open:
            self._rowacc.apply(gs, self.round + 1, self.plane)
            self.round += 1
            return
        if not self._acc:
            return
        if len(self._acc) == 1 and self.world == 1:
            slots, g = self._acc[0]  # unique slots already
            self.shard.apply(slots, g, gs, self.round + 1, sorted_runs=False)
        else:
            slots = torch.cat([a for a, _ in self._acc])
            g = torch.cat([b for _, b in self._acc])
            self.shard.apply(slots, g, gs, self.round + 1, sorted_runs=True)
        self._acc = []
        self.round += 1

    def _grad_of(self, plan: _Plan) -> Optional[torch.Tensor]:
        g = plan.leaf.grad if plan.leaf is not None else None
        if g is None:
            return None
        g = g.float()
        if plan.grad_fn is not None:
            g = plan.grad_fn(g, plan)
        return g.contiguous()

    def _push_plan(self, plan: _Plan, apply_now: bool) -> None:
        if plan.pushed:
            return
        g = self._grad_of(plan)
        if g is None:
            plan.pushed = True
            return
        if self.overlap:
            cur = torch.cuda.current_stream(self.device)
            comm = side_stream(self.device)
            ev = torch.cuda.Event()
            ev.record(cur)
            comm.wait_event(ev)
            g.record_stream(comm)
            if plan.rslots is not None:
                plan.rslots.record_stream(comm)
            for v in plan.extra.get("plane", {}).values():  # the row plane's per-round index tensors
                if isinstance(v, torch.Tensor) and v.is_cuda:
                    v.record_stream(comm)
            with torch.cuda.stream(comm):
                self._exchange_grads(plan, g)
                if apply_now:
                    self._apply_acc()
                done = torch.cuda.Event()
                done.record(comm)
            self._push_done = done
        else:
            self._exchange_grads(plan, g)
            if apply_now:
                self._apply_acc()
        plan.leaf = None

    def push_pending(self) -> int:
        """Push every looked-up-but-not-yet-pushed plan; apply unless accumulating."""
        n = 0
        for plan in self._pending:
            if not plan.pushed:
                self._push_plan(plan, apply_now=False)
                n += plan.nu
        self._pending = []
        if not self.accumulating:
            if self.overlap and (self._acc or (self._rowacc is not None and self._rowacc.open)):
                comm = side_stream(self.device)
                comm.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(comm):
                    self._apply_acc()
                    done = torch.cuda.Event()
                    done.record(comm)
                self._push_done = done
            else:
                self._apply_acc()
        return n

    def drop_pending(self) -> None:
        self._pending = []

    def synchronize(self) -> None:
        self._wait_push()
        self.shard.check()
        self.check_ids()

    def close(self) -> None:
        """Release the row plane's shared memory (collective)."""
        if self.plane is not None:
            self.plane.close()
            self.plane = None

    def row_stats(self) -> dict:
        """``stats`` with the sync-free path's device-side unique-row count read back (a sync)."""
        d = dict(self.stats)
        if self.world == 1 and self.gpu:
            d["rows_pulled"] = int(self._rows_dev.item())
        return d

    # ------------------------------------------------------------------ checkpoint
    def state_dict(self) -> dict:
        self.synchronize()
        d = self.shard.state_dict()
        d["round"] = self.round
        d["world"], d["rank"] = self.world, self.rank
        return d

    def load_state_dict(self, d: dict) -> None:
        if int(d.get("world", self.world)) != self.world:
            raise ValueError("sparse-table checkpoint was written with a different world size")
        self.shard.load_state_dict(d)
        self.round = int(d["round"])


class SparseTable(ShardedSparseTable):
    """Standalone (W = 1) table: ``SparseTable(name, dim, rows, updater, init=..., id_mode=...)``."""

    def __init__(self, name: str, dim: int, rows: Union[int, Sequence[int]], updater: Optional[Updater] = None, *,
                 init: Tuple[float, float] = (0.0, 0.0), id_mode: str = "direct", seed: int = 0, device=None,
                 fields: int = 1, overlap: bool = False):
        super().__init__(name, dim, rows, None, updater, init=init, id_mode=id_mode, seed=seed, device=device,
                         fields=fields, overlap=overlap)


# ------------------------------------------------------------------------------ TCP rows
class TcpSparseTable:
    """A sparse table whose rows live in the native TCP servers' row tables (dedicated-server
    topology, -Dmode=dist).  pull = one ROW_PULL per server with the unique keys routed by
    key hash (the reference's getList fan-out, store/KVStore.java:74-107, with creation on the
    server: deterministic init from (seed, key), so the first writer trivially wins); push =
    one ROW_PUSH per server with the per-key summed gradient (BSP: accumulated, applied by the
    barrier; SSP/ASP: applied on arrival)."""

    def __init__(self, name: str, dim: int, rows: Union[int, Sequence[int]], client, updater: Optional[Updater] = None,
                 *, init: Tuple[float, float] = (0.0, 0.0), id_mode: str = "map", seed: int = 0, fields: int = 1,
                 device=None):
        self.client = client
        self.name, self.dim, self.id_mode, self.seed = name, int(dim), id_mode, int(seed)
        if isinstance(rows, int):
            rows = [int(rows)] * int(fields)
        self.field_rows = [int(r) for r in rows]
        self.fields = len(self.field_rows)
        off = [0]
        for r in self.field_rows[:-1]:
            off.append(off[-1] + r)
        self.field_off = off
        self.init = init
        self.updater = updater
        self.accumulating = False
        self.round = 0
        self._pending: List[dict] = []
        self.device = torch.device(device) if device is not None else torch.device("cpu")

    def set_updater(self, u: Updater) -> None:
        self.updater = u

    def keys_of(self, ids: torch.Tensor) -> torch.Tensor:
        ids = ids.detach().cpu().long()
        if self.fields > 1:
            f = torch.arange(self.fields).expand_as(ids)
        else:
            f = torch.zeros_like(ids)
        ids, f = ids.reshape(-1), f.reshape(-1)
        if self.id_mode == "map":
            if bool(((ids < 0) | (ids >= (1 << KEY_ID_BITS))).any()):
                raise IndexError(f"{self.name}: ids out of range")
            return (f << KEY_ID_BITS) | ids
        rows_f = torch.tensor(self.field_rows)[f]
        if self.id_mode == "hash":
            ids = torch.remainder(ids, rows_f)
        if bool(((ids < 0) | (ids >= rows_f)).any()):
            raise IndexError(f"{self.name}: ids out of range")
        return torch.tensor(self.field_off)[f] + ids

    def _pull_unique(self, ukeys: torch.Tensor) -> torch.Tensor:
        lo, hi = self.init
        return self.client.row_pull(self.name, self.dim, ukeys, lo, hi, self.seed)

    def lookup(self, ids: torch.Tensor, out_dtype=None, grad_fn: Optional[Callable] = None) -> torch.Tensor:
        keys = self.keys_of(ids)
        ukeys, inv, counts = torch.unique(keys, return_inverse=True, return_counts=True)
        rows = self._pull_unique(ukeys).to(self.device)
        want_grad = torch.is_grad_enabled()
        leaf = rows.detach().requires_grad_(want_grad)
        out = leaf[inv.to(self.device)]
        if out_dtype is not None:
            out = out.to(out_dtype)
        if want_grad:
            self._pending.append({"keys": ukeys, "leaf": leaf, "grad_fn": grad_fn,
                                  "plan": _TcpPlan(keys.numel(), counts)})
        return out.view(*ids.shape, self.dim)

    def pull(self, ids: torch.Tensor) -> torch.Tensor:
        keys = self.keys_of(ids)
        ukeys, inv = torch.unique(keys, return_inverse=True)
        out = self._pull_unique(ukeys)[inv]
        return out if self.fields == 1 else out.view(*ids.shape, self.dim)

    def _spec(self) -> str:
        if self.updater is None:
            raise RuntimeError(f"table {self.name} has no updater")
        return self.updater.name

    def push(self, ids: torch.Tensor, grads: torch.Tensor) -> None:
        keys = self.keys_of(ids)
        ukeys, inv = torch.unique(keys, return_inverse=True)
        g = torch.zeros(ukeys.numel(), self.dim).index_add_(0, inv, grads.detach().cpu().float().reshape(-1, self.dim))
        self.client.row_push(self.name, self.dim, ukeys, g, self._spec())
        self.round += 1

    def push_pending(self) -> int:
        n = 0
        merged_k, merged_g = [], []
        for p in self._pending:
            leaf = p["leaf"]
            if leaf.grad is None:
                continue
            g = leaf.grad.detach().float()
            if p["grad_fn"] is not None:
                g = p["grad_fn"](g, p["plan"])
            merged_k.append(p["keys"])
            merged_g.append(g.cpu())
            n += p["keys"].numel()
        self._pending = []
        if merged_k:
            keys = torch.cat(merged_k)
            g = torch.cat(merged_g)
            uk, inv = torch.unique(keys, return_inverse=True)
            red = torch.zeros(uk.numel(), self.dim).index_add_(0, inv, g)
            self.client.row_push(self.name, self.dim, uk, red, self._spec())
            self.round += 1
        return n

    def drop_pending(self) -> None:
        self._pending = []

    def synchronize(self) -> None:
        pass


@dataclass
class _TcpPlan:
    n: int
    counts: torch.Tensor
