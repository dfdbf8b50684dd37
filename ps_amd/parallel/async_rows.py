"""Asynchronous sparse rows: embedding / wide rows under ASP and SSP without lockstep traffic.

Reference: every embedding row and every wide weight is its own PS key, pulled per batch with
``getList`` (store/KVStore.java:74-127, layer/EmbeddingField.java:57-64, layer/LRLayer.java:62-70)
and pushed through the same fire-and-forget ``push`` as the dense keys; an async server
applies each push on arrival (net/PServer.java:164-184).  The collective sparse exchange of
``ShardedSparseTable`` (all-to-alls) keeps every rank in lockstep; here, as for the dense keys
of ``AsyncPS``, no rank ever waits for another rank to reach a matching call:

* rows are owned by ``mix64(key) % W`` (the sharded table's rule); each owner keeps its shard in
  a ``RowShard`` (device hash map, fp32 rows, lazy-init flags, optimizer state) that ONLY its
  own row-service thread touches;
* pull  = the worker writes its unique keys for owner o into o's request mailbox (IPC-mapped
  memory), bumps ``req[o][me]`` and waits for ``resp[o][me]`` -- i.e. for owner o's service
  thread, never for another worker -- then reads the rows out of o's response buffer;
* push  = the worker writes (keys, summed row gradients) into o's push mailbox (2 deep: push k
  lands in slot k % 2) and bumps ``pseq[o][me]``; it waits only if its push k-2 is still
  unapplied.  The owner applies the row optimizer (gradient / W) on arrival;
* SSP(s): before its pull at round c a worker waits until every owner applied every worker's
  first c - s row pushes (the dense gate of ``AsyncPS`` for the rows); ASP: no gate.

GPU: device-resident end to end.  The worker dedupes and owner-sorts its keys on the device
(counts never reach its host) and ONE segment kernel writes every owner's piece -- with its
count -- into that owner's IPC-mapped mailbox; a completion thread bumps the request word once
the copy landed (the training thread does not wait for it).  Each owner runs a NATIVE service
thread (csrc/async_rows_gpu.cpp: no Python, no GIL) that reads the count on its own stream and
launches the HIP hash lookup, lazy init, gather into its response mailbox, or the row optimizer
for a push.  The worker copies its rows back out of the owners' response mailboxes with one
kernel: keys, rows and gradients never pass through host memory.
CPU: a native poller (csrc/runtime/bindings_native.cpp ``rows.Service``) calls back into Python
for the row work (the same ops' torch oracles).
"""
from __future__ import annotations

import uuid
from typing import Optional, Sequence, Tuple, Union

import torch

from .async_ps import _addr, _native, _Shared, _ShmSeg
from ..ops import sparse as _sp
from .sparse_table import KEY_ID_BITS, KEY_MASK, OWNER_SHIFT, RowShard, TcpSparseTable, _mix64
from .transport import Transport
from .updaters import Updater

_MAGIC_WORDS = 4


class _RowCtl:
    """Word addresses of one table's control block (layout: csrc/runtime/bindings_native.cpp)."""

    def __init__(self, base: int, W: int, mb: int):
        self.base, self.W, self.mb = base, W, mb

    def _w(self, k: int, o: int, w: int) -> int:
        return self.base + 8 * (_MAGIC_WORDS + k * self.W * self.W + o * self.W + w)

    def req(self, o, w):
        return self._w(0, o, w)

    def resp(self, o, w):
        return self._w(1, o, w)

    def nreq(self, o, w):
        return self._w(2, o, w)

    def pseq(self, o, w):
        return self._w(3, o, w)

    def pack(self, o, w):
        return self._w(4, o, w)

    def npush(self, o, w, m):
        return self.base + 8 * (_MAGIC_WORDS + 5 * self.W * self.W + (o * self.W + w) * self.mb + m)

    @property
    def stop(self):
        return self.base + 16


class _AsyncRowClient:
    """The ``row_pull`` / ``row_push`` of ``TcpSparseTable`` over owner mailboxes."""

    def __init__(self, table: "AsyncRowTable"):
        self.tb = table

    def row_pull(self, name, dim, ukeys: torch.Tensor, lo, hi, seed) -> torch.Tensor:
        return self.tb._pull(ukeys)

    def row_push(self, name, dim, ukeys: torch.Tensor, grads: torch.Tensor, spec: str) -> None:
        self.tb._push(ukeys, grads)


class AsyncRowTable(TcpSparseTable):
    """A sparse table whose rows live on the co-located owners, reached one-sidedly (module
    docstring).  ``staleness=None`` is ASP, an int s is SSP(s).  ``capacity``: max unique keys
    one worker sends one owner per pull / push; ``rows_per_owner``: owner shard capacity."""

    def __init__(self, name: str, dim: int, rows: Union[int, Sequence[int]], transport: Transport,
                 updater: Optional[Updater] = None, *, init: Tuple[float, float] = (0.0, 0.0), id_mode: str = "map",
                 seed: int = 0, fields: int = 1, device=None, staleness: Optional[int] = None,
                 capacity: int = 1 << 15, rows_per_owner: Optional[int] = None, timeout_s: float = 600.0):
        self.t = transport
        self.W, self.me = transport.world, transport.rank
        super().__init__(name, dim, rows, _AsyncRowClient(self), updater, init=init, id_mode=id_mode, seed=seed,
                         fields=fields, device=device)
        self.staleness = staleness
        # SSP audit (AsyncPS.gate_log's twin): a list records (clock, gate target, min applied
        # row push seen) per gated pull
        self.gate_log: Optional[list] = None
        self.C = int(capacity)
        self.timeout_s = timeout_s
        self.gpu = self.device.type == "cuda"
        total = sum(self.field_rows)
        cap = rows_per_owner or max(1024, 2 * total // self.W + 1024)
        self.shard = RowShard(self.dim, cap, "map", 0, self.seed, self.init, self.device, updater)
        W, MB = self.W, None
        N = _native()
        MB = N.async_ctl.MBOX()
        self.MB = MB
        # owner-side mailboxes (shared): request keys, response rows, push keys / gradients
        self.share = _Shared(transport, self.device)
        C, D = self.C, self.dim
        # (GPU: the word after a mailbox's C keys carries the request's count, written on device)
        self.rq = self.share.alloc((W, C + 1), torch.int64)
        self.rs = self.share.alloc((W, C, D), torch.float32)
        self.pk = self.share.alloc((W, MB, C + 1), torch.int64)
        self.pg = self.share.alloc((W, MB, C, D), torch.float32)
        self.peer_rq = self.share.exchange(self.rq)
        self.peer_rs = self.share.exchange(self.rs)
        self.peer_pk = self.share.exchange(self.pk)
        self.peer_pg = self.share.exchange(self.pg)
        # control block: rank 0 creates it
        R = N.rows
        cname = transport.all_gather_object(f"psamd_rows_{uuid.uuid4().hex[:16]}" if self.me == 0 else None)[0]
        if self.me == 0:
            self._ctl = _ShmSeg(cname, R.ctl_size(W), create=True)
            R.ctl_init(_addr(self._ctl), W)
        transport.barrier()
        if self.me != 0:
            self._ctl = _ShmSeg(cname)
        self.ctl = _RowCtl(_addr(self._ctl), W, MB)
        self.shm = N.shm
        self.pulls = 0
        self.pushes = 0
        self.applied = 0
        # the owner's row work and the worker's mailbox copies run on streams of their own: a
        # copy never waits behind the compute stream's queued kernels
        self._svc_stream = torch.cuda.Stream(device=self.device) if self.gpu else None
        self._io_stream = torch.cuda.Stream(device=self.device) if self.gpu else None
        if self.gpu:
            from .. import _C  # type: ignore

            self._R = _C.rows
            self.service = self._R.Service(self.ctl.base, self.me, C, D)
            self.service.set_mailboxes(self.rq, self.rs, self.pk, self.pg)
            self._configure_native()
            self._notify = self._R.Notifier()
            self._nbad = None
        else:
            self.service = R.Service(self.ctl.base, self.me, self._serve)
        transport.barrier()
        # start-up probe of the one-sided writes into the owners' mailboxes (VERDICT r5 Next #2):
        # fails on every rank alike with RemoteWriteUnavailable (loud, no silent wrong rows)
        self.info = {"engine": "AsyncRowTable"}
        if self.W > 1:
            try:
                self.info["remote_write_probe"] = self._probe_remote_writes()
            except Exception:
                self.share.close(unlink=True)
                self._ctl.close()
                if self.me == 0:
                    self._ctl.unlink()
                raise
        self.service.start()

    def _probe_remote_writes(self, rows: int = 4) -> str:
        """Every rank writes a pattern into slot 0 of its gradient mailbox row on every owner with
        the production segment kernel (``rows.to_peers``, the push's write); each owner reads the
        W - 1 rows it received through an acquiring kernel once the writers' copies completed --
        three rounds over the same lines, then the lines are zeroed (before the service starts)."""
        from .remote_probe import pattern, run_probe

        W, me, D = self.W, self.me, self.dim
        n = rows * D
        peers = [w for w in range(W) if w != me]
        if self.gpu:
            from .. import _C  # type: ignore

            P = _C.plane
            io, rs = self._io_stream, torch.cuda.Stream(device=self.device)
            out = torch.zeros(W, n, dtype=torch.float32, device=self.device)
            meta = torch.tensor([o * rows for o in range(W)] + [rows] * W, dtype=torch.int64, device=self.device)

            def write(k):
                buf = pattern(k, me, n).repeat(W).to(self.device)  # owner-major: W pieces of `rows` rows
                io.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(io):
                    self._R.to_peers(buf, meta, [self.peer_pg[o][me][0].data_ptr() for o in range(W)], [], D, self.C)
                io.synchronize()

            def publish(k):
                self.t.barrier()

            def read(k):
                for w in peers:
                    P.read_acquire(self.pg[w][0].data_ptr(), n, False, out[w], rs.cuda_stream)
                rs.synchronize()
                return out[peers].cpu()

            def settle():
                torch.cuda.synchronize(self.device)
                self.t.barrier()
        else:
            def write(k):
                src = pattern(k, me, n).view(rows, D)
                for o in peers:
                    self.peer_pg[o][me][0][:rows].copy_(src)

            def publish(k):
                self.t.barrier()

            def read(k):
                return torch.stack([self.pg[w][0][:rows].reshape(-1).clone() for w in peers])

            def settle():
                self.t.barrier()

        rec = run_probe(self.t, "asyncrows", 3, write, publish, read,
                        lambda k: torch.stack([pattern(k, w, n) for w in peers]), settle)
        with torch.no_grad():
            for w in range(W):
                self.pg[w][0][:rows].zero_()
        if self.gpu:
            torch.cuda.synchronize(self.device)
        self.t.barrier()
        return rec

    def _configure_native(self) -> None:
        """Hand the shard (and the updater, once known) to the native GPU service.  The service
        thread reads its configuration without a lock, so a reconfiguration after ``start()``
        (``set_updater``, the ``init`` setter) stops the thread, reconfigures and restarts it;
        requests that arrive meanwhile wait in the control words.  The hyper-parameters are a
        snapshot taken here: changing ``updater.lr`` later needs another ``set_updater``."""
        if not self.gpu or getattr(self, "service", None) is None:
            return
        was = self.service.running
        if was:
            self.service.stop()
        try:
            self._configure_native_body()
        finally:
            if was:
                self.service.start()

    def _configure_native_body(self) -> None:
        sh = self.shard
        st = list(sh.states) + [None] * (2 - len(sh.states))
        lo, hi = sh.init
        self.service.set_shard(sh.table, sh.flags, sh.hkeys, sh.row_base, sh.status, st[0], st[1], sh.seed,
                               float(lo), float(hi))
        u = self.updater
        if u is not None:
            from ..ops import optim as _o
            from .async_ps import _BIAS_MODE, _HYPER
            from .updaters import AdamUpdater

            h = _o._hp(u.hyper(1))
            bias = _BIAS_MODE[u.bias_correction] if isinstance(u, AdamUpdater) else 0
            self.service.set_updater(u.kind, [float(h[k]) for k in _HYPER], bias, bool(getattr(u, "rowwise", False)),
                                     getattr(u, "mode", "") == "reference", 1.0 / self.W)

    # ------------------------------------------------------------------ config
    def set_updater(self, u: Updater) -> None:
        self.updater = u
        self.shard.updater = u
        self.shard.alloc_states()
        self._configure_native()

    @property
    def init(self):
        return self._init

    @init.setter
    def init(self, v):
        self._init = tuple(v)
        if getattr(self, "shard", None) is not None:
            self.shard.init = self._init
            self._configure_native()

    # ------------------------------------------------------------------ worker side
    def _owner(self, keys: torch.Tensor) -> torch.Tensor:
        return torch.remainder(_mix64(keys), self.W) if self.W > 1 else torch.zeros_like(keys)

    def _check_cap(self, n: int, what: str = "request") -> None:
        """Mailbox bound.  CPU: ``n`` = one owner's unique keys.  GPU: the per-owner counts stay on
        the device (no host sync), so the host checks the bound it knows -- the request's unique
        ids over ALL owners -- i.e. on the GPU the capacity C is per request, not per owner: size
        it to at least the (unique) ids of one step."""
        if n > self.C:
            who = "for one owner" if not self.gpu else "in one GPU request (all owners; capacity is per request)"
            raise RuntimeError(f"async row table {self.name}: {what} of {n} keys {who} exceeds capacity {self.C}")

    def _ssp_gate(self) -> None:
        """SSP(s): every owner applied every worker's first (clock - s) row pushes -- this
        worker's clock = rounds pushed, the same target AsyncPS's dense gate uses for its pull
        (host words, no device sync)."""
        if self.staleness is None or self.W == 1:
            return
        W, c = self.W, self.ctl
        words = [c.pack(o, w) for o in range(W) for w in range(W)]
        target = self.pushes - int(self.staleness)
        if target > 0:
            self.shm.wait_ge(words, target, c.stop, self.timeout_s)
        if self.gate_log is not None:
            self.gate_log.append((self.pushes, target, min(self.shm.ld(a) for a in words)))

    def _pull(self, ukeys: torch.Tensor) -> torch.Tensor:
        """Rows of the unique ``ukeys`` (CPU int64) -> [n, dim] fp32 on CPU."""
        W, me, c = self.W, self.me, self.ctl
        self._ssp_gate()
        own = self._owner(ukeys)
        parts = []
        with self._io():
            for o in range(W):
                ko = ukeys[own == o]
                self._check_cap(ko.numel())
                if ko.numel():
                    self.peer_rq[o][me][:ko.numel()].copy_(ko)
                parts.append(ko)
            self._io_sync()  # the keys are in the owners' memory before the requests go up
        for o in range(W):
            self.shm.st(c.nreq(o, me), parts[o].numel())
        self.pulls += 1
        for o in range(W):
            self.shm.add(c.req(o, me), 1)
        self.shm.wait_ge([c.resp(o, me) for o in range(W)], self.pulls, c.stop, self.timeout_s)
        out = torch.empty(ukeys.numel(), self.dim, dtype=torch.float32)
        with self._io():
            for o, ko in enumerate(parts):
                if ko.numel():
                    out[own == o] = self.peer_rs[o][me][:ko.numel()].to("cpu")
        return out

    def _io(self):
        return torch.cuda.stream(self._io_stream) if self.gpu else _Null()

    def _io_sync(self) -> None:
        if self.gpu:
            self._io_stream.synchronize()

    def _push(self, ukeys: torch.Tensor, grads: torch.Tensor) -> None:
        W, me, c = self.W, self.me, self.ctl
        k = self.pushes
        slot = k % self.MB
        if k >= 2:  # mailbox slot k % 2 is free once push k - 2 was applied
            self.shm.wait_ge([c.pack(o, me) for o in range(W)], k - 1, c.stop, self.timeout_s)
        own = self._owner(ukeys)
        g = grads.float().cpu()
        ns = []
        with self._io():
            for o in range(W):
                sel = own == o
                ko = ukeys[sel]
                self._check_cap(ko.numel())
                if ko.numel():
                    self.peer_pk[o][me][slot][:ko.numel()].copy_(ko)
                    self.peer_pg[o][me][slot][:ko.numel()].copy_(g[sel])
                ns.append(ko.numel())
            self._io_sync()
        for o in range(W):
            self.shm.st(c.npush(o, me, slot), ns[o])
        for o in range(W):
            self.shm.add(c.pseq(o, me), 1)
        self.pushes += 1

    def push_pending(self) -> int:
        """Every round pushes (possibly nothing): the owners' applied counts are the clocks of
        the SSP gate."""
        if self.gpu:
            return self._push_pending_dev()
        n = super().push_pending()
        if n == 0 and not self.accumulating:
            self._push(torch.empty(0, dtype=torch.int64), torch.empty(0, self.dim))
            self.round += 1
        return n

    # ------------------------------------------------------------------ worker side, GPU
    # (device-resident: no key, row, gradient or count passes through host memory)
    def _keys_dev(self, ids: torch.Tensor) -> torch.Tensor:
        """Flat int64 keys on the device; out-of-range ids are clamped and counted for a deferred
        check (synchronize), as the sync-free sharded table does."""
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
            rows_f = torch.tensor(self.field_rows, device=self.device)[f]
            if self.id_mode == "hash":
                ids = torch.remainder(ids, rows_f)
            bad = (ids < 0) | (ids >= rows_f)
            keys = torch.tensor(self.field_off, device=self.device)[f] + ids.clamp(min=0).minimum(rows_f - 1)
        nb = bad.sum()
        self._nbad = nb if self._nbad is None else self._nbad + nb
        return keys

    def _route_dev(self, keys: torch.Tensor) -> dict:
        """Dedupe + owner-major sort on the device.  Negative keys (pads of a merged push) go to a
        virtual owner W: they sort last and are in no owner's count, so they are never sent."""
        from ..ops._ext import native

        W, n = self.W, keys.numel()
        own = torch.remainder(_mix64(keys), W) if W > 1 else torch.zeros_like(keys)
        own = torch.where(keys < 0, torch.full_like(own, W), own)
        srt, perm = torch.sort((own << OWNER_SHIFT) | (keys & KEY_MASK))
        head = torch.ones(n, dtype=torch.bool, device=self.device)
        if n > 1:
            head[1:] = srt[1:] != srt[:-1]
        cum = torch.cumsum(head.long(), 0)
        uidx = cum - 1
        ubuf = torch.full((n,), -1, dtype=torch.int64, device=self.device)
        seg = torch.full((n + 1,), n, dtype=torch.int64, device=self.device)
        if n:
            native().unique_runs(srt, uidx, KEY_MASK, ubuf, seg)
        bounds = torch.searchsorted(srt, torch.arange(W + 1, device=self.device, dtype=torch.int64) << OWNER_SHIFT)
        cum0 = torch.cat([torch.zeros(1, dtype=torch.int64, device=self.device), cum])
        cnt = cum0[bounds[1:]] - cum0[bounds[:-1]]
        meta = torch.cat([torch.cumsum(cnt, 0) - cnt, cnt]).contiguous()
        inv = torch.empty(n, dtype=torch.int64, device=self.device)
        inv[perm] = uidx
        return {"n": n, "ubuf": ubuf, "meta": meta, "inv": inv, "perm": perm, "seg": seg}

    def _send(self, buf: torch.Tensor, meta: torch.Tensor, boxes, counted: bool, width: int) -> None:
        """The owners' pieces of ``buf`` into their mailboxes ``boxes[o]`` (this worker's row of
        each), on the io stream behind the compute stream."""
        io = self._io_stream
        io.wait_stream(torch.cuda.current_stream(self.device))
        buf.record_stream(io)
        meta.record_stream(io)
        ptrs = [b.data_ptr() for b in boxes]
        cnts = [b.data_ptr() + self.C * 8 for b in boxes] if counted else []
        with torch.cuda.stream(io):
            self._R.to_peers(buf, meta, ptrs, cnts, width, self.C)

    def _pull_dev(self, plan: dict) -> torch.Tensor:
        W, me, c = self.W, self.me, self.ctl
        self._ssp_gate()
        self._check_cap(plan["n"])
        self._send(plan["ubuf"], plan["meta"], [self.peer_rq[o][me] for o in range(W)], True, 1)
        self._notify.after(self._io_stream.cuda_stream, self.device.index, [c.req(o, me) for o in range(W)])
        self.pulls += 1
        self.shm.wait_ge([c.resp(o, me) for o in range(W)], self.pulls, c.stop, self.timeout_s)
        rows = torch.zeros(plan["n"], self.dim, dtype=torch.float32, device=self.device)
        self._R.from_peers(rows, plan["meta"], [self.peer_rs[o][me].data_ptr() for o in range(W)], self.dim, self.C)
        return rows

    def _push_dev(self, plan: dict, ug: torch.Tensor) -> None:
        W, me, c = self.W, self.me, self.ctl
        k = self.pushes
        slot = k % self.MB
        if k >= 2:  # mailbox slot k % 2 is free once push k - 2 was applied
            self.shm.wait_ge([c.pack(o, me) for o in range(W)], k - 1, c.stop, self.timeout_s)
        self._check_cap(plan["n"])
        self._send(plan["ubuf"], plan["meta"], [self.peer_pk[o][me][slot] for o in range(W)], True, 1)
        self._send(ug.contiguous(), plan["meta"], [self.peer_pg[o][me][slot] for o in range(W)], False, self.dim)
        self._notify.after(self._io_stream.cuda_stream, self.device.index, [c.pseq(o, me) for o in range(W)])
        self.pushes += 1

    def lookup(self, ids: torch.Tensor, out_dtype=None, grad_fn=None) -> torch.Tensor:
        if not self.gpu:
            return super().lookup(ids, out_dtype, grad_fn)
        plan = self._route_dev(self._keys_dev(ids))
        want_grad = torch.is_grad_enabled()
        if want_grad:
            # the round's lookups leave as ONE merged push: check its bound now, before this pull,
            # rather than in push_pending after the round's pulls already went out
            merged = plan["n"] + sum(p["dev"]["n"] for p in self._pending) + sum(d["n"] for d, _ in
                                                                               getattr(self, "_held", []))
            self._check_cap(merged, "merged push")
        rows = self._pull_dev(plan)
        leaf = rows.detach().requires_grad_(want_grad)
        out = _sp.gather_unique(leaf, plan["inv"], plan["perm"], plan["seg"], out_dtype)
        if want_grad:
            self._pending.append({"dev": plan, "leaf": leaf, "grad_fn": grad_fn, "plan": _DevPlan(plan["seg"])})
        return out.view(*ids.shape, self.dim)

    def pull(self, ids: torch.Tensor) -> torch.Tensor:
        if not self.gpu:
            return super().pull(ids)
        plan = self._route_dev(self._keys_dev(ids))
        out = self._pull_dev(plan)[plan["inv"]]
        return out if self.fields == 1 else out.view(*ids.shape, self.dim)

    def push(self, ids: torch.Tensor, grads: torch.Tensor) -> None:
        if not self.gpu:
            return super().push(ids, grads)
        plan = self._route_dev(self._keys_dev(ids))
        ug = torch.zeros(plan["n"], self.dim, dtype=torch.float32, device=self.device)
        _sp.segment_reduce_rows(grads.to(self.device).float().reshape(plan["n"], self.dim).contiguous(), plan["perm"],
                                plan["seg"], ug, False)
        self._push_dev(plan, ug)
        self.round += 1

    def _push_pending_dev(self) -> int:
        items = []
        for p in self._pending:
            leaf = p["leaf"]
            if leaf.grad is None:
                continue
            g = leaf.grad.detach().float()
            if p["grad_fn"] is not None:
                g = p["grad_fn"](g, p["plan"])
            items.append((p["dev"], g))
        self._pending = []
        if self.accumulating:  # micro-batches: keep them for the round's one push
            self._held = getattr(self, "_held", []) + items
            return sum(d["n"] for d, _ in items)
        items = getattr(self, "_held", []) + items
        self._held = []
        if len(items) == 1:
            plan, ug = items[0]
        elif items:  # several lookups this round: merge into ONE push (pads carry key -1)
            keys = torch.cat([d["ubuf"] for d, _ in items])
            g = torch.cat([x for _, x in items]).contiguous()
            plan = self._route_dev(keys)
            ug = torch.zeros(plan["n"], self.dim, dtype=torch.float32, device=self.device)
            _sp.segment_reduce_rows(g, plan["perm"], plan["seg"], ug, False)
        else:  # nothing looked up: an empty push still advances this worker's row clock
            plan = self._route_dev(torch.empty(0, dtype=torch.int64, device=self.device))
            ug = torch.zeros(0, self.dim, dtype=torch.float32, device=self.device)
        self._push_dev(plan, ug)
        self.round += 1
        return sum(d["n"] for d, _ in items)

    # ------------------------------------------------------------------ owner side
    def _serve(self, op: str, worker: int, n: int, m: int) -> None:
        """Row-service callback (native thread, GIL held): the owner's work for one request."""
        ctx = torch.cuda.stream(self._svc_stream) if self.gpu else _Null()
        with ctx, torch.no_grad():
            if op == "pull":
                if n:
                    keys = self.rq[worker][:n]
                    slots = self.shard.slots(keys, insert=True)
                    self.rs[worker][:n].copy_(self.shard.read(slots, keys))
            elif op == "push":
                if n:
                    keys = self.pk[worker][m][:n]
                    slots = self.shard.slots(keys, insert=True)
                    self.shard.apply(slots, self.pg[worker][m][:n], 1.0 / self.W, self.applied + 1, sorted_runs=False)
                self.applied += 1
            else:
                raise ValueError(op)
            if self.gpu:
                self._svc_stream.synchronize()
                self.shard.check()

    def clocks(self):
        """Row pushes deposited by every worker (its row clock)."""
        return [self.shm.ld(self.ctl.pseq(0, w)) for w in range(self.W)]

    # ------------------------------------------------------------------ lifecycle
    def synchronize(self) -> None:
        """Wait until every owner applied every row push of this worker (and, GPU, raise on ids
        out of range since the last check)."""
        c = self.ctl
        if self.gpu:
            self._notify.drain()
        try:
            self.shm.wait_ge([c.pack(o, self.me) for o in range(self.W)], self.pushes, c.stop, self.timeout_s)
        finally:
            err = self.service.error() if (self.gpu and self.service is not None) else ""
            if err:  # the owner service stopped the table (e.g. its hash map is full): say why
                raise RuntimeError(f"async row table {self.name}: owner service failed: {err}")
        if self.gpu:
            self.shard.check()  # this rank's own shard: overflow of its device hash map
        if self.gpu and self._nbad is not None:
            nb = int(self._nbad.item())
            self._nbad = None
            if nb:
                raise IndexError(f"{self.name}: {nb} ids out of range for id_mode={self.id_mode!r}")

    def state_dict(self) -> dict:
        self.synchronize()
        self.t.barrier()
        if self.gpu:
            torch.cuda.synchronize(self.device)
        d = self.shard.state_dict()
        d["applied"] = self.service.applied if self.gpu else self.applied
        self.t.barrier()
        return d

    def load_state_dict(self, d: dict) -> None:
        self.synchronize()
        self.t.barrier()
        self.shard.load_state_dict(d)
        self.applied = int(d.get("applied", 0))
        if self.gpu:
            torch.cuda.synchronize(self.device)
            self.service.set_applied(self.applied)
        self.t.barrier()

    def close(self) -> None:
        if getattr(self, "service", None) is None:
            return
        self.synchronize()
        self.t.barrier()
        self.service.stop()
        err = self.service.error()
        self.service = None
        self.t.barrier()
        self.share.close(unlink=not self.share.threads)
        self._ctl.close()
        if self.me == 0:
            self._ctl.unlink()
        if err:
            raise RuntimeError(f"async row table {self.name}: {err}")


class _DevPlan:
    """What a reference gradient mode needs of a device lookup: occurrences per unique key."""

    def __init__(self, seg: torch.Tensor):
        self._seg = seg

    @property
    def counts(self) -> torch.Tensor:
        return (self._seg[1:] - self._seg[:-1]).clamp(min=1)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def async_table_factory(transport: Transport, device=None, seed: int = 0, staleness: Optional[int] = None,
                        capacity: int = 1 << 15):
    """Tables for the reference models under -Dconsistency=asp|ssp on the co-located servers."""
    from .sparse_table import stable_seed

    def make(name, dim, rows, init, mode=None, fields=1):
        return AsyncRowTable(name, dim, rows, transport, init=init, seed=stable_seed(name, seed), fields=fields,
                             device=device, staleness=staleness, capacity=capacity)

    return make
