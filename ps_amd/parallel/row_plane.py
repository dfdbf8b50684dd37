"""One-node sparse-row exchange over IPC-mapped memory (no RCCL all-to-alls, no host split sizes).

Reference: a batched row pull fans out per shard (store/KVStore.java:74-107 ->
net/PSRouterClient.java:60-85, 93-122 -> net/PServer.java:101-117, 143-162) and row pushes ride
the per-key push (store/KVStore.java:259).  ``ShardedSparseTable`` at W > 1 used collectives for
that: a count all-to-all, split sizes copied to the host, key / row / gradient all-to-alls.  On
one MI355X node every rank can read and write its peers' device memory directly, so here:

* every rank owns one ARENA (IPC-mapped by every peer) holding
    skeys  [cap]       int64  its unique keys of the current pull, sorted by owner
    meta   [2W]        int64  offset and count of each owner's segment in skeys
    rows   [cap, dim]  fp32   the rows of skeys (written by the owners)
    grads  [cap, dim]  fp32   its pushed gradient rows, in skeys order (read by the owners);
* pull   = the worker writes skeys / meta (device ops: counts never leave the device) and
           records an event; every owner, once every peer's event is in its stream, runs ONE
           kernel that copies its segment of every worker's keys into a [W][cap] view (pads -1,
           csrc/kernels/sparse.hip row_plane_recv_kernel), resolves slots in its device hash map
           (creating rows: deterministic lazy init keyed by the global key) and ONE kernel that
           writes the rows straight into every worker's arena at that worker's offsets
           (row_plane_send_kernel) -- W owners stream over all links at once;
* push   = the worker writes its unique gradient rows into its arena; every owner accumulates
           the W workers' rows for its slots into an fp32 accumulator in rank order (one launch
           per worker: deterministic sums, no atomics on the data; a slot first seen this round
           goes on a touched list) and applies ONE row-optimizer update per touched row
           (gradient / W) -- the BSP "sum the W pushes, then step" of the collective path.

Cross-rank ordering: a POSIX shared-memory control block holds one epoch word per (stage,
rank); a rank bumps its word right after ENQUEUEING the stage, and the consumer of a stage waits
(on the host) only until every peer's word reached the epoch -- i.e. until the peers ENQUEUED
their part -- then makes its stream wait on the peers' inter-process events (GPU processes:
hipEventInterprocess handles, csrc/plane.cpp IpcEvent; GPU thread-ranks: shared events; CPU
ranks: every stage is synchronous).  No device->host copy of a count or size anywhere.  Every
reuse of a buffer is ordered by a wait on the stage that last read it (pull t+1 overwrites skeys
after its stream waited for the owners' rows of pull t; push t+1 overwrites grads after waiting
for every owner's accumulate of push t).

Capacity: ``cap`` keys per rank and pull (the host knows n before every pull); all ranks agree
through the control block and grow together (a collective re-map) when any rank needs more.
"""
from __future__ import annotations

import os
import time
import uuid
from typing import List, Optional

import torch

from .async_ps import _addr, _native, _ShmSeg
from .transport import Transport

_STAGES = ("n", "pub", "rows", "grd", "acc")
_HDR = 8  # magic, W, abort, max-n words per rank follow the stage words


def _round_cap(n: int) -> int:
    return max(1024, (int(n) + 1023) // 1024 * 1024)


class RowPlane:
    def __init__(self, transport: Transport, dim: int, device, timeout_s: float = 600.0):
        self.t = transport
        self.W, self.me = transport.world, transport.rank
        self.dim = int(dim)
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.threads = transport.backend == "loopback"
        self.timeout_s = float(timeout_s)
        self.shm = _native().shm
        # control block: [hdr][stage][rank] epochs + per-rank requested n
        words = _HDR + len(_STAGES) * self.W + self.W
        name = self.t.all_gather_object(f"psamd_rows_{uuid.uuid4().hex[:16]}" if self.me == 0 else None)[0]
        if self.me == 0:
            self._ctl = _ShmSeg(name, words * 8, create=True)
            base = _addr(self._ctl)
            for i in range(words):
                self.shm.st(base + 8 * i, 0)
        self.t.barrier()
        if self.me != 0:
            self._ctl = _ShmSeg(name)
        self.ctl = _addr(self._ctl)
        self.ep = {s: 0 for s in _STAGES}
        self.cap = 0
        self._arena = None
        self._seg = None
        self._opened: List[_ShmSeg] = []
        self._ev = None
        self._peer_ev = None
        self.stats = {"pulls": 0, "pushes": 0, "grows": 0, "host_syncs": 0}
        # per-stage timing (bench --timing / PS_AMD_ROWPLANE_TIMING=1): device events around each
        # stage's own work and host wall time in each cross-rank wait, plus the bytes every stage
        # moves (``timing_summary``)
        self.timing = os.environ.get("PS_AMD_ROWPLANE_TIMING", "0") == "1"
        self._tev: List[tuple] = []  # (phase, start event, end event)
        self._tsum: dict = {}
        self._tn = {"pulls": 0, "pushes": 0, "applies": 0}
        # the response rows are written into the workers' arenas by the owners' kernels: prove the
        # production write (row_plane_send) + publish (IPC events) + read (the worker's copy out)
        # before the first pull (remote_probe.py); on a failure every rank raises together and
        # the table falls back to the RCCL all-to-alls
        self.info = {}
        if self.W > 1 and not self.threads:
            try:
                self.info["remote_write_probe"] = self._probe_remote_writes()
            except Exception:
                self.close()
                raise

    def _probe_remote_writes(self, k: int = 16) -> str:
        from ..ops._ext import native
        from .remote_probe import pattern, run_probe

        W, me, dim = self.W, self.me, self.dim
        self._alloc(_round_cap(W * k))
        cap = self.cap
        rslots = torch.full((W * cap,), -1, dtype=torch.int64, device=self.device)
        for w in range(W):
            rslots[w * cap:w * cap + k] = torch.arange(k, device=self.device)
        pmeta = torch.tensor([v for _ in range(W) for v in (me * k, k)], dtype=torch.int64, device=self.device)
        tables = {}

        def write(r):
            tables[r] = pattern(r, me, k * dim).view(k, dim).to(self.device)
            if self.gpu:
                native().row_plane_send(tables[r], rslots, pmeta, [self._ptr(w, "rows") for w in range(W)], cap)
            else:  # CPU ranks: the same rows into the peers' shared-memory arenas
                for w in range(W):
                    self._peer(w, "rows", torch.float32, cap * dim).view(cap, dim)[me * k:(me + 1) * k].copy_(tables[r])

        def read(r):
            return self.rows[:W * k].clone().cpu()

        def settle():
            if self.gpu:
                torch.cuda.synchronize(self.device)
            self.t.barrier()

        rec = run_probe(self.t, "rowplane", 3, write, lambda r: self._stage("rows"), read,
                        lambda r: torch.cat([pattern(r, o, k * dim).view(k, dim) for o in range(W)]), settle)
        self.rows[:W * k].zero_()
        settle()
        return rec

    # ------------------------------------------------------------------ timing
    def _t0(self):
        """Start of a timed device phase on the current stream (None when timing is off)."""
        if not self.timing:
            return None
        if not self.gpu:
            return time.perf_counter()
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.device))
        return ev

    def _t1(self, phase: str, start) -> None:
        if start is None:
            return
        if not self.gpu:
            self._tadd(phase + "_ms", (time.perf_counter() - start) * 1e3)
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.device))
        self._tev.append((phase, start, ev))

    def _tadd(self, k: str, v: float) -> None:
        self._tsum[k] = self._tsum.get(k, 0.0) + float(v)

    def timing_summary(self, reset: bool = True) -> dict:
        """Per-pull / per-push means: device ms of each stage's own kernels (pub: key + segment
        table copies; serve: the owner's recv + slot resolve + lazy init + row send; out: the
        pulled rows copied out; grd: gradient rows into the arena; acc: the owner's rank-order
        accumulate; apply: the one row-optimizer update), host ms waiting for the peers at each
        cross-rank point (wait_*), and bytes moved per pull / push with the GB/s they imply."""
        if self.gpu and self._tev:
            torch.cuda.synchronize(self.device)  # the stages ran on the compute and side streams
        for phase, a, b in self._tev:
            self._tadd(phase + "_ms", a.elapsed_time(b))
        self._tev = []
        out = {}
        n = self._tn
        for k, v in self._tsum.items():
            if k.endswith("_bytes"):
                continue
            per = n["pulls"] if k.split("_")[0] in ("pub", "serve", "out", "wait") and not k.startswith(
                ("wait_grd", "wait_acc")) else (n["applies"] if k.startswith("apply") else n["pushes"])
            out[k] = round(v / max(1, per), 4)
        for k in ("pull_bytes", "serve_bytes", "push_bytes", "acc_bytes"):
            if k in self._tsum:
                per = n["pulls"] if k in ("pull_bytes", "serve_bytes") else n["pushes"]
                out[k] = round(self._tsum[k] / max(1, per))
        for b, t in (("serve_bytes", "serve_ms"), ("acc_bytes", "acc_ms")):
            if out.get(t):
                out[t.replace("_ms", "_GBps")] = round(out[b] / out[t] / 1e6, 2)
        out.update({k: v for k, v in n.items()})
        if reset:
            self._tsum, self._tn = {}, {"pulls": 0, "pushes": 0, "applies": 0}
        return out

    # ------------------------------------------------------------------ control words
    def _w(self, stage: str, r: int) -> int:
        return self.ctl + 8 * (_HDR + _STAGES.index(stage) * self.W + r)

    def _nw(self, r: int) -> int:
        return self.ctl + 8 * (_HDR + len(_STAGES) * self.W + r)

    def _publish(self, stage: str) -> int:
        self.ep[stage] += 1
        e = self.ep[stage]
        self.shm.st(self._w(stage, self.me), e)
        return e

    def _wait_all(self, stage: str, e: int) -> None:
        t = time.perf_counter() if self.timing else None
        self.shm.wait_ge([self._w(stage, r) for r in range(self.W)], e, self.ctl + 16, self.timeout_s)
        if t is not None:
            self._tadd(f"wait_{stage}_ms", (time.perf_counter() - t) * 1e3)

    # ------------------------------------------------------------------ arena
    def _layout(self, cap: int):
        W, dim = self.W, self.dim
        off, o = {}, 0
        for nm, nbytes in (("skeys", cap * 8), ("meta", 2 * W * 8), ("rows", cap * dim * 4), ("grads", cap * dim * 4)):
            off[nm] = o
            o = (o + nbytes + 255) // 256 * 256
        return off, o

    def _alloc(self, cap: int) -> None:
        """(Re)allocate every rank's arena for ``cap`` keys and map the peers' (collective).

        A grow frees this rank's arena and unmaps the peers': a peer's previous push
        accumulate (or row send) may still be reading / writing our arena over IPC on its own
        stream, and ``hipFree`` only waits for this process's work.  So every rank first drains
        its device and then meets the others at a barrier: after it, no kernel of any rank
        touches an old arena."""
        if self.cap > 0:
            if self.gpu:
                torch.cuda.synchronize(self.device)
            self.t.barrier()
        self._release_arena()
        self.cap = cap
        self.off, nbytes = self._layout(cap)
        if self.gpu and not self.threads:
            from .ipc_arena import IpcArena

            self._arena = IpcArena(nbytes, self.device.index)
            mine = self._arena.tensor()
            hs = self.t.all_gather_object((self._arena.handle(), self.device.index))
            bases = [self._arena.base if r == self.me else self._arena.open(h, d) for r, (h, d) in enumerate(hs)]
            self.peers = [None] * self.W
            self.bases = bases
        elif self.threads:
            mine = torch.zeros(nbytes, dtype=torch.uint8, device=self.device)
            self.peers = self.t.all_gather_object(mine)
            self.bases = [p.data_ptr() for p in self.peers]
        else:
            self._seg = _ShmSeg(f"psamd_rarena_{uuid.uuid4().hex[:16]}", nbytes, create=True)
            mine = torch.frombuffer(self._seg.buf, dtype=torch.uint8, count=nbytes)
            names = self.t.all_gather_object(self._seg.name)
            self.peers = []
            for r, nm in enumerate(names):
                if r == self.me:
                    self.peers.append(mine)
                else:
                    sg = _ShmSeg(nm)
                    self._opened.append(sg)
                    self.peers.append(torch.frombuffer(sg.buf, dtype=torch.uint8, count=nbytes))
            self.bases = [0] * self.W
        self.arena = mine
        self.skeys = self._view(mine, "skeys", torch.int64, cap)
        self.meta = self._view(mine, "meta", torch.int64, 2 * self.W)
        self.rows = self._view(mine, "rows", torch.float32, cap * self.dim).view(cap, self.dim)
        self.grads = self._view(mine, "grads", torch.float32, cap * self.dim).view(cap, self.dim)
        if self.gpu and self._ev is None:
            self._make_events()
        self.t.barrier()
        self.stats["grows"] += 1

    def _view(self, buf, nm, dt, n):
        o = self.off[nm]
        return buf[o:o + n * torch.empty((), dtype=dt).element_size()].view(dt)

    def _peer(self, r: int, nm: str, dt, n):
        return self._view(self.peers[r], nm, dt, n)

    def _ptr(self, r: int, nm: str) -> int:
        return int(self.bases[r]) + self.off[nm]

    def _make_events(self) -> None:
        if self.threads:
            evs = {s: torch.cuda.Event() for s in ("pub", "rows", "grd", "acc")}
            allev = self.t.all_gather_object(evs)
            self._ev = evs
            self._peer_ev = allev
            return
        from .. import _C  # type: ignore

        P = _C.plane
        self._ev = {s: P.IpcEvent(self.device.index) for s in ("pub", "rows", "grd", "acc")}
        hs = self.t.all_gather_object({s: e.handle() for s, e in self._ev.items()})
        self._peer_ev = [None if r == self.me else {s: P.IpcEvent(h, self.device.index) for s, h in hr.items()}
                         for r, hr in enumerate(hs)]

    def _record(self, stage: str) -> None:
        if not self.gpu:
            return
        st = torch.cuda.current_stream(self.device)
        if self.threads:
            self._ev[stage].record(st)
        else:
            self._ev[stage].record(st.cuda_stream)

    def _stream_wait_peers(self, stage: str) -> None:
        if not self.gpu:
            return
        st = torch.cuda.current_stream(self.device)
        for r in range(self.W):
            if r == self.me:
                continue
            if self.threads:
                st.wait_event(self._peer_ev[r][stage])
            else:
                self._peer_ev[r][stage].wait(st.cuda_stream)

    def _stage(self, stage: str) -> None:
        """Record this rank's stage event, publish the epoch, wait until every peer ENQUEUED
        the same stage, and order this stream after the peers' events."""
        self._record(stage)
        e = self._publish(stage)
        self._wait_all(stage, e)
        self._stream_wait_peers(stage)

    # ------------------------------------------------------------------ pull
    def pull(self, ubuf: torch.Tensor, counts: torch.Tensor, n: int, shard, fetch: bool = True):
        """Rows for this rank's ``n`` unique-key slots ``ubuf`` (owner-major, pads -1 at the
        tail; ``counts`` [W] per owner, device) -> (rows [n, dim] fp32, owner-side state for
        the matching push).  Collective."""
        # capacity agreement (host words: the sizes are host-known on every rank)
        self.shm.st(self._nw(self.me), int(n))
        e = self._publish("n")
        self._wait_all("n", e)
        need = max(self.shm.ld(self._nw(r)) for r in range(self.W))
        if need > self.cap:
            self._alloc(_round_cap(need))
        cap, W = self.cap, self.W
        # publish this rank's keys + segment table (device ops, no host copy of a count)
        t = self._t0()
        if n:
            self.skeys[:n].copy_(ubuf[:n])
        cnt = counts[:W].to(torch.int64)
        self.meta[W:].copy_(cnt)
        self.meta[:W].copy_(torch.cumsum(cnt, 0) - cnt)
        self._t1("pub", t)
        self._stage("pub")
        # owner: every worker's segment for me -> slots -> rows into the workers' arenas
        t = self._t0()
        st = self._serve(shard, fetch)
        self._t1("serve", t)
        self._stage("rows")
        t = self._t0()
        out = self.rows[:n].clone() if fetch else None
        self._t1("out", t)
        if self.timing:
            # this rank's keys out + its rows back; the owner side moves the W workers' segments
            # for it, about the same volume summed over the node
            self._tadd("pull_bytes", n * 8 + (n * self.dim * 4 if fetch else 0))
            self._tadd("serve_bytes", n * 8 + (n * self.dim * 4 if fetch else 0))
            self._tn["pulls"] += 1
        self.stats["pulls"] += 1
        return out, st

    def _serve(self, shard, fetch: bool = True):
        W, cap, me = self.W, self.cap, self.me
        if self.gpu:
            from ..ops._ext import native

            rkeys = torch.empty(W * cap, dtype=torch.int64, device=self.device)
            pmeta = torch.empty(2 * W, dtype=torch.int64, device=self.device)
            native().row_plane_recv([self._ptr(r, "skeys") for r in range(W)], [self._ptr(r, "meta") for r in range(W)],
                                    me, cap, rkeys, pmeta)
            slots = shard.slots(rkeys, insert=True)
            lo, hi = shard.init
            if lo != 0.0 or hi != 0.0:
                from ..ops import sparse as _sp

                _sp.lazy_init_rows(shard.table, slots, shard.flags, shard.seed, 0, lo, hi, keys=rkeys)
            if fetch:  # (a push-only plan needs the owners' slots, not the rows)
                native().row_plane_send(shard.table, slots, pmeta, [self._ptr(r, "rows") for r in range(W)], cap)
            return {"slots": slots, "pmeta": pmeta}
        # CPU ranks: the same steps as host-sized torch ops on the shared segments
        segs = []
        for r in range(W):
            pm = self._peer(r, "meta", torch.int64, 2 * W)
            off, c = int(pm[me]), int(pm[W + me])
            segs.append((off, c, self._peer(r, "skeys", torch.int64, cap)[off:off + c].clone()))
        keys = torch.cat([k for _, _, k in segs]) if segs else torch.empty(0, dtype=torch.int64)
        slots = shard.slots(keys, insert=True) if keys.numel() else keys
        rows = shard.read(slots, keys) if keys.numel() else torch.empty(0, self.dim)
        o = 0
        for r, (off, c, _) in enumerate(segs):
            if c:
                self._peer(r, "rows", torch.float32, cap * self.dim).view(cap, self.dim)[off:off + c].copy_(rows[o:o + c])
            o += c
        return {"slots": slots, "segs": [(off, c) for off, c, _ in segs]}

    # ------------------------------------------------------------------ push
    def push(self, ug: torch.Tensor, nu_bound: int, st: dict, shard, acc: "RowAccumulator") -> None:
        """This rank's unique gradient rows ``ug`` (skeys order, [nu_bound, dim] fp32) to their
        owners; every owner adds them into its accumulator (applied by ``acc.apply``).
        Collective."""
        W, cap = self.W, self.cap
        # every owner finished reading our previous push before the buffer is overwritten
        if self.ep["acc"] > 0:
            self._wait_all("acc", self.ep["acc"])
            self._stream_wait_peers("acc")
        t = self._t0()
        if nu_bound:
            self.grads[:nu_bound].copy_(ug[:nu_bound])
        self._t1("grd", t)
        self._stage("grd")
        if self.timing:
            self._tadd("push_bytes", nu_bound * self.dim * 4)
            self._tadd("acc_bytes", nu_bound * self.dim * 4 * 3)  # read grads, read + write acc
            self._tn["pushes"] += 1
        if self.gpu:
            t = self._t0()
            acc.add_gpu(self, st)
            self._t1("acc", t)
        else:
            parts = []
            for r, (off, c) in enumerate(st["segs"]):
                parts.append(self._peer(r, "grads", torch.float32, cap * self.dim).view(cap, self.dim)[off:off + c].clone())
            acc.add_cpu(st["slots"], torch.cat(parts) if parts else torch.empty(0, self.dim))
        self._record("acc")
        self._publish("acc")
        self.stats["pushes"] += 1

    # ------------------------------------------------------------------ teardown
    def _release_arena(self) -> None:
        if self._arena is not None:
            self._arena.close()
            self._arena = None
        for s in self._opened:
            s.close()
        self._opened = []
        if self._seg is not None:
            self._seg.close()
            self._seg.unlink()
            self._seg = None

    def close(self) -> None:
        if self.gpu:
            torch.cuda.current_stream(self.device).synchronize()
        self.t.barrier()
        self._release_arena()
        if self._ctl is not None:
            self._ctl.close()
            if self.me == 0:
                self._ctl.unlink()
            self._ctl = None


class RowAccumulator:
    """Owner-side sum of the W workers' pushed rows per slot (rank order), then one optimizer
    update per touched row (shard.apply semantics: gradient * gscale, step counter)."""

    def __init__(self, shard):
        self.shard = shard
        self.open = False
        self.tag = 0
        if shard.gpu:
            self.acc = torch.zeros_like(shard.table)
            self.tflag = torch.zeros(shard.capacity, dtype=torch.int32, device=shard.device)
            self.touched = torch.full((shard.capacity,), -1, dtype=torch.int64, device=shard.device)
            self.tcount = torch.zeros(1, dtype=torch.int32, device=shard.device)
        self._cpu: List[tuple] = []

    def _begin(self) -> None:
        if not self.open:
            self.open = True
            self.tag += 1
            if self.shard.gpu:
                self.touched.fill_(-1)
                self.tcount.zero_()

    def add_gpu(self, plane: RowPlane, st: dict) -> None:
        from ..ops._ext import native

        self._begin()
        native().row_plane_accum([plane._ptr(r, "grads") for r in range(plane.W)], st["slots"], st["pmeta"], self.acc,
                                 self.tflag, self.tag, self.touched, self.tcount, plane.cap)

    def add_cpu(self, slots: torch.Tensor, g: torch.Tensor) -> None:
        self._begin()
        self._cpu.append((slots, g))

    def apply(self, gscale: float, step: int, plane: Optional[RowPlane] = None) -> None:
        if not self.open:
            return
        self.open = False
        t = plane._t0() if plane is not None else None
        self._apply(gscale, step)
        if t is not None:
            plane._t1("apply", t)
            plane._tn["applies"] += 1

    def _apply(self, gscale: float, step: int) -> None:
        sh = self.shard
        if sh.gpu:
            u = sh.updater
            skip = getattr(u, "mode", "") == "reference"
            # the touched list is capacity-sized; its live length is the device count tcount
            u.step_rows(sh.table, sh.states, self.touched, self.acc, gscale=gscale, step=step,
                        rowwise=getattr(u, "rowwise", False), skip_zero=skip, perm=self.touched, ncount=self.tcount)
            return
        slots = torch.cat([s for s, _ in self._cpu])
        g = torch.cat([x for _, x in self._cpu])
        self._cpu = []
        sh.apply(slots, g, gscale, step, sorted_runs=True)


def plane_rows_wanted(transport: Transport, device, req: Optional[str] = None) -> bool:
    """Choice of the one-node row exchange.  ``req`` (default PS_AMD_ROW_EXCHANGE, else "auto"):
    "auto" takes the IPC / shared-memory plane when every rank is on this host, "plane" insists
    on it (raises across hosts), "collective" keeps the all-to-all path."""
    req = req or os.environ.get("PS_AMD_ROW_EXCHANGE", "auto")
    if req == "collective" or transport.world <= 1:
        return False
    import socket

    hosts = transport.all_gather_object(socket.gethostname())
    same = len(set(hosts)) == 1
    if req == "plane" and not same:
        raise RuntimeError("PS_AMD_ROW_EXCHANGE=plane needs every rank on one host")
    from .. import _C  # noqa: F401  -- the kernels / IPC handles live in the extension

    return same and transport.world <= 16
