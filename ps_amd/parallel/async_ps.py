"""Asynchronous parameter server: ASP and SSP(s) without lockstep collectives.

Reference: the async PServer applies each push the moment it arrives and the barrier returns
at once (net/PServer.java:176-184, 242-248; the worker only pushes fire-and-forget,
net/PSClient.java:159-161) -- Hogwild, no staleness bound.  SURVEY §2.3 row 3 / §5.8 asks for
a per-GPU server progress thread and bounded staleness (SSP).

MI355X-native design (one node, one process per GPU, or threads / CPU processes in tests):

* the flat parameter space (laid out in BACKWARD order, cut into 64-element-aligned buckets) is
  range-partitioned; rank r OWNS shard r: fp32 master + the optimizer state of every updater
  SEGMENT (per-key-prefix updaters resolved exact -> longest prefix -> default, as
  store/KVStore.java:242-252 -- e.g. FTRL on ``wide.*`` and Adam elsewhere), 2 gradient
  MAILBOXES per worker (push k lands in slot k % 2) and 3 PUBLISHED weight slots, all in its HBM;
* push  = as soon as a bucket's last gradient is accumulated (autograd hook) the worker lands it
          in its gradient flat and ONE copy kernel (csrc/kernels/plane.hip) writes the bucket's
          pieces straight into the owners' IPC-mapped mailboxes -- all owners' links at once --
          on a side stream; at ``finish_step`` a native completion thread bumps seq[r][w] once
          every copy landed.  The training thread never waits for a copy, and waits for an
          owner only if that owner has not yet applied the worker's push from TWO steps ago;
* serve = a NATIVE progress thread per owner (csrc/async_ps_gpu.cpp; CPU: csrc/runtime)
          polls the shared control block, runs the fused HIP optimizer of every segment on each
          deposited push in arrival order (Hogwild-style, one update per push, gradient scaled
          by 1/W), writes the new weights into a free slot, publishes it and acknowledges;
* pull  = the worker pins every owner's current slot (the owner never overwrites a pinned
          slot: no torn reads) and ONE copy kernel on a pull stream fills the BACK replica
          buffer; the compute stream waits on that copy (the host does not), then the buffers
          swap -- the pull overlaps the tail of the step that still reads the front buffer;
* SSP(s): before pulling at clock c the worker waits until every owner has APPLIED every
          worker's first c - s pushes (so the weights read contain all updates older than
          s steps); s = 0 is BSP semantics without any collective, ``staleness=None`` is ASP.

No rank ever blocks on another rank reaching a matching collective: a slow worker only slows
the others through the staleness bound (SSP) or not at all (ASP).  The control block lives in
POSIX shared memory (csrc/include/async_ctl.h); buffers are exchanged once at start-up through
the transport's object all-gather (CUDA IPC handles between processes, named shared memory for
CPU processes, plain tensors between loopback thread-ranks).  Sparse rows take the same
one-sided path (parallel/async_rows.py).
"""
from __future__ import annotations

import os
import uuid
from functools import partial
from typing import Dict, List, Optional, Union

import torch

from ..obs import trace as _trace
from ..ops import optim as _o
from ..ops import side_stream as _side
from .transport import Transport, side_stream
from .updaters import AdamUpdater, Updater, resolve_updater

_BIAS_MODE = {"none": 0, "step": 1, "reference": 2}


def _native():
    from .. import _native  # type: ignore

    return _native


class _ShmSeg:
    """A POSIX shared-memory segment (/dev/shm) mapped into this process -- created by one rank,
    opened by name by the others.  No multiprocessing resource tracker: only the creator
    unlinks, so ranks spawned from one parent cannot unregister each other's segments."""

    def __init__(self, name: str, size: int = 0, create: bool = False):
        import mmap

        self.name = name.lstrip("/")
        path = "/dev/shm/" + self.name
        flags = os.O_RDWR | (os.O_CREAT | os.O_EXCL if create else 0)
        fd = os.open(path, flags, 0o600)
        try:
            if create:
                os.ftruncate(fd, max(1, size))
            self.size = os.fstat(fd).st_size
            self.buf = mmap.mmap(fd, self.size)
        finally:
            os.close(fd)
        self.created = create

    def close(self) -> None:
        try:
            self.buf.close()
        except BufferError:  # tensors still view it: the mapping goes with the process
            pass

    def unlink(self) -> None:
        try:
            os.unlink("/dev/shm/" + self.name)
        except FileNotFoundError:
            pass


class _Shared:
    """Allocate buffers other ranks can map, and open theirs (see module docstring)."""

    def __init__(self, transport: Transport, device: torch.device):
        self.t = transport
        self.device = device
        self.threads = transport.backend == "loopback"
        self._segs = []  # SharedMemory segments this rank created (kept alive, unlinked at close)
        self._opened = []  # segments of other ranks mapped here

    def alloc(self, shape, dtype) -> torch.Tensor:
        if self.device.type == "cuda" or self.threads:
            return torch.zeros(shape, dtype=dtype, device=self.device)
        n = 1
        for s in shape:
            n *= s
        nbytes = max(1, n * torch.tensor([], dtype=dtype).element_size())
        seg = _ShmSeg(f"psamd_{uuid.uuid4().hex[:20]}", nbytes, create=True)
        self._segs.append(seg)
        t = torch.frombuffer(seg.buf, dtype=dtype, count=n).view(*shape)
        t.zero_()
        return t

    def _handle(self, t: torch.Tensor):
        if self.threads:
            return t
        if t.is_cuda:
            from torch.multiprocessing.reductions import reduce_tensor

            return ("cuda",) + reduce_tensor(t)
        seg = next(s for s in self._segs if t.data_ptr() == _addr(s))
        return ("shm", seg.name, tuple(t.shape), str(t.dtype).replace("torch.", ""))

    def _open(self, h):
        if isinstance(h, torch.Tensor):
            return h
        if h[0] == "cuda":
            fn, args = h[1], h[2]
            return fn(*args)
        _, name, shape, dt = h
        seg = _ShmSeg(name)
        self._opened.append(seg)
        dtype = getattr(torch, dt)
        n = 1
        for s in shape:
            n *= s
        return torch.frombuffer(seg.buf, dtype=dtype, count=n).view(*shape)

    def exchange(self, t: torch.Tensor) -> List[torch.Tensor]:
        """Every rank's buffer ``t`` (its own is returned as is)."""
        hs = self.t.all_gather_object(self._handle(t))
        return [t if r == self.t.rank else self._open(h) for r, h in enumerate(hs)]

    def close(self, unlink: bool) -> None:
        for s in self._opened + self._segs:
            try:
                s.close()
            except Exception:  # noqa: BLE001 -- best effort at shutdown (views may still exist)
                pass
        if unlink:
            for s in self._segs:
                try:
                    s.unlink()
                except Exception:  # noqa: BLE001
                    pass
        self._segs, self._opened = [], []


def _addr(seg) -> int:
    import ctypes

    return ctypes.addressof(ctypes.c_char.from_buffer(seg.buf))


class AsyncPS:
    """Drop-in for ColocatedPS when the consistency mode is ASP or SSP-without-lockstep:
    gradients leave bucket by bucket from the backward hooks (one-sided copies into the owners'
    mailboxes), ``finish_step()`` closes the push and pulls what the staleness bound allows into
    the back replica buffer; parameters are views of the front buffer."""

    def __init__(self, model: torch.nn.Module, updaters: Union[Updater, Dict[str, Updater]],
                 transport: Optional[Transport] = None, *, staleness: Optional[int] = None,
                 gscale: Optional[float] = None, timeout_s: float = 600.0, bucket_mb: float = 25.0,
                 overlap: bool = True):
        self.model = model
        self.t = transport or Transport()
        self.world, self.rank = self.t.world, self.t.rank
        W, me = self.world, self.rank
        self.umap = updaters if isinstance(updaters, dict) else {"default": updaters}
        params = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        if not params:
            raise ValueError("model has no trainable parameters")
        dtypes = {p.dtype for _, p in params}
        if len(dtypes) != 1:
            raise ValueError("AsyncPS needs one parameter dtype")
        self.dtype = dtypes.pop()
        self.device = params[0][1].device
        self.gpu = self.device.type == "cuda"
        if not self.gpu and self.dtype != torch.float32:
            raise ValueError("CPU AsyncPS shards are fp32")
        self.staleness = staleness
        self.timeout_s = timeout_s
        # SSP audit: set to a list to record (clock, gate target, min ack seen) per gated pull --
        # AsyncRowTable.gate_log records the same triple for the rows (one round window for both)
        self.gate_log: Optional[list] = None
        self.gscale = (1.0 / W) if gscale is None else float(gscale)
        self.params = dict(params)
        self.overlap = overlap
        self.threads = self.t.backend == "loopback"
        # ---------------- flat layout in BACKWARD order, cut into buckets (64-element aligned
        # starts, so every piece of a bucket copy is 16-B aligned)
        esz = torch.empty((), dtype=self.dtype).element_size()
        cap = max(64, int(bucket_mb * 2**20) // esz)
        self.offsets: Dict[str, tuple] = {}
        self.buckets: List[List[str]] = []
        self.bucket_range: List[tuple] = []
        off, cur, start = 0, [], 0
        for nme, p in reversed(params):
            if cur and off - start + p.numel() > cap:
                self.buckets.append(cur)
                self.bucket_range.append((start, off))
                off = (off + 63) // 64 * 64
                cur, start = [], off
            self.offsets[nme] = (off, p.numel(), p.shape)
            cur.append(nme)
            off += p.numel()
        self.buckets.append(cur)
        self.bucket_range.append((start, off))
        self._key_bucket = {n: b for b, ks in enumerate(self.buckets) for n in ks}
        self.L = ((off + W - 1) // W + 63) // 64 * 64
        L = self.L
        # ---------------- double-buffered replica + gradient flat (parameters are views)
        self.flats = [torch.zeros(W * L, dtype=self.dtype, device=self.device) for _ in range(2)]
        self.cur = 0
        self.gflat = torch.zeros(W * L, dtype=self.dtype, device=self.device)
        with torch.no_grad():
            for nme, p in params:
                o, n, _ = self.offsets[nme]
                self.flats[0][o:o + n].copy_(p.detach().reshape(-1))
            self.t.broadcast(self.flats[0], src=0)
            self.flats[1].copy_(self.flats[0])
        self._bind()
        # ---------------- owner shard: fp32 master + per-key-prefix updater segments
        self.share = _Shared(self.t, self.device)
        lo = me * L
        self.master = self.flats[0][lo:lo + L].float().clone()
        self.segs = self._segments(lo, lo + L)  # [(updater, a, z)] shard-local
        self.states = [u.new_states(self.master[a:z]) for (u, a, z) in self.segs] if self.gpu else []
        A = _native().async_ctl
        self.MB = A.MBOX()
        self.mbox = self.share.alloc((W * self.MB, L), self.dtype)
        self.pub = self.share.alloc((3, L), self.dtype)
        with torch.no_grad():
            self.pub.copy_(self.flats[0][lo:lo + L].expand(3, L))
        # control block: rank 0 creates the shared segment, everyone maps it
        name = self.t.all_gather_object(f"psamd_ctl_{uuid.uuid4().hex[:16]}" if me == 0 else None)[0]
        if me == 0:
            self._ctl = _ShmSeg(name, A.SIZE, create=True)
            A.init(_addr(self._ctl), W)
        self.t.barrier()
        if me != 0:
            self._ctl = _ShmSeg(name)
        self.ctl = _addr(self._ctl)
        if not A.valid(self.ctl):
            raise RuntimeError("async PS control block not initialised")
        self.A = A
        self.peer_mbox = self.share.exchange(self.mbox)
        self.peer_pub = self.share.exchange(self.pub)
        # one-sided pushes write into the owners' HBM: prove the production write + read path on
        # the mailbox lines themselves before relying on it (remote_probe.py); every rank raises
        # RemoteWriteUnavailable together on a failure and the caller falls back
        self.info = {"engine": "AsyncPS"}
        if W > 1 and not self.threads:
            try:
                self.info["remote_write_probe"] = self._probe_remote_writes()
            except Exception:
                self.share.close(unlink=True)
                self._ctl.close()
                if me == 0:
                    self._ctl.unlink()
                raise
        # ---------------- native progress thread (owner) + completion thread (worker)
        if self.gpu:
            from .. import _C  # type: ignore

            self._C = _C
            self.server = _C.GpuAsyncServer(self.ctl, me, self.master, [self.mbox[i] for i in range(W * self.MB)],
                                            [self.pub[s] for s in range(3)], self.gscale)
            for (u, a, z), st in zip(self.segs, self.states):
                h = _o._hp(u.hyper(1))
                bias = _BIAS_MODE[u.bias_correction] if isinstance(u, AdamUpdater) else 0
                st2 = list(st) + [None] * (2 - len(st))
                self.server.add_segment(u.kind, a, z, st2[0], st2[1], [float(h[k]) for k in _HYPER], bias)
            self.notifier = _C.GpuNotifier(self.ctl)
            self.push_stream = side_stream(self.device)
            self.pull_stream = torch.cuda.Stream(device=self.device)
            self._done_ev: List[Optional[torch.cuda.Event]] = [None, None]
        else:
            self.server = _native().CpuAsyncServer(
                self.ctl, me, L, self.master.data_ptr(), [self.mbox[i].data_ptr() for i in range(W * self.MB)],
                [self.pub[s].data_ptr() for s in range(3)], self.gscale)
            for u, a, z in self.segs:
                self.server.add_segment(u.name, a, z)
            self.notifier = None
        self.t.barrier()
        self.server.start()
        self.clock = 0
        self.round = 0
        self.accumulating = False
        self.stats = {"gate_waits": 0, "bucket_pushes": 0}
        self._pending = [len(ks) for ks in self.buckets]
        self._launched = [False] * len(self.buckets)
        self._landing: List[Dict[str, torch.Tensor]] = [dict() for _ in self.buckets]
        self._step_open = False
        self._hooks = ([p.register_post_accumulate_grad_hook(partial(self._on_ready, n)) for n, p in params]
                       if overlap else [])

    def _probe_remote_writes(self) -> str:
        """Every rank writes a pattern into the first 64 elements of its slot-0 mailbox row on every
        owner by the push's copy kernel; the owner reads its W - 1 rows by the serve's acquire
        kernel once the writers' completion was observed on the host (the control-block seq
        protocol) -- three rounds over the same lines, then the lines are zeroed again."""
        from .remote_probe import pattern, run_probe

        W, me, MB, n = self.world, self.rank, self.MB, 64
        peers = [w for w in range(W) if w != me]
        if self.gpu:
            from .. import _C  # type: ignore

            P = _C.plane
            ws, rs = torch.cuda.Stream(device=self.device), torch.cuda.Stream(device=self.device)
            out = torch.zeros(W, n, dtype=torch.float32, device=self.device)
            srcs = {}

            def write(k):
                src = srcs[k] = pattern(k, me, n).to(self.device, self.dtype)
                ws.wait_stream(torch.cuda.current_stream(self.device))
                es = src.element_size()
                P.copy_many([(src.data_ptr(), self.peer_mbox[r][me * MB].data_ptr(), n * es) for r in peers],
                            ws.cuda_stream, self.device.index)

            def publish(k):
                ws.synchronize()  # the host observed every copy's completion (as the notifier does)
                self.t.barrier()

            def read(k):
                for w in peers:
                    P.read_acquire(self.mbox[w * MB].data_ptr(), n, self.dtype == torch.bfloat16, out[w],
                                   rs.cuda_stream)
                rs.synchronize()
                return out[peers].cpu()

            def settle():
                torch.cuda.synchronize(self.device)
                self.t.barrier()
        else:
            def write(k):
                src = pattern(k, me, n).to(self.dtype)
                for r in peers:
                    self.peer_mbox[r][me * MB][:n].copy_(src)

            def publish(k):
                self.t.barrier()

            def read(k):
                return torch.stack([self.mbox[w * MB][:n].float().clone() for w in peers])

            def settle():
                self.t.barrier()

        rec = run_probe(self.t, "asyncps", 3, write, publish, read,
                        lambda k: torch.stack([pattern(k, w, n) for w in peers]), settle)
        with torch.no_grad():
            for w in peers:
                self.mbox[w * MB][:n].zero_()
        if self.gpu:
            torch.cuda.synchronize(self.device)
        self.t.barrier()
        return rec

    def _segments(self, lo: int, hi: int) -> List[tuple]:
        """Updater segments of the shard [lo, hi): exact key -> longest prefix -> default per key
        (store/KVStore.java:242-252), adjacent runs merged, padding given to its neighbours."""
        segs: List[tuple] = []
        for nme, (o, n, _) in sorted(self.offsets.items(), key=lambda kv: kv[1][0]):
            a, z = max(o, lo), min(o + n, hi)
            if a >= z:
                continue
            u = resolve_updater(nme, self.umap)
            if segs and segs[-1][0] is u:
                segs[-1] = (u, segs[-1][1], z - lo)
            else:
                if segs:  # a gap (bucket padding) belongs to the previous segment
                    segs[-1] = (segs[-1][0], segs[-1][1], a - lo)
                segs.append((u, a - lo, z - lo))
        if not segs:  # pure padding shard
            return [(resolve_updater(next(iter(self.offsets)), self.umap), 0, hi - lo)]
        segs[0] = (segs[0][0], 0, segs[0][2])
        segs[-1] = (segs[-1][0], segs[-1][1], hi - lo)
        return segs

    # ------------------------------------------------------------------ views
    def _bind(self) -> None:
        fl = self.flats[self.cur]
        for nme, p in self.params.items():
            off, n, shape = self.offsets[nme]
            p.data = fl[off:off + n].view(shape)
            p.grad = None

    def weight(self, name: str) -> torch.Tensor:
        off, n, shape = self.offsets[name]
        return self.flats[self.cur][off:off + n].view(shape)

    @property
    def flat(self) -> torch.Tensor:
        return self.flats[self.cur]

    # ------------------------------------------------------------------ push path
    def push_key(self, name: str, grad: torch.Tensor) -> None:
        """Key-level push (parallel/gpu_kvstore.py), as ColocatedPS.push_key."""
        p = self.params[name]
        b = self._key_bucket[name]
        g = grad.detach().to(device=p.device, dtype=p.dtype).reshape(p.shape)
        if name in self._landing[b]:
            self._landing[b][name] = self._landing[b][name] + g
            return
        if self._launched[b]:
            raise RuntimeError(f"key {name!r} was already pushed this round (its bucket has left)")
        p.grad = g
        if self.overlap:
            self._on_ready(name, p)
        else:
            self._landing[b][name] = g

    def _on_ready(self, name: str, p: torch.Tensor) -> None:
        if self.accumulating:
            return
        b = self._key_bucket[name]
        if name not in self._landing[b]:
            self._pending[b] -= 1
        self._landing[b][name] = p.grad
        if self._pending[b] == 0:
            self._push_bucket(b)

    def _open_step(self) -> None:
        """Before the first bucket of push ``clock`` leaves: the mailbox slot it lands in
        (clock % 2) must be free on every owner -- push clock - 2 applied, i.e. ack >= clock - 1
        (we gate on our OWN push count: seq lags behind on GPU).  The previous push's copies
        must have read gflat before it is overwritten."""
        if self._step_open:
            return
        self._step_open = True
        if self.clock >= 2:
            for r in range(self.world):
                self.A.wait_ack(self.ctl, r, self.rank, self.clock - 1, self.timeout_s)
        if self.gpu:
            torch.cuda.current_stream(self.device).wait_stream(self.push_stream)

    def _push_bucket(self, b: int) -> None:
        if self._launched[b]:
            return
        self._launched[b] = True
        self._open_step()
        if self.gpu:  # weight gradients still in flight on the side stream (ops/side_stream.py)
            _side.join(device=self.device)
        parked = self._landing[b]
        lo, hi = self.bucket_range[b]
        L, MB, me = self.L, self.MB, self.rank
        slot = self.clock % MB
        own_lo, own_hi = me * L, (me + 1) * L
        own_box = self.mbox[me * MB + slot]
        dst, src = [], []

        def land(view_off, n, g):
            # the piece this rank owns lands straight in its own mailbox slot (no copy); the
            # rest in the gradient flat, from where one kernel sends it to the other owners
            for a, z in ((view_off, min(view_off + n, own_lo)), (max(view_off, own_lo), min(view_off + n, own_hi)),
                         (max(view_off, own_hi), view_off + n)):
                if a >= z:
                    continue
                v = own_box[a - own_lo:z - own_lo] if own_lo <= a < own_hi else self.gflat[a:z]
                if g is None:
                    v.zero_()
                else:
                    dst.append(v)
                    src.append(g[a - view_off:z - view_off])

        for nme in self.buckets[b]:
            off, n, _ = self.offsets[nme]
            g = parked.get(nme)
            land(off, n, None if g is None else g.reshape(-1))
            self.params[nme].grad = None
        if dst:
            torch._foreach_copy_(dst, src)
        self._landing[b] = {}
        pieces = []
        for r in range(self.world):
            a, z = max(lo, r * L), min(hi, (r + 1) * L)
            if a < z and r != me:
                pieces.append((r, a, z))
        if self.gpu:
            self.push_stream.wait_stream(torch.cuda.current_stream(self.device))
            if not pieces:
                self.stats["bucket_pushes"] += 1
                return
            es = self.gflat.element_size()
            segs = [(self.gflat.data_ptr() + a * es,
                     self.peer_mbox[r][me * MB + slot].data_ptr() + (a - r * L) * es, (z - a) * es)
                    for r, a, z in pieces]
            with torch.cuda.stream(self.push_stream):
                self._C.plane.copy_many(segs, self.push_stream.cuda_stream, self.device.index)
        else:
            for r, a, z in pieces:
                self.peer_mbox[r][me * MB + slot][a - r * L:z - r * L].copy_(self.gflat[a:z])
        self.stats["bucket_pushes"] += 1

    def finish_step(self) -> None:
        """Close this step's push (buckets the hooks did not send leave now; the owners see it
        once every copy landed), advance the clock, and pull the newest weights the staleness
        bound allows into the back buffer."""
        if self.accumulating:
            return
        with _trace.range(f"async_ps.step.c{self.clock}"):
            self._finish_step()

    def _finish_step(self) -> None:
        W, me, A = self.world, self.rank, self.A
        if not self.overlap:  # gradients were accumulated into p.grad: park them all now
            for nme, p in self.params.items():
                b = self._key_bucket[nme]
                self._landing[b][nme] = p.grad
        for b in range(len(self.buckets)):
            self._push_bucket(b)
        if self.gpu:
            self.notifier.after(self.push_stream.cuda_stream, self.device.index, list(range(W)), me, True, [])
        else:
            for r in range(W):
                A.bump_seq(self.ctl, r, me)
            A.bump_clock(self.ctl, me)
        self.clock += 1
        self.round += 1
        self._pending = [len(ks) for ks in self.buckets]
        self._launched = [False] * len(self.buckets)
        self._step_open = False
        self._pull()

    def _pull(self, gate: bool = True) -> None:
        """Copy every owner's current published slot (pinned: never overwritten while read) into
        the BACK replica buffer with one kernel, then make it the front buffer: the compute stream
        waits on the copy, the host does not."""
        W, L, A = self.world, self.L, self.A
        if gate and self.staleness is not None:
            target = self.clock - int(self.staleness)
            A.wait_min_ack(self.ctl, target, self.timeout_s)
            if self.gate_log is not None:
                self.gate_log.append((self.clock, target, min(min(r) for r in A.snapshot(self.ctl)["ack"])))
        pins = [(r, A.pin(self.ctl, r)) for r in range(W)]
        back = 1 - self.cur
        dst = self.flats[back]
        if self.gpu:
            comp = torch.cuda.current_stream(self.device)
            ev = self._done_ev[back]
            if ev is not None:  # the step that last read the back buffer is done with it
                self.pull_stream.wait_event(ev)
            es = dst.element_size()
            segs = [(self.peer_pub[r][s].data_ptr(), dst.data_ptr() + r * L * es, L * es) for r, s in pins]
            with torch.cuda.stream(self.pull_stream):
                self._C.plane.copy_many(segs, self.pull_stream.cuda_stream, self.device.index)
            self.notifier.after(self.pull_stream.cuda_stream, self.device.index, [], self.rank, False, pins)
            done = torch.cuda.Event()
            done.record(comp)  # everything issued so far on the front buffer
            self._done_ev[self.cur] = done
            comp.wait_stream(self.pull_stream)
        else:
            with torch.no_grad():
                for r, s in pins:
                    dst[r * L:(r + 1) * L].copy_(self.peer_pub[r][s])
            for r, s in pins:
                A.unpin(self.ctl, r, s)
        self.cur = back
        self._bind()

    # ------------------------------------------------------------------ control
    def snapshot(self) -> dict:
        return self.A.snapshot(self.ctl)

    def synchronize(self, collective: bool = False) -> None:
        """Wait until every push of THIS worker has been applied by every owner, then pull.
        ``collective`` (every rank calls it): then a barrier and a second pull, so the replica
        holds every worker's pushes -- without it a faster rank's replica may still miss a slower
        rank's last push."""
        if self.gpu:
            torch.cuda.current_stream(self.device).synchronize()
            self.push_stream.synchronize()
            self.notifier.drain()
        import time

        t0 = time.time()
        while True:
            snap = self.A.snapshot(self.ctl)
            if all(snap["ack"][r][self.rank] >= self.clock for r in range(self.world)):
                break
            if time.time() - t0 > self.timeout_s:
                raise RuntimeError("async PS: pushes not applied in time")
            time.sleep(0.0005)
        self._pull()
        if self.gpu:
            torch.cuda.current_stream(self.device).synchronize()
            self.notifier.drain()
        if collective and self.world > 1:
            self.t.barrier()  # every rank's pushes are applied everywhere
            self._pull(gate=False)
            if self.gpu:
                torch.cuda.current_stream(self.device).synchronize()
                self.notifier.drain()

    # ------------------------------------------------------------------ checkpoint
    def _state_list(self) -> List[torch.Tensor]:
        if self.gpu:
            return [s for st in self.states for s in st]
        return [torch.from_numpy(a) for a in self.server.states()]

    def shard_state(self) -> dict:
        """This owner's shard (fp32 master, optimizer state per updater segment, update count)
        at a QUIESCENT point: every rank calls it at the same step boundary; after the barrier no
        push is in flight."""
        self.synchronize()
        self.t.barrier()
        version = int(self.A.snapshot(self.ctl)["version"][self.rank])
        snap = {"rank": self.rank, "world": self.world, "round": self.round, "clock": self.clock, "version": version,
                "master": self.master.detach().to("cpu", copy=True),
                "states": [s.detach().to("cpu", copy=True) for s in self._state_list()],
                "segments": [(u.name, a, z) for u, a, z in self.segs], "staleness": self.staleness}
        self.t.barrier()
        return snap

    def load_shard_state(self, st: dict) -> None:
        if st["world"] != self.world or st["rank"] != self.rank:
            raise ValueError("checkpoint was written with a different world size / rank")
        self.synchronize()
        self.t.barrier()  # every server idle: no push in flight anywhere
        with torch.no_grad():
            self.master.copy_(st["master"].to(self.master.device))
            if self.gpu:
                for s, src in zip([s for sts in self.states for s in sts], st["states"]):
                    s.copy_(src.to(s.device))
            else:
                self.server.set_states([x.numpy() for x in st["states"]])
            self.pub.copy_(self.master.to(self.dtype).expand(3, self.L))  # every slot = restored shard
            # the owner's update count drives Adam's bias correction (serve_loop applies with
            # step = version + 1): a fresh control block would restart it at 1 on warm moments
            self.A.set_version(self.ctl, self.rank, int(st.get("version", 0)))
        if self.gpu:
            torch.cuda.current_stream(self.device).synchronize()
        self.round = int(st["round"])
        self.t.barrier()
        self.refresh()

    def refresh(self) -> None:
        """Pull the newest published weights (no staleness gate), e.g. after a final barrier."""
        self._pull(gate=False)
        if self.gpu:
            torch.cuda.current_stream(self.device).synchronize()
            self.notifier.drain()

    def close(self) -> None:
        """Stop the progress thread (after every rank is done) and release shared memory."""
        if getattr(self, "server", None) is None:
            return
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self.synchronize()
        self.t.barrier()
        self.server.stop()
        if self.notifier is not None:
            self.notifier.drain()
        self.t.barrier()
        self.server = None
        self.peer_mbox = self.peer_pub = None
        self.share.close(unlink=not self.share.threads)
        self._ctl.close()
        if self.rank == 0:
            self._ctl.unlink()


_HYPER = ("lr", "beta1", "beta2", "eps", "wd", "momentum", "dampening", "nesterov", "adamw", "bc1", "bc2", "l1", "l2",
          "fbeta", "ftrl_mode", "gscale")
