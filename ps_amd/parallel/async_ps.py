"""Asynchronous parameter server: ASP and SSP(s) without lockstep collectives.

Reference: the async PServer applies each push the moment it arrives and the barrier returns
at once (net/PServer.java:176-184, 242-248; the worker only pushes fire-and-forget,
net/PSClient.java:159-161) -- Hogwild, no staleness bound.  SURVEY §2.3 row 3 / §5.8 asks for
a per-GPU server progress thread and bounded staleness (SSP).

MI355X-native design (one node, one process per GPU, or threads / CPU processes in tests):

* the flat parameter space is range-partitioned; rank r OWNS shard r: fp32 master + optimizer
  state, W gradient MAILBOXES (one per worker) and 3 PUBLISHED weight slots, all in its HBM;
* push  = the worker copies its gradient slice for shard r straight into mailbox[w] of owner r
          (peer copies over xGMI into IPC-mapped memory, on a side stream), then a native
          completion thread bumps seq[r][w] once the copies landed -- the training thread never
          waits for it;
* serve = a NATIVE progress thread per owner (csrc/async_ps_gpu.cpp; CPU: csrc/runtime)
          polls the shared control block, runs the fused HIP optimizer on each deposited push
          in arrival order (Hogwild-style, one update per push, gradient scaled by 1/W), writes
          the new weights into a free slot, publishes it and acknowledges the push;
* pull  = the worker pins every owner's current slot (the owner never overwrites a pinned
          slot: no torn reads) and copies it into its replica;
* SSP(s): before pulling at clock c the worker waits until every owner has APPLIED every
          worker's first c - s pushes (so the weights read contain all updates older than
          s steps); s = 0 is BSP semantics without any collective, ``staleness=None`` is ASP.

No rank ever blocks on another rank reaching a matching collective: a slow worker only slows
the others through the staleness bound (SSP) or not at all (ASP).  The control block lives in
POSIX shared memory (csrc/include/async_ctl.h); buffers are exchanged once at start-up through
the transport's object all-gather (CUDA IPC handles between processes, named shared memory for
CPU processes, plain tensors between loopback thread-ranks).
"""
from __future__ import annotations

import os
import uuid
from typing import Dict, List, Optional, Union

import torch

from ..obs import trace as _trace
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
    ``finish_step()`` after backward pushes asynchronously and pulls what the staleness bound
    allows; parameters are views of the flat replica."""

    def __init__(self, model: torch.nn.Module, updaters: Union[Updater, Dict[str, Updater]],
                 transport: Optional[Transport] = None, *, staleness: Optional[int] = None,
                 gscale: Optional[float] = None, timeout_s: float = 600.0):
        self.model = model
        self.t = transport or Transport()
        self.world, self.rank = self.t.world, self.t.rank
        W, me = self.world, self.rank
        umap = updaters if isinstance(updaters, dict) else {"default": updaters}
        params = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        if not params:
            raise ValueError("model has no trainable parameters")
        us = {id(resolve_updater(n, umap)) for n, _ in params}
        if len(us) != 1:
            raise ValueError("AsyncPS applies one updater to the whole flat space")
        self.updater = resolve_updater(params[0][0], umap)
        dtypes = {p.dtype for _, p in params}
        if len(dtypes) != 1:
            raise ValueError("AsyncPS needs one parameter dtype")
        self.dtype = dtypes.pop()
        self.device = params[0][1].device
        self.gpu = self.device.type == "cuda"
        self.staleness = staleness
        self.timeout_s = timeout_s
        self.gscale = (1.0 / W) if gscale is None else float(gscale)
        self.params = dict(params)
        n = sum(p.numel() for _, p in params)
        self.L = ((n + W - 1) // W + 63) // 64 * 64
        L = self.L
        # ---------------- replica + gradient flats (parameters are views)
        self.flat = torch.zeros(W * L, dtype=self.dtype, device=self.device)
        self.gflat = torch.zeros(W * L, dtype=self.dtype, device=self.device)
        self.offsets = {}
        off = 0
        with torch.no_grad():
            for nme, p in params:
                self.flat[off:off + p.numel()].copy_(p.detach().reshape(-1))
                self.offsets[nme] = (off, p.numel(), p.shape)
                off += p.numel()
            self.t.broadcast(self.flat, src=0)
        self._bind()
        # ---------------- owner state + shared buffers
        self.share = _Shared(self.t, self.device)
        lo = me * L
        self.master = self.flat[lo:lo + L].float().clone()
        self.states = self.updater.new_states(self.master) if self.gpu else []
        self.mbox = self.share.alloc((W, L), self.dtype)
        self.pub = self.share.alloc((3, L), self.dtype)
        with torch.no_grad():
            self.pub.copy_(self.flat[lo:lo + L].expand(3, L))
        # control block: rank 0 creates the shared segment, everyone maps it
        A = _native().async_ctl
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
        # ---------------- native progress thread (owner) + completion thread (worker)
        if self.gpu:
            from .. import _C  # type: ignore

            h = self.updater.hyper(1)
            st = self.states + [None] * (2 - len(self.states))
            bias = _BIAS_MODE[self.updater.bias_correction] if isinstance(self.updater, AdamUpdater) else 0
            self.server = _C.GpuAsyncServer(
                self.ctl, me, self.updater.kind, self.master, st[0], st[1], [self.mbox[w] for w in range(W)],
                [self.pub[s] for s in range(3)], h.get("lr", 0.01), h.get("beta1", 0.9), h.get("beta2", 0.999),
                h.get("eps", 1e-8), h.get("wd", 0.0), h.get("momentum", 0.0), h.get("dampening", 0.0),
                bool(h.get("nesterov", False)), bool(h.get("adamw", False)), bias, h.get("l1", 0.0), h.get("l2", 0.0),
                h.get("fbeta", 1.0), int(h.get("ftrl_mode", 0)), self.gscale)
            self.notifier = _C.GpuNotifier(self.ctl)
            self.push_stream = side_stream(self.device)
        else:
            if self.dtype != torch.float32:
                raise ValueError("CPU AsyncPS shards are fp32")
            self.server = _native().CpuAsyncServer(
                self.ctl, me, self.updater.name, L, self.master.data_ptr(), [self.mbox[w].data_ptr() for w in range(W)],
                [self.pub[s].data_ptr() for s in range(3)], self.gscale)
            self.notifier = None
        self.t.barrier()
        self.server.start()
        self.clock = 0
        self.round = 0
        self.accumulating = False
        self.stats = {"gate_waits": 0}

    # ------------------------------------------------------------------ views
    def _bind(self) -> None:
        for nme, p in self.params.items():
            off, n, shape = self.offsets[nme]
            p.data = self.flat[off:off + n].view(shape)
            p.grad = None

    def weight(self, name: str) -> torch.Tensor:
        off, n, shape = self.offsets[name]
        return self.flat[off:off + n].view(shape)

    # ------------------------------------------------------------------ step
    def _land(self) -> None:
        dst, src = [], []
        for nme, p in self.params.items():
            off, n, _ = self.offsets[nme]
            v = self.gflat[off:off + n]
            if p.grad is None:
                v.zero_()
            else:
                dst.append(v)
                src.append(p.grad.reshape(-1))
            p.grad = None
        if dst:
            torch._foreach_copy_(dst, src)

    def finish_step(self) -> None:
        """Push this step's gradient to every owner (asynchronously), advance the clock, and
        pull the newest weights the staleness bound allows."""
        if self.accumulating:
            return
        with _trace.range(f"async_ps.step.c{self.clock}"):
            self._finish_step()

    def _finish_step(self) -> None:
        W, me, L, A = self.world, self.rank, self.L, self.A
        if self.gpu:
            torch.cuda.current_stream(self.device).wait_stream(self.push_stream)  # gflat free again
        self._land()
        # each owner must have APPLIED every earlier push of ours before the next copy lands in the
        # 1-deep mailbox: gate on our own push count (seq lags behind on GPU -- it is bumped by
        # the completion thread after the copy finished -- so "ack == seq" could pass while the
        # previous copy is still queued, and the owner would read a mailbox being overwritten)
        for r in range(W):
            A.wait_ack(self.ctl, r, me, self.clock, self.timeout_s)
        if self.gpu:
            cur = torch.cuda.current_stream(self.device)
            self.push_stream.wait_stream(cur)
            with torch.cuda.stream(self.push_stream):
                for r in range(W):
                    self.peer_mbox[r][me].copy_(self.gflat[r * L:(r + 1) * L], non_blocking=True)
                self.notifier.after(self.push_stream.cuda_stream, self.device.index, list(range(W)), me, True, [])
        else:
            for r in range(W):
                self.peer_mbox[r][me].copy_(self.gflat[r * L:(r + 1) * L])
                A.bump_seq(self.ctl, r, me)
            A.bump_clock(self.ctl, me)
        self.clock += 1
        self.round += 1
        self._pull()

    def _pull(self) -> None:
        W, L, A = self.world, self.L, self.A
        if self.staleness is not None:
            A.wait_min_ack(self.ctl, self.clock - int(self.staleness), self.timeout_s)
        pins = [(r, A.pin(self.ctl, r)) for r in range(W)]
        with torch.no_grad():
            for r, s in pins:
                self.flat[r * L:(r + 1) * L].copy_(self.peer_pub[r][s], non_blocking=True)
        if self.gpu:
            self.notifier.after(torch.cuda.current_stream(self.device).cuda_stream, self.device.index, [],
                                self.rank, False, pins)
        else:
            for r, s in pins:
                A.unpin(self.ctl, r, s)

    # ------------------------------------------------------------------ control
    def snapshot(self) -> dict:
        return self.A.snapshot(self.ctl)

    def synchronize(self) -> None:
        """Wait until every push of THIS worker has been applied by every owner, then pull."""
        if self.gpu:
            torch.cuda.current_stream(self.device).synchronize()
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

    # ------------------------------------------------------------------ checkpoint
    def shard_state(self) -> dict:
        """This owner's shard (fp32 master, optimizer state, version) at a QUIESCENT point: every
        rank calls it at the same step boundary; after the barrier no push is in flight."""
        self.synchronize()
        self.t.barrier()
        st = self.states if self.gpu else [torch.from_numpy(a) for a in self.server.states()]
        version = int(self.A.snapshot(self.ctl)["version"][self.rank])
        snap = {"rank": self.rank, "world": self.world, "round": self.round, "clock": self.clock, "version": version,
                "master": self.master.detach().to("cpu", copy=True),
                "states": [s.detach().to("cpu", copy=True) for s in st], "staleness": self.staleness}
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
                for s, src in zip(self.states, st["states"]):
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
        self._pull_latest()

    def _pull_latest(self) -> None:
        s, self.staleness = self.staleness, None
        try:
            self._pull()
        finally:
            self.staleness = s
        if self.gpu:
            torch.cuda.current_stream(self.device).synchronize()
            self.notifier.drain()

    def close(self) -> None:
        """Stop the progress thread (after every rank is done) and release shared memory."""
        if getattr(self, "server", None) is None:
            return
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
