"""The xGMI plane: one-sided push / serve / pull of the co-located parameter server.

Reference round: workers push every key to the key's server
(store/KVStore.java:259 -> net/PSClient.java:154-174), meet at a barrier
(net/PSRouterClient.java:131-151 -> net/PServer.java:238-283), the server applies the updater
(net/PServer.java:197-214) and workers pull again (store/KVStore.java:136-159).

On one MI355X node the ranks share a host, so the parameter server needs no collective
library at all ("per-key reduce over xGMI sized for 7 point-to-point
links").  Every rank allocates ONE device arena holding its replica weight slots, gradient
slots and 1-bit push buffers (identical layout on every rank), maps every peer's arena
through CUDA-IPC handles, and a native engine (csrc/plane.cpp) runs each bucket's round:

* push  -- the backward hook lands the bucket's gradients in the rank's OWN gradient slot and
  hands (bucket, round, landing event) to the engine, which publishes ``ready[me][b]`` in a
  shared-memory control block once the event completed;
* serve -- when all W ranks are ready, ONE kernel on every owner reads its chunk of the bucket
  from all W arenas at once (W concurrent xGMI streams), sums in fp32 in rank order and
  applies the fused optimizer in the same pass (csrc/kernels/optim.hip fused_opt_multi): the
  reduced gradient never exists in HBM; ``served[me][b]`` follows;
* pull  -- when every owner served the bucket, ONE kernel copies the other W-1 owners' fresh
  chunks into the local replica, blocks dealt over the owners (csrc/kernels/plane.hip).

The training thread never waits for a peer: before the forward that needs round t's weights
it only blocks until the engine has ENQUEUED round t's pulls, then its compute stream waits on
the last pull event.  No kernel spins on a flag (every cross-rank wait is on the host, with a
deadline and an abort word), so a dead peer can stop the job but cannot hang a GPU.

Ordering is causal (why no buffer is overwritten while a peer still reads it): with a ring of
S = staleness + 1 slots, rank p lands round t + S in gradient slot t mod S only after the
forward of step t + S, which waited for the pulls of round t + S - s - 1 = t, which waited
for every owner to have served round t, i.e. to have finished reading slot t mod S.  The same
argument covers weight slots (round t's pull reads slot (t+1) mod S; the owner rewrites it at
round t + S only after every rank landed round t + S).

Modes: GPU ranks as processes (CUDA-IPC), GPU thread-ranks of one process (raw pointers), and
CPU ranks (gloo processes over /dev/shm segments, or loopback threads) where the same native
state machine drives Python callbacks -- the CPU tests exercise the exact protocol.
"""
from __future__ import annotations

import os
import uuid
from typing import Dict, List, Optional

import torch

from ..ops import compress as _cmp
from ..ops import optim as _o
from ..ops import reduce as _red
from .async_ps import _addr, _ShmSeg
from .ipc_arena import IpcArena
from .transport import Transport

_ALIGN = 256


def _esize(dt: torch.dtype) -> int:
    return torch.empty((), dtype=dt).element_size()


def _C():
    from .. import _C as m  # type: ignore

    return m


class PlaneUnavailable(RuntimeError):
    """Raised on EVERY rank (the ranks agree at each step) when the plane cannot be set up --
    the caller may fall back to the collective path without the ranks diverging."""


def plane_available(transport: Transport, device: torch.device) -> bool:
    """The xGMI plane needs every rank on this host (one node) and at most MAX_WORLD ranks."""
    if transport.world <= 1:
        return False
    try:
        lim = _C().plane.MAX_WORLD
    except Exception:  # noqa: BLE001 -- extension missing: collective path
        return False
    if transport.world > lim:
        return False
    import socket

    hosts = transport.all_gather_object(socket.gethostname())
    return len(set(hosts)) == 1


class XgmiPlane:
    """Arena, control block and native engine of one rank (see module docstring)."""

    def __init__(self, transport: Transport, reg, device: torch.device, nslots: int, *, onebit: bool = False,
                 clip_norm: Optional[float] = None, average: bool = True, timeout_s: float = 600.0):
        self.t = transport
        self.W, self.me = transport.world, transport.rank
        self.reg = reg
        self.device = device
        self.gpu = device.type == "cuda"
        self.threads = transport.backend == "loopback"
        self.nslots = nslots
        self.onebit = onebit
        self.clip_norm = clip_norm
        self.average = average
        self.timeout_s = timeout_s
        P = _C().plane
        if self.W > P.MAX_WORLD:
            raise ValueError(f"the xGMI plane supports at most {P.MAX_WORLD} ranks")
        # ---------------- arena layout (byte offsets, identical on every rank)
        self._off = 0
        self.woff = {g: [self._take(n * _esize(reg.group_dtype[g])) for _ in range(nslots)]
                     for g, n in reg.group_size.items()}
        self.goff = {g: [self._take(n * _esize(reg.group_dtype[g])) for _ in range(nslots)]
                     for g, n in reg.group_size.items()}
        self.words_off: List[List[int]] = []
        self.scales_off: List[List[int]] = []
        for b in reg.buckets:
            if onebit:
                nw, ns = _cmp.packed_sizes(b.size)
                self.words_off.append([self._take(nw * 8) for _ in range(nslots)])
                self.scales_off.append([self._take(ns * 4) for _ in range(nslots)])
            else:
                self.words_off.append([0] * nslots)
                self.scales_off.append([0] * nslots)
        self.sq_off = self._take(2 * 4)
        self.probe_off = self._take(self.W * 64 * 4)
        self.nbytes = self._off
        # ---------------- allocate + share (every fallible local step ends in an agreement, so a
        # failure raises PlaneUnavailable on all ranks at the same point)
        self._arena = None
        self._seg = None
        self._ctl = None
        # what the bench JSON reports at N > 1: mapping mode, self-test result, round-end mechanism
        self.info: Dict[str, str] = {"mode": "threads" if self.threads else "shm (cpu)", "self_test": "skipped",
                                     "round_end": "host flags"}
        self._tmp_engine = None
        self._opened: List[_ShmSeg] = []
        if self.gpu:
            err = None
            try:
                self._arena = IpcArena(self.nbytes, device.index)  # VMM chunks above 1 GiB (ipc_arena.py)
                self.arena = self._arena.tensor()
                mine = (self._arena.handle() if not self.threads else self._arena.base, device.index)
            except Exception as e:  # noqa: BLE001 -- reported through the agreement
                err, mine = e, None
            hs = self.t.all_gather_object(mine)
            self._agree(err is None and all(h is not None for h in hs), f"arena allocation failed: {err!r}")
            bases = []
            try:
                for r, (h, d) in enumerate(hs):
                    if r == self.me or self.threads:
                        bases.append(self._arena.base if r == self.me else int(h))
                    else:
                        bases.append(self._arena.open(h, d))
            except Exception as e:  # noqa: BLE001
                err = e
            self._agree(err is None, f"mapping the peer arenas failed: {err!r}")
            self.bases = bases
            self.peers = None
            devs = sorted({d for _, d in hs})
            self.info["mode"] = "threads (shared device pointers)" if self.threads else (
                "ipc, one device" if len(devs) == 1 else f"ipc, peer access across {len(devs)} devices")
        else:
            if self.threads:
                self.arena = torch.zeros(self.nbytes, dtype=torch.uint8)
                self.peers = self.t.all_gather_object(self.arena)
            else:
                name = f"psamd_plane_{uuid.uuid4().hex[:16]}"
                self._seg = _ShmSeg(name, self.nbytes, create=True)
                self.arena = torch.frombuffer(self._seg.buf, dtype=torch.uint8, count=self.nbytes)
                self.arena.zero_()
                names = self.t.all_gather_object(name)
                self.peers = []
                for r, nm in enumerate(names):
                    if r == self.me:
                        self.peers.append(self.arena)
                    else:
                        sg = _ShmSeg(nm)
                        self._opened.append(sg)
                        self.peers.append(torch.frombuffer(sg.buf, dtype=torch.uint8, count=self.nbytes))
            self.bases = [0] * self.W
        # ---------------- control block (rank 0 creates it in /dev/shm)
        size = P.ctl_size(self.W, len(reg.buckets))
        cname = self.t.all_gather_object(f"psamd_pctl_{uuid.uuid4().hex[:16]}" if self.me == 0 else None)[0]
        if self.me == 0:
            self._ctl = _ShmSeg(cname, size, create=True)
            P.ctl_init(_addr(self._ctl), self.W, len(reg.buckets))
        self.t.barrier()
        if self.me != 0:
            self._ctl = _ShmSeg(cname)
        self.ctl = _addr(self._ctl)
        self.engine = None
        self._hyper_round = -1
        self._uids: Dict[int, int] = {}
        self._ups: List = []
        if self.gpu and not self.threads:
            err = None
            try:
                self.self_test()
            except Exception as e:  # noqa: BLE001
                err = e
            self._agree(err is None, f"self-test failed: {err!r}")
            self.info["self_test"] = "ok (2 probe round trips through every peer arena)"

    def _agree(self, ok: bool, what: str) -> None:
        oks = self.t.all_gather_object(bool(ok))
        if not all(oks):
            bad = [r for r, o in enumerate(oks) if not o]
            raise PlaneUnavailable(f"xGMI plane unavailable (ranks {bad}): " + (what if not ok else "peer failure"))

    # ------------------------------------------------------------------ layout helpers
    def _take(self, nbytes: int) -> int:
        o = self._off
        self._off = (o + max(1, nbytes) + _ALIGN - 1) // _ALIGN * _ALIGN
        return o

    def view(self, off: int, dtype: torch.dtype, numel: int, rank: Optional[int] = None) -> torch.Tensor:
        """``numel`` elements of ``dtype`` at byte ``off`` of this rank's arena (CPU modes: of
        ``rank``'s arena)."""
        src = self.arena if rank is None or rank == self.me else self.peers[rank]
        return src[off:off + numel * _esize(dtype)].view(dtype)

    def slots(self, which: str) -> Dict[str, List[torch.Tensor]]:
        offs = self.woff if which == "w" else self.goff
        return {g: [self.view(o, self.reg.group_dtype[g], self.reg.group_size[g]) for o in offs[g]]
                for g in self.reg.group_size}

    def words(self, b: int, slot: int, rank: Optional[int] = None):
        nw, ns = _cmp.packed_sizes(self.reg.buckets[b].size)
        return (self.view(self.words_off[b][slot], torch.int64, nw, rank),
                self.view(self.scales_off[b][slot], torch.float32, ns, rank))

    # ------------------------------------------------------------------ engine
    def attach(self, ps) -> None:
        """Register buckets and updater segments of a ColocatedPS and start the engine."""
        P = _C().plane
        self.ps = ps
        R = self.reg
        clip = float(self.clip_norm) if self.clip_norm is not None else 0.0
        dev = self.device.index if self.gpu else -1
        eng = P.Engine(self.ctl, self.me, self.W, len(R.buckets), self.nslots, self.gpu, dev if dev is not None else 0,
                       float(self.timeout_s), clip, bool(self.average))
        if self.gpu:
            eng.set_bases([int(b) for b in self.bases])
        self.gshard: List[Optional[torch.Tensor]] = []
        for b, bk in enumerate(R.buckets):
            dt = R.group_dtype[bk.group]
            es = _esize(dt)
            gsh = torch.zeros(bk.chunk, dtype=torch.float32, device=self.device) if self.clip_norm is not None else None
            self.gshard.append(gsh)
            eng.add_bucket(b, dt == torch.bfloat16, es, bk.chunk,
                           [o + bk.start * es for o in self.goff[bk.group]],
                           [o + bk.start * es for o in self.woff[bk.group]],
                           self.words_off[b], self.scales_off[b], gsh.data_ptr() if (gsh is not None and self.gpu) else 0)
            for (u, a, z), st in zip(ps.segs[b], ps.states[b]):
                uid = self._uid(u)
                if self.gpu:
                    m = ps.master[b]
                    s0 = st[0][...].data_ptr() if len(st) > 0 else 0
                    s1 = st[1].data_ptr() if len(st) > 1 else 0
                    eng.add_segment(b, uid, u.kind, a, z, m[a:z].data_ptr(), s0, s1)
                else:
                    eng.add_segment(b, uid, u.kind, a, z, 0, 0, 0)
        if self.clip_norm is not None:
            self._total = torch.zeros(1, dtype=torch.float32, device=self.device)
            self._factor = torch.ones(1, dtype=torch.float32, device=self.device)
            self._partial = torch.zeros(1024, dtype=torch.float32, device=self.device)
            if self.gpu:
                eng.set_norm(self.sq_off, self._total.data_ptr(), self._factor.data_ptr(), self._partial.data_ptr())
        if not self.gpu:
            eng.set_callback(self._callback)
        # round end on the device (PS_AMD_PLANE_IPC_EVENTS=1, GPU processes): owners publish a
        # serve as soon as it is enqueued and peers' pulls wait on its inter-process event, so no
        # host waits for another rank's serve kernel to finish (csrc/plane.cpp enable_ipc_events)
        self.ipc_events = (self.gpu and not self.threads and self.W > 1
                           and os.environ.get("PS_AMD_PLANE_IPC_EVENTS", "0") == "1")
        if self.ipc_events:
            hs = eng.ipc_event_handles(self.nslots + 1)
            eng.enable_ipc_events(self.t.all_gather_object(list(hs)))
            self.info["round_end"] = "ipc events (serve published at enqueue)"
        self.engine = eng
        self._tmp_engine = None
        eng.start()

    def _uid(self, u) -> int:
        k = id(u)
        if k not in self._uids:
            self._uids[k] = len(self._ups)
            self._ups.append(u)
        return self._uids[k]

    def begin_round(self, rnd: int) -> None:
        """Hand the engine every updater's hyper-parameters for round ``rnd`` (LR schedules and
        Adam bias correction are evaluated here, on the host, once per round)."""
        if rnd <= self._hyper_round:
            return
        self._hyper_round = rnd
        for uid, u in enumerate(self._ups):
            h = _o._hp(u.hyper(rnd + 1))
            self.engine.set_hyper(rnd, uid, [float(h[k]) for k in (
                "lr", "beta1", "beta2", "eps", "wd", "momentum", "dampening", "nesterov", "adamw", "bc1", "bc2", "l1",
                "l2", "fbeta", "ftrl_mode", "gscale")])

    def push(self, b: int, rnd: int, gslot: int, wslot: int, onebit: bool) -> None:
        self.begin_round(rnd)
        stream = torch.cuda.current_stream(self.device).cuda_stream if self.gpu else 0
        self.engine.push(b, rnd, gslot, wslot, 1 if onebit else 0, stream)

    def wait_pulled(self, rnd: int) -> None:
        stream = torch.cuda.current_stream(self.device).cuda_stream if self.gpu else 0
        self.engine.wait_pulled(rnd, stream)

    def restore_round(self, rnd: int) -> None:
        """After a checkpoint restore at PS clock ``rnd``: mark this rank's control words as if
        rounds 0 .. rnd-1 had run here (csrc/plane.cpp restore_round)."""
        self.engine.restore_round(int(rnd))

    def stats(self, reset: bool = False) -> dict:
        return dict(self.engine.stats(reset)) if self.engine is not None else {}

    # ------------------------------------------------------------------ one-off transfers
    def broadcast_weights(self, wbuf: Dict[str, List[torch.Tensor]], src: int = 0) -> None:
        """Every rank's weight slot 0 := rank ``src``'s (start-up); collective."""
        self._sync()
        self.t.barrier()
        if self.me != src:
            for g, offs in self.woff.items():
                nb = self.reg.group_size[g] * _esize(self.reg.group_dtype[g])
                if self.gpu:
                    self.engine_or_tmp().copy_peer(src, offs[0], nb, torch.cuda.current_stream(self.device).cuda_stream)
                else:
                    wbuf[g][0].copy_(self.view(offs[0], self.reg.group_dtype[g], self.reg.group_size[g], src))
        self._sync()
        self.t.barrier()

    def gather_all(self, wslot: int) -> None:
        """Pull every bucket of weight slot ``wslot`` from its owners now (checkpoint restore;
        the caller wrote its own chunks and every rank calls this)."""
        self._sync()
        self.t.barrier()
        for b, bk in enumerate(self.reg.buckets):
            if self.gpu:
                self.engine.gather_now(b, wslot, torch.cuda.current_stream(self.device).cuda_stream)
            else:
                self._pull(b, wslot)
        self._sync()
        self.t.barrier()

    def engine_or_tmp(self):
        if self.engine is not None:
            return self.engine
        # before attach(): a bare engine for the start-up copies (never started)
        if self._tmp_engine is None:
            P = _C().plane
            self._tmp_engine = P.Engine(self.ctl, self.me, self.W, len(self.reg.buckets), self.nslots, True,
                                        self.device.index, 60.0, 0.0, True)
            self._tmp_engine.set_bases([int(b) for b in self.bases])
        return self._tmp_engine

    def _sync(self) -> None:
        if self.gpu:
            torch.cuda.current_stream(self.device).synchronize()

    def self_test(self) -> None:
        """Round-trip a probe through every peer arena twice (with different values) before the
        first real round: a mapping that does not work, or reads that come back stale, fail
        here loudly instead of corrupting training."""
        probe = self.view(self.probe_off, torch.float32, self.W * 64)
        eng = self.engine_or_tmp()
        for it in range(2):
            val = float(1000 * (it + 1) + self.me + 1)
            probe[self.me * 64:(self.me + 1) * 64].fill_(val)
            self._sync()
            self.t.barrier()
            st = torch.cuda.current_stream(self.device).cuda_stream
            for p in range(self.W):
                if p != self.me:
                    eng.copy_peer(p, self.probe_off + p * 256, 256, st)
            self._sync()
            got = probe.view(self.W, 64).cpu()
            for p in range(self.W):
                want = float(1000 * (it + 1) + p + 1)
                if not bool((got[p] == want).all()):
                    raise RuntimeError(f"xGMI plane self-test failed: rank {self.me} read {got[p][0].item()} from rank "
                                       f"{p}, expected {want}")
            self.t.barrier()

    # ------------------------------------------------------------------ CPU callbacks
    def _grad_src(self, b: int, gslot: int, p: int, onebit: bool) -> torch.Tensor:
        """Rank p's push of this rank's chunk of bucket b (fp32)."""
        bk = self.reg.buckets[b]
        lo, hi = bk.owner_range(self.me)
        dt = self.reg.group_dtype[bk.group]
        if onebit:
            words, scales = self.words(b, gslot, p)
            nwc, nsc = bk.chunk // 64, bk.chunk // _cmp.CHUNK
            out = torch.zeros(bk.chunk, dtype=torch.float32)
            _cmp.onebit_unpack_reduce(words[self.me * nwc:(self.me + 1) * nwc].view(1, -1),
                                      scales[self.me * nsc:(self.me + 1) * nsc].view(1, -1), out)
            return out
        g = self.view(self.goff[bk.group][gslot], dt, self.reg.group_size[bk.group], p)
        return g[lo:hi].float()

    def _reduced(self, b: int, gslot: int, onebit: bool) -> torch.Tensor:
        acc = self._grad_src(b, gslot, 0, onebit).clone()
        for p in range(1, self.W):
            acc += self._grad_src(b, gslot, p, onebit)
        return acc

    def _serve(self, b: int, rnd: int, gslot: int, wslot: int, g: torch.Tensor, gscale_t=None) -> None:
        ps = self.ps
        bk = self.reg.buckets[b]
        lo, hi = bk.owner_range(self.me)
        own = ps.wbuf[bk.group][wslot][lo:hi]
        gs = 1.0 / self.W if self.average else 1.0
        for (u, a, z), st in zip(ps.segs[b], ps.states[b]):
            u.step_flat(ps.master[b][a:z], st, g[a:z], wout=own[a:z], gscale=gs, gscale_t=gscale_t, step=rnd + 1)

    def _pull(self, b: int, wslot: int) -> None:
        bk = self.reg.buckets[b]
        dt = self.reg.group_dtype[bk.group]
        mine = self.view(self.woff[bk.group][wslot], dt, self.reg.group_size[bk.group])
        for o in range(self.W):
            if o == self.me:
                continue
            lo, hi = bk.owner_range(o)
            src = self.view(self.woff[bk.group][wslot], dt, self.reg.group_size[bk.group], o)
            mine[lo:hi].copy_(src[lo:hi])

    def _sq(self, rank: int, rnd: int) -> torch.Tensor:
        return self.view(self.sq_off, torch.float32, 2, rank)[rnd & 1:(rnd & 1) + 1]

    def _callback(self, op: str, b: int, rnd: int, gslot: int, wslot: int, flags: int) -> None:
        onebit = bool(flags & 1)
        if op == "serve":
            self._serve(b, rnd, gslot, wslot, self._reduced(b, gslot, onebit))
        elif op == "pull":
            self._pull(b, wslot)
        elif op == "reduce":
            g = self._reduced(b, gslot, onebit)
            self.gshard[b].copy_(g)
            _red.sumsq(g, self._sq(self.me, rnd), accumulate=True)
        elif op == "zero_sq":
            self._sq(self.me, rnd).zero_()
        elif op == "factor":
            tot = self._sq(0, rnd).clone()
            for p in range(1, self.W):
                tot += self._sq(p, rnd)
            self._total.copy_(tot)
            mx = float(self.clip_norm) * (self.W if self.average else 1)
            _red.clip_factor(self._total, mx, self._factor)
        elif op == "serve_clipped":
            self._serve(b, rnd, gslot, wslot, self.gshard[b], gscale_t=self._factor)
        else:
            raise ValueError(op)

    # ------------------------------------------------------------------ shutdown
    def close(self) -> None:
        if self.engine is not None:
            self.engine.stop()
            err = self.engine.error()
            self.engine = None
            if err:
                raise RuntimeError(f"xGMI plane: {err}")

    def abort(self) -> None:
        _C().plane.ctl_abort(self.ctl, self.me)

    def snapshot(self) -> List[int]:
        return list(_C().plane.ctl_snapshot(self.ctl))

    def release(self) -> None:
        """Unmap / unlink shared memory (after every rank closed)."""
        for s in self._opened:
            s.close()
        self._opened = []
        if self._seg is not None:
            self._seg.close()
            self._seg.unlink()
            self._seg = None
        if self._ctl is not None:
            self._ctl.close()
            if self.me == 0:
                self._ctl.unlink()
            self._ctl = None


def env_plane(default: str = "auto") -> str:
    return os.environ.get("PS_AMD_PLANE", default)
