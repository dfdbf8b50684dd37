"""Transport: the collective data plane under the parameter server.

The reference moves every parameter over unary gRPC calls with protobuf ``repeated float``
payloads (net/PSClient.java:47-186, src/main/resources/proto/ps.proto:7-71).  Here the data
plane is torch.distributed:

* GPU: backend "nccl" == RCCL over xGMI.  One process per GPU.  A push of a bucket is one
  ``reduce_scatter_tensor`` (every rank sends 1/W of the bucket to each owner over its 7
  xGMI links), a pull one ``all_gather_into_tensor``, sparse rows go through
  ``all_to_all_single`` with per-peer split sizes.
* CPU: backend "gloo" over TCP loopback (the BASELINE "plumbing" config and the tests).

Control plane (rendezvous, heartbeats, SSP clocks) uses the c10d TCPStore.

Debug aid (SURVEY §5.2 a): with ``check_order=True`` every collective is folded into a
running hash of (op, numel, dtype) and ``verify_order()`` all-gathers the hashes -- a
mismatch means two ranks issued collectives in different orders (a future deadlock).
"""
from __future__ import annotations

import hashlib
import os
from typing import List, Optional

import torch
import torch.distributed as dist


_SIDE_STREAMS = {}


def side_stream(device) -> "torch.cuda.Stream":
    """One shared side stream per device for parameter-server traffic issued from autograd
    hooks (sparse row pushes); collectives on it still serialise in issue order inside the
    process group, so every rank sees the same collective sequence."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _SIDE_STREAMS.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx)
        _SIDE_STREAMS[idx] = s
    return s


def _share(t: torch.Tensor) -> torch.Tensor:
    """Snapshot a tensor for another (thread-)rank of the loopback hub: GPU tensors are
    cloned on the caller's stream and that stream is drained, so the reader may use the
    copy from any stream."""
    c = t.detach().clone()
    if c.is_cuda:
        torch.cuda.current_stream(c.device).synchronize()
    return c


class Transport:
    def __init__(self, group=None, check_order: bool = False):
        self.group = group
        self.initialized = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.initialized else 1
        self.rank = dist.get_rank(group) if self.initialized else 0
        self.backend = dist.get_backend(group) if self.initialized else "local"
        self.check_order = check_order or os.environ.get("PS_AMD_CHECK_ORDER", "0") == "1"
        self._h = hashlib.sha1()
        self.n_ops = 0
        self.bytes_sent = 0

    # ------------------------------------------------------------------ bookkeeping
    def _note(self, op: str, t: torch.Tensor):
        self.n_ops += 1
        self.bytes_sent += t.numel() * t.element_size()
        if self.check_order:
            self._h.update(f"{op}:{t.numel()}:{t.dtype};".encode())

    def order_digest(self) -> str:
        return self._h.hexdigest()

    def verify_order(self) -> bool:
        """All-gather the collective-order digests; raise if ranks diverged."""
        if self.world == 1:
            return True
        d = torch.tensor(list(bytes.fromhex(self.order_digest())), dtype=torch.uint8)
        dev = self._dev()
        d = d.to(dev)
        out = torch.empty(self.world * d.numel(), dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(out, d, group=self.group)
        rows = out.view(self.world, -1).cpu()
        if not all(torch.equal(rows[0], rows[i]) for i in range(self.world)):
            raise RuntimeError("collective order mismatch across ranks (PS_AMD_CHECK_ORDER)")
        return True

    def _dev(self):
        if self.backend == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    # ------------------------------------------------------------------ collectives
    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, average: bool = False):
        """out = (sum over ranks of inp)[rank's chunk].  inp: world*len(out) elements."""
        self._note("rs", inp)
        if self.world == 1:
            if out.data_ptr() != inp.data_ptr():
                out.copy_(inp.view_as(out))
        else:
            dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=self.group)
        if average and self.world > 1:
            out.div_(self.world)
        return out

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor):
        """out = concat over ranks of inp.  ``inp`` may alias out's own chunk (in place)."""
        self._note("ag", out)
        if self.world == 1:
            if out.data_ptr() != inp.data_ptr():
                out.copy_(inp.view_as(out))
            return out
        dist.all_gather_into_tensor(out, inp, group=self.group)
        return out

    def all_reduce(self, t: torch.Tensor, op=None):
        self._note("ar", t)
        if self.world > 1:
            dist.all_reduce(t, op=op or dist.ReduceOp.SUM, group=self.group)
        return t

    def broadcast(self, t: torch.Tensor, src: int = 0):
        self._note("bc", t)
        if self.world > 1:
            dist.broadcast(t, src=src, group=self.group)
        return t

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits: Optional[List[int]] = None,
                   in_splits: Optional[List[int]] = None):
        self._note("a2a", inp)
        if self.world == 1:
            out.copy_(inp.view_as(out))
            return out
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)
        return out

    def all_gather_object(self, obj):
        if self.world == 1:
            return [obj]
        res = [None] * self.world
        dist.all_gather_object(res, obj, group=self.group)
        return res

    def split(self) -> "Transport":
        """A second transport over the same ranks with its OWN communicator (RCCL: its own
        internal stream), e.g. for pulls that should not queue behind pushes.
        Collective: every rank must call it, in the same order."""
        if self.world == 1:
            return Transport()
        ranks = list(range(self.world)) if self.group is None else dist.get_process_group_ranks(self.group)
        return Transport(group=dist.new_group(ranks), check_order=self.check_order)

    def barrier(self):
        if self.world > 1:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier(group=self.group)


_RANKS_PER_DEVICE: Optional[int] = None


def device_key(device=None) -> str:
    """Identity of the GPU (or host, for CPU ranks) this process computes on, unique across a
    node whatever CUDA_VISIBLE_DEVICES says: hostname + the device UUID (index as fallback)."""
    import socket

    host = socket.gethostname()
    if device is None or torch.device(device).type != "cuda":
        return f"{host}/cpu/{os.getpid()}"
    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    uid = getattr(torch.cuda.get_device_properties(idx), "uuid", None)
    return f"{host}/gpu/{uid if uid is not None else idx}"


def count_sharing(keys: List[str], rank: int) -> int:
    """How many ranks share ``rank``'s device, given every rank's ``device_key``."""
    return sum(1 for k in keys if k == keys[rank])


def ranks_per_device(refresh: bool = False, device=None) -> int:
    """Ranks of this job that compute on this rank's GPU: 1 on a real node (one process per
    GPU), W in the one-GPU rehearsals.  The stream policies that were tuned on a single process
    (ops/side_stream.py, bench.py's compute-stream priority) key on this, not on WORLD_SIZE.
    Computed once by an all-gather of ``device_key`` -- a collective: the first call must be made
    by every rank (``init_distributed`` does it); later calls return the cached count."""
    global _RANKS_PER_DEVICE
    if _RANKS_PER_DEVICE is not None and not refresh:
        return _RANKS_PER_DEVICE
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        _RANKS_PER_DEVICE = 1
        return 1
    if not refresh:
        # a policy query before the collective count (a process group not made by
        # init_distributed): never gather lazily from inside model code -- estimate from the
        # launcher's env (local ranks over visible devices) and leave the cache empty
        return _local_share_estimate()
    if device is None and torch.cuda.is_available():
        device = torch.device("cuda", torch.cuda.current_device())
    keys = [None] * dist.get_world_size()
    dist.all_gather_object(keys, device_key(device))
    _RANKS_PER_DEVICE = count_sharing(keys, dist.get_rank())
    return _RANKS_PER_DEVICE


def _local_share_estimate() -> int:
    """ceil(LOCAL_WORLD_SIZE / visible GPUs) without any collective (device_count does not
    initialise the GPU); 1 for CPU ranks."""
    if not torch.cuda.is_available():
        return 1
    local = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    ndev = max(1, torch.cuda.device_count())
    return max(1, -(-local // ndev))


def init_distributed(backend: Optional[str] = None, timeout_s: float = 600.0) -> Transport:
    """Initialise torch.distributed from the torchrun env (RANK/WORLD_SIZE/MASTER_*).

    backend defaults to "nccl" (RCCL) when a GPU is visible, else "gloo".  With WORLD_SIZE
    unset (or 1) no process group is created and a local Transport is returned.
    """
    import datetime

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return Transport()
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(**kw)
    ranks_per_device(refresh=True)  # collective, once per job: the stream policies key on it
    return Transport()


# ------------------------------------------------------------------------------ loopback
class LoopbackHub:
    """Rendezvous of ``world`` in-process ranks (threads): every collective is one exchange
    of per-rank payloads behind a pair of barriers.  The SURVEY §7.6 "fake backend": PS and
    consistency logic run deterministically in one process, reductions in rank order."""

    def __init__(self, world: int, timeout_s: float = 120.0):
        import threading

        self.world = world
        self.slots: List[object] = [None] * world
        self.bar = threading.Barrier(world, timeout=timeout_s)
        self.timeout_s = timeout_s
        self._child = None
        self._lock = threading.Lock()

    def child(self) -> "LoopbackHub":
        """The hub of the split (second) communicator, shared by every thread-rank."""
        with self._lock:
            if self._child is None:
                self._child = LoopbackHub(self.world, self.timeout_s)
            return self._child

    def exchange(self, rank: int, obj):
        self.slots[rank] = obj
        self.bar.wait()
        got = list(self.slots)
        self.bar.wait()  # nobody overwrites a slot before every rank has read it
        return got

    def abort(self):
        self.bar.abort()


class LoopbackTransport(Transport):
    """Transport over a LoopbackHub (same API as the RCCL/gloo Transport)."""

    def __init__(self, hub: LoopbackHub, rank: int, check_order: bool = False):
        self.group = None
        self.initialized = True
        self.hub = hub
        self.world = hub.world
        self.rank = rank
        self.backend = "loopback"
        self.check_order = check_order
        self._h = hashlib.sha1()
        self.n_ops = 0
        self.bytes_sent = 0

    def _sum(self, parts):
        acc = parts[0].clone()
        for p in parts[1:]:
            acc += p
        return acc

    def verify_order(self) -> bool:
        got = self.hub.exchange(self.rank, self.order_digest())
        if any(g != got[0] for g in got):
            raise RuntimeError("collective order mismatch across ranks (loopback)")
        return True

    def reduce_scatter(self, out, inp, average: bool = False):
        self._note("rs", inp)
        parts = self.hub.exchange(self.rank, _share(inp))
        total = self._sum(parts).view(self.world, -1)[self.rank]
        out.copy_(total.view_as(out))
        if average:
            out.div_(self.world)
        return out

    def all_gather(self, out, inp):
        self._note("ag", out)
        parts = self.hub.exchange(self.rank, _share(inp).reshape(-1))
        out.copy_(torch.cat(parts).view_as(out))
        return out

    def all_reduce(self, t, op=None):
        self._note("ar", t)
        parts = self.hub.exchange(self.rank, _share(t))
        if op is not None and op == dist.ReduceOp.MAX:
            r = parts[0].clone()
            for p in parts[1:]:
                r = torch.maximum(r, p)
        else:
            r = self._sum(parts)
        t.copy_(r)
        return t

    def broadcast(self, t, src: int = 0):
        self._note("bc", t)
        parts = self.hub.exchange(self.rank, _share(t))
        t.copy_(parts[src])
        return t

    def all_to_all(self, out, inp, out_splits=None, in_splits=None):
        self._note("a2a", inp)
        w = self.world
        if in_splits is None:
            in_splits = [inp.shape[0] // w] * w
        parts = self.hub.exchange(self.rank, (_share(inp), list(in_splits)))
        chunks = []
        for src in range(w):
            t, sp = parts[src]
            off = sum(sp[:self.rank])
            chunks.append(t[off:off + sp[self.rank]])
        out.copy_(torch.cat(chunks).view_as(out))
        return out

    def all_gather_object(self, obj):
        return self.hub.exchange(self.rank, obj)

    def split(self) -> "LoopbackTransport":
        return LoopbackTransport(self.hub.child(), self.rank, self.check_order)

    def barrier(self):
        self.hub.exchange(self.rank, None)


def run_loopback(fn, world: int, *args, timeout_s: float = 120.0):
    """Run ``fn(transport, *args)`` on ``world`` threads joined by a LoopbackHub; returns the
    per-rank results (re-raises the first rank failure)."""
    import threading

    hub = LoopbackHub(world, timeout_s)
    res: List[object] = [None] * world
    err: List[BaseException] = []

    def body(r):
        try:
            res[r] = fn(LoopbackTransport(hub, r), *args)
        except BaseException as e:  # noqa: BLE001 -- surfaced below
            err.append(e)
            hub.abort()

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if err:
        raise err[0]
    return res
