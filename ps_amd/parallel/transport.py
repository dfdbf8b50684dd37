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

    def barrier(self):
        if self.world > 1:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier(group=self.group)


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
    return Transport()
