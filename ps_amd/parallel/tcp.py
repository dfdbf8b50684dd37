"""Dedicated-server topology over the native TCP parameter server (csrc/runtime/ps_server.cpp).

Reference classes and their equivalents:
  PServer        (net/PServer.java)        -> ``PServer``: owns a native server thread pool
  PSClient       (net/PSClient.java)       -> ``PSClient``: one connection to one server
  PSRouterClient (net/PSRouterClient.java) -> ``PSRouterClient``: S servers, keys routed by a
                 pluggable ``Router`` (net/Router.java / Mod.java, negative-hash crash fixed),
                 list ops grouped by shard and fanned out on a thread pool, barrier to all.

Tensors cross as float32 numpy arrays (the C++ side frames them as raw floats); pushes
carry many keys per request.  CLI: ``python -m ps_amd.parallel.tcp --port 8890 --workers 2``.
"""
from __future__ import annotations

import argparse
import json
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np
import torch

from .registry import hash_router


def _native():
    from .. import _native  # type: ignore

    return _native


def _np(t) -> np.ndarray:
    if isinstance(t, torch.Tensor):
        return t.detach().float().cpu().contiguous().numpy()
    return np.ascontiguousarray(t, dtype=np.float32)


class PServer:
    """A parameter-server shard process (BSP / SSP / ASP)."""

    def __init__(self, port: int = 0, workers: int = 1, mode: str = "bsp", staleness: int = 0,
                 barrier_timeout_s: float = 600.0, bind_any: bool = False):
        self._s = _native().PSServer(port, workers, mode, staleness, barrier_timeout_s)
        if bind_any:
            self._s.set_bind_any(True)
        self.mode = mode

    def start(self) -> "PServer":
        self._s.start()
        return self

    @property
    def port(self) -> int:
        return self._s.port

    @property
    def generation(self) -> int:
        return self._s.generation

    def wait(self) -> None:
        self._s.wait()

    def stop(self) -> None:
        self._s.stop()


class PSClient:
    """Single-server client (net/PSClient.java:47-186)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 8890, timeout_s: float = 30.0):
        self.host, self.port = host, port
        self._c = _native().PSClient(host, port, timeout_s)

    def get(self, key: str) -> Optional[torch.Tensor]:
        a = self._c.get(key)
        return None if a is None else torch.from_numpy(a)

    def get_list(self, keys: Sequence[str]) -> Dict[str, Optional[torch.Tensor]]:
        res = self._c.get_list(list(keys))
        return {k: (None if a is None else torch.from_numpy(a)) for k, a in zip(keys, res)}

    def update(self, key: str, value, replace: bool = False) -> torch.Tensor:
        """Upsert; with replace=False the first writer wins and the stored value returns."""
        _, a = self._c.upsert(key, _np(value), replace)
        return torch.from_numpy(a)

    def update_list(self, items: Dict[str, object], replace: bool = False) -> Dict[str, torch.Tensor]:
        keys = list(items)
        res = self._c.upsert_list(keys, [_np(items[k]) for k in keys], replace)
        return {k: torch.from_numpy(a) for k, (_, a) in zip(keys, res)}

    def push(self, grads: Dict[str, object], updater_spec: str, apply_now: bool = False) -> None:
        keys = list(grads)
        self._c.push(keys, [_np(grads[k]) for k in keys], updater_spec, 2 if apply_now else 0)

    def barrier(self, worker: int = 0) -> int:
        return self._c.barrier(worker)

    def row_pull(self, table: str, dim: int, keys: torch.Tensor, lo: float = 0.0, hi: float = 0.0,
                 seed: int = 0) -> torch.Tensor:
        """Rows of int64 ``keys`` from the server's row table (created on first pull with the
        deterministic (seed, key) init the GPU lazy-init kernel uses)."""
        k = keys.detach().cpu().long().contiguous().numpy()
        return torch.from_numpy(self._c.row_pull(table, int(dim), k, float(lo), float(hi), int(seed)))

    def row_push(self, table: str, dim: int, keys: torch.Tensor, grads, updater_spec: str,
                 apply_now: bool = False) -> None:
        k = keys.detach().cpu().long().contiguous().numpy()
        self._c.row_push(table, int(dim), k, _np(grads).reshape(len(k), int(dim)), updater_spec, 2 if apply_now else 0)

    def clock(self, worker: int, c: int) -> int:
        return self._c.clock(worker, c)

    def rendezvous(self, worker: int = 0) -> int:
        """All W workers meet, in any consistency mode (independent of the BSP generation)."""
        return self._c.rendezvous(worker)

    def register_updater(self, spec: str) -> None:
        self._c.register_updater(spec)

    def stats(self) -> dict:
        return json.loads(self._c.stats())

    def save(self, path: str) -> None:
        self._c.save(path)

    def load(self, path: str) -> None:
        self._c.load(path)

    def heartbeat(self, worker: int) -> None:
        self._c.heartbeat(worker)

    def shutdown(self) -> None:
        self._c.shutdown()

    @property
    def bytes_sent(self) -> int:
        return self._c.bytes_sent


class PSRouterClient:
    """Sharded client over several servers (net/PSRouterClient.java:23-152)."""

    def __init__(self, addrs: Sequence[str], router: Optional[Callable[[str], int]] = None, timeout_s: float = 30.0):
        self.clients: List[PSClient] = []
        for a in addrs:
            host, port = a.rsplit(":", 1)
            self.clients.append(PSClient(host, int(port), timeout_s))
        self.router = router or hash_router(len(self.clients))
        self.pool = ThreadPoolExecutor(max_workers=max(1, len(self.clients)))

    def _group(self, keys: Sequence[str]) -> Dict[int, List[str]]:
        g: Dict[int, List[str]] = {}
        for k in keys:
            g.setdefault(self.router(k), []).append(k)
        return g

    def get(self, key: str):
        return self.clients[self.router(key)].get(key)

    def get_list(self, keys: Sequence[str]):
        out = {}
        futs = [self.pool.submit(self.clients[s].get_list, ks) for s, ks in self._group(keys).items()]
        for f in futs:
            out.update(f.result())
        return out

    def update(self, key: str, value, replace: bool = False):
        return self.clients[self.router(key)].update(key, value, replace)

    def update_list(self, items: Dict[str, object], replace: bool = False):
        out = {}
        futs = [self.pool.submit(self.clients[s].update_list, {k: items[k] for k in ks}, replace)
                for s, ks in self._group(list(items)).items()]
        for f in futs:
            out.update(f.result())
        return out

    def push(self, grads: Dict[str, object], updater_spec: str, apply_now: bool = False) -> None:
        futs = [self.pool.submit(self.clients[s].push, {k: grads[k] for k in ks}, updater_spec, apply_now)
                for s, ks in self._group(list(grads)).items()]
        for f in futs:
            f.result()

    def _key_groups(self, keys: torch.Tensor) -> Dict[int, torch.Tensor]:
        """Row keys -> server (the row analogue of the key router): multiplicative hash mod S."""
        k = keys.detach().cpu().long()
        s = torch.remainder((k * 0x9E3779B1) >> 16, len(self.clients))
        return {int(i): torch.nonzero(s == i).reshape(-1) for i in torch.unique(s).tolist()}

    def row_pull(self, table: str, dim: int, keys: torch.Tensor, lo: float = 0.0, hi: float = 0.0,
                 seed: int = 0) -> torch.Tensor:
        keys = keys.detach().cpu().long()
        out = torch.empty(keys.numel(), int(dim))
        groups = self._key_groups(keys)
        futs = {s: self.pool.submit(self.clients[s].row_pull, table, dim, keys[pos], lo, hi, seed)
                for s, pos in groups.items()}
        for s, f in futs.items():
            out[groups[s]] = f.result()
        return out

    def row_push(self, table: str, dim: int, keys: torch.Tensor, grads, updater_spec: str,
                 apply_now: bool = False) -> None:
        keys = keys.detach().cpu().long()
        g = torch.as_tensor(_np(grads)).reshape(keys.numel(), int(dim))
        futs = [self.pool.submit(self.clients[s].row_push, table, dim, keys[pos], g[pos], updater_spec, apply_now)
                for s, pos in self._key_groups(keys).items()]
        for f in futs:
            f.result()

    def barrier(self, worker: int = 0) -> int:
        """Barrier on ALL shards (net/PSRouterClient.java:131-151)."""
        futs = [self.pool.submit(c.barrier, worker) for c in self.clients]
        return max(f.result() for f in futs)

    def clock(self, worker: int, c: int) -> int:
        futs = [self.pool.submit(cl.clock, worker, c) for cl in self.clients]
        return min(f.result() for f in futs)

    def rendezvous(self, worker: int = 0) -> int:
        """Meet every worker on every shard (used around a store reload)."""
        futs = [self.pool.submit(c.rendezvous, worker) for c in self.clients]
        return max(f.result() for f in futs)

    def register_updater(self, spec: str) -> None:
        for c in self.clients:
            c.register_updater(spec)

    def stats(self) -> List[dict]:
        return [c.stats() for c in self.clients]

    def save(self, path_prefix: str) -> None:
        for i, c in enumerate(self.clients):
            c.save(f"{path_prefix}.shard{i}")

    def load(self, path_prefix: str) -> None:
        for i, c in enumerate(self.clients):
            c.load(f"{path_prefix}.shard{i}")

    def shutdown(self) -> None:
        for c in self.clients:
            c.shutdown()


def main(argv=None):  # pragma: no cover - CLI
    ap = argparse.ArgumentParser(description="ps_amd dedicated parameter server (TCP)")
    ap.add_argument("--port", type=int, default=8890)
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--mode", default="bsp", choices=["bsp", "ssp", "asp"])
    ap.add_argument("--staleness", type=int, default=0)
    ap.add_argument("--bind-any", action="store_true")
    a = ap.parse_args(argv)
    s = PServer(a.port, a.workers, a.mode, a.staleness, bind_any=a.bind_any).start()
    print(f"ps_amd PServer listening on {s.port} ({a.mode}, workers={a.workers})", flush=True)
    s.wait()
    s.stop()


if __name__ == "__main__":  # pragma: no cover
    main()
