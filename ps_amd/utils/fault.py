"""Failure detection + fault injection (the reference has neither -- a dead PS
hangs its barrier forever, net/PServer.java:251-258).

* ``Heartbeat``: every rank bumps ``hb/<rank>`` in the c10d TCPStore every ``period`` s on
  a daemon thread; ``Watchdog`` (every rank) scans them and, when a rank has been silent for
  ``timeout`` s, records the failure and invokes ``on_failure`` (default: abort the process
  group and EXIT the process with ``EXIT_PEER_LOST`` so a rank blocked in a collective with a
  dead peer does not hang).  ``start_failure_detection`` wires both from ``Config.heartbeat_s``.
* Recovery = restart every rank from the last committed checkpoint with the same world size:
  ``python -m ps_amd.launch --nproc N --max-restarts R -- <cmd>`` (ps_amd/launch.py) restarts
  the whole job when a rank dies; apps resume from ``Config.checkpoint_dir``.
* Fault injection from ``PS_AMD_FAULT`` (or Config.fault), e.g.
    ``kill:rank=1:step=5``      rank 1 exits hard at step 5 (first attempt only; ``attempt=k``
                                to fire on the k-th restart -- PS_AMD_RESTART is set by launch.py)
    ``delay_push:ms=50``        sleep before every push (staleness tests)
    ``drop_push:p=0.01``        drop a fraction of ASP pushes (TCP topology only)
  ``FaultInjector.at_step(step)`` / ``before_push()`` / ``drop()`` are called by trainers.
"""
from __future__ import annotations

import os
import random
import threading
import time
from typing import Callable, Dict, Optional


def parse_fault(spec: str) -> Dict[str, Dict[str, str]]:
    out: Dict[str, Dict[str, str]] = {}
    for part in filter(None, (spec or "").split(",")):
        fields = part.split(":")
        kind, kv = fields[0], {}
        for f in fields[1:]:
            k, v = f.split("=", 1)
            kv[k] = v
        out[kind] = kv
    return out


class FaultInjector:
    def __init__(self, spec: Optional[str] = None, rank: int = 0, seed: int = 0):
        env = os.environ.get("PS_AMD_FAULT") or os.environ.get("HIPPS_FAULT", "")  # SURVEY §5.3 spelling
        self.spec = parse_fault(spec if spec is not None else env)
        self.rank = rank
        self.rng = random.Random(seed + rank)

    def at_step(self, step: int) -> None:
        k = self.spec.get("kill")
        attempt = int(os.environ.get("PS_AMD_RESTART", "0"))
        if (k and int(k.get("rank", -1)) == self.rank and int(k.get("step", -1)) == step
                and int(k.get("attempt", 0)) == attempt):
            os._exit(int(k.get("code", 17)))

    def before_push(self) -> None:
        d = self.spec.get("delay_push")
        if d and int(d.get("rank", self.rank)) == self.rank:
            time.sleep(float(d.get("ms", 0)) / 1e3)

    def drop(self) -> bool:
        d = self.spec.get("drop_push")
        return bool(d) and self.rng.random() < float(d.get("p", 0))


EXIT_PEER_LOST = 75  # a peer rank stopped heart-beating: the job must restart from a checkpoint


class Heartbeat:
    def __init__(self, store, rank: int, period: float = 1.0):
        self.store, self.rank, self.period = store, rank, period
        self._stop = threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)

    def start(self) -> "Heartbeat":
        self.t.start()
        return self

    def _run(self):
        n = 0
        while not self._stop.is_set():
            n += 1
            try:
                self.store.set(f"hb/{self.rank}", str(time.time()))
            except Exception:
                return
            self._stop.wait(self.period)

    def stop(self):
        self._stop.set()


class Watchdog:
    def __init__(self, store, world: int, timeout: float = 30.0, period: float = 1.0,
                 on_failure: Optional[Callable[[int, float], None]] = None):
        self.store, self.world, self.timeout, self.period = store, world, timeout, period
        self.on_failure = on_failure or self._abort
        self.failed: Dict[int, float] = {}
        self._stop = threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)

    @staticmethod
    def _abort(rank: int, silent_s: float) -> None:
        import sys

        import torch.distributed as dist

        sys.stderr.write(f"[ps_amd watchdog] rank {rank} silent for {silent_s:.1f}s: aborting (exit "
                         f"{EXIT_PEER_LOST})\n")
        sys.stderr.flush()
        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass
        os._exit(EXIT_PEER_LOST)

    def start(self) -> "Watchdog":
        self.t.start()
        return self

    def check(self) -> Dict[int, float]:
        now = time.time()
        out = {}
        for r in range(self.world):
            try:
                if not self.store.check([f"hb/{r}"]):  # get() would block on a missing key
                    continue
                last = float(self.store.get(f"hb/{r}").decode())
            except Exception:
                continue
            if now - last > self.timeout:
                out[r] = now - last
        return out

    def _run(self):
        while not self._stop.is_set():
            for r, s in self.check().items():
                if r not in self.failed:
                    self.failed[r] = s
                    self.on_failure(r, s)
            self._stop.wait(self.period)

    def stop(self):
        self._stop.set()


def start_failure_detection(heartbeat_s: float, rank: int, world: int, store=None):
    """Heartbeat on every rank + a watchdog on every rank (timeout = 5 periods, min 5 s) over
    the default c10d store; returns (heartbeat, watchdog) or None when disabled / world 1."""
    if not heartbeat_s or heartbeat_s <= 0 or world <= 1:
        return None
    if store is None:
        import torch.distributed as dist

        if not dist.is_initialized():
            return None
        from torch.distributed import distributed_c10d

        store = distributed_c10d._get_default_store()
    hb = Heartbeat(store, rank, heartbeat_s).start()
    wd = Watchdog(store, world, timeout=max(5.0, 5 * heartbeat_s), period=heartbeat_s).start()
    return hb, wd
