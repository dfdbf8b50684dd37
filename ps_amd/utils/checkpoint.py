"""Sharded checkpoint / resume (the reference keeps everything in memory).

Every rank writes ITS server shard -- fp32 master weights + optimizer state of the ranges
it owns (ColocatedPS.shard_state), its sparse-table rows + init flags + optimizer state,
the PS clock -- to ``<dir>/step<k>/rank<r>.pt``; rank 0 also writes ``manifest.json``
(key -> bucket/offset/shape/dtype, bucket layout, world size, step, data cursors, seeds).
Writes run on a background thread from host copies taken at a round boundary, so training
continues while the file is written.  Loading is with ``torch.load(weights_only=True)``
(tensors / plain containers only) and rebuilds every replica with one pull.

Commit protocol: every rank writes ``rank<r>.pt`` atomically (tmp + rename); rank 0's writer
then waits until all ``world`` rank files of that step exist and only then writes ``COMMIT``.
``latest()`` / ``load(None)`` consider committed steps only, so after a crash in the middle of
a save every rank resumes from the same, complete step.
"""
from __future__ import annotations

import json
import os
import threading
from typing import Dict, Optional

import torch


class CheckpointManager:
    def __init__(self, directory: str, rank: int = 0, world: int = 1, keep: int = 2, commit_timeout_s: float = 600.0):
        self.dir = directory
        self.rank, self.world, self.keep = rank, world, keep
        self.commit_timeout_s = commit_timeout_s
        self._thread: Optional[threading.Thread] = None
        os.makedirs(directory, exist_ok=True)

    def _path(self, step: int) -> str:
        return os.path.join(self.dir, f"step{step:08d}")

    def save(self, step: int, ps=None, tables: Optional[Dict[str, object]] = None, extra: Optional[dict] = None,
             blocking: bool = False) -> str:
        """Snapshot now (host copies), write asynchronously."""
        self.wait()
        state = {"step": step, "world": self.world, "rank": self.rank}
        if ps is not None:
            state["ps"] = ps.shard_state()
        if tables:
            # rows + init flags + optimizer state + the id -> slot map of this rank's shard
            state["tables"] = {name: t.state_dict() for name, t in tables.items()}
        if extra:
            state["extra"] = extra
        path = self._path(step)

        def write():
            os.makedirs(path, exist_ok=True)
            tmp = os.path.join(path, f"rank{self.rank}.pt.tmp")
            torch.save(state, tmp)
            os.replace(tmp, os.path.join(path, f"rank{self.rank}.pt"))
            if self.rank == 0:
                man = {"step": step, "world": self.world, "extra": extra or {}}
                if ps is not None:
                    man["keys"] = state["ps"]["manifest"]
                    man["buckets"] = state["ps"]["buckets"]
                with open(os.path.join(path, "manifest.json"), "w") as f:
                    json.dump(man, f, indent=1)
                self._commit(path)
                self._gc()

        if blocking:
            write()
        else:
            self._thread = threading.Thread(target=write, daemon=True)
            self._thread.start()
        return path

    def wait(self) -> None:
        if self._thread is not None:
            self._thread.join()
            self._thread = None

    def _commit(self, path: str) -> None:
        """rank 0: COMMIT once every rank's shard of this step is on disk."""
        import time

        deadline = time.time() + self.commit_timeout_s
        want = [os.path.join(path, f"rank{r}.pt") for r in range(self.world)]
        while not all(os.path.exists(f) for f in want):
            if time.time() > deadline:
                return  # never committed: resume falls back to the previous step
            time.sleep(0.01)
        with open(os.path.join(path, "COMMIT"), "w") as f:
            f.write("ok\n")

    def committed(self) -> list:
        return sorted(int(d[4:]) for d in os.listdir(self.dir)
                      if d.startswith("step") and os.path.exists(os.path.join(self.dir, d, "COMMIT")))

    def _gc(self) -> None:
        if self.rank != 0:
            return
        keep = set(self.committed()[-self.keep:])
        steps = sorted(d for d in os.listdir(self.dir) if d.startswith("step"))
        for d in steps[:-self.keep]:
            if int(d[4:]) in keep:
                continue
            p = os.path.join(self.dir, d)
            for f in os.listdir(p):
                os.remove(os.path.join(p, f))
            os.rmdir(p)

    def latest(self) -> Optional[int]:
        """Newest COMMITTED step (all ranks' shards complete), or None."""
        c = self.committed()
        return c[-1] if c else None

    def load(self, step: Optional[int] = None, ps=None, tables: Optional[Dict[str, object]] = None) -> dict:
        step = self.latest() if step is None else step
        if step is None:
            raise FileNotFoundError(f"no checkpoint in {self.dir}")
        state = torch.load(os.path.join(self._path(step), f"rank{self.rank}.pt"), weights_only=True)
        if state["world"] != self.world:
            raise ValueError(f"checkpoint world {state['world']} != current world {self.world} (no elasticity)")
        if ps is not None:
            ps.load_shard_state(state["ps"])
        for name, t in (tables or {}).items():
            t.load_state_dict(state["tables"][name])
        return state
