"""Data pipeline (data/*.java).

  DataSource / FileSource  line source with ``offset`` / ``step`` worker sharding
                           (data/DataSource.java:8-46).  The reference never sets them, so
                           every worker reads the same lines (Q11); here they default to
                           (rank, world) from the environment.
  Feature, Parser, LibsvmParser   ``label idx:val ...`` -> [Feature] (data/LibsvmParser.java)
  DataSet                  reader threads -> bounded queue of parsed batches; ``next()``
                           polls with a timeout, ``has_next``/``reset`` (data/DataSet.java:14-103);
                           subclasses implement ``parse_feature(lines) -> dict of tensors``.
  NativeBatchDataSet       the same contract on the C++ threaded reader
                           (csrc/runtime/loader.cpp) for csv / libsvm / ctr files.
  synthetic_*              deterministic generators for benchmarks and tests (no network,
                           no downloaded datasets).
"""
from __future__ import annotations

import os
import queue
import threading
from dataclasses import dataclass
from typing import Dict, Iterator, List, Optional

import numpy as np
import torch


def _rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))


class DataSource:
    def __init__(self, offset: Optional[int] = None, step: Optional[int] = None):
        r, w = _rank_world()
        self.offset = r if offset is None else int(offset)
        self.step = w if step is None else int(step)
        if not (0 <= self.offset < self.step):
            raise ValueError("need 0 <= offset < step")

    def read_line(self) -> Optional[str]:  # pragma: no cover - abstract
        raise NotImplementedError

    def reset(self) -> None:  # pragma: no cover - abstract
        raise NotImplementedError


class FileSource(DataSource):
    def __init__(self, path: str, offset: Optional[int] = None, step: Optional[int] = None, skip_header: bool = False):
        super().__init__(offset, step)
        self.path = path
        self.skip_header = skip_header
        self._lock = threading.Lock()
        self.reset()

    def reset(self) -> None:
        with self._lock:
            self._f = open(self.path, "r")
            if self.skip_header:
                self._f.readline()
            self._i = -1

    def read_line(self) -> Optional[str]:
        with self._lock:
            while True:
                line = self._f.readline()
                if not line:
                    return None
                self._i += 1
                if self._i % self.step == self.offset:
                    return line.rstrip("\n")


class MemorySource(DataSource):
    def __init__(self, lines: List[str], offset: Optional[int] = None, step: Optional[int] = None):
        super().__init__(offset, step)
        self.lines = lines
        self.reset()

    def reset(self):
        self._i = self.offset

    def read_line(self):
        if self._i >= len(self.lines):
            return None
        line = self.lines[self._i]
        self._i += self.step
        return line


@dataclass
class Feature:
    idx: int
    value: object


class Parser:
    def parse(self, line: str) -> List[Feature]:  # pragma: no cover - abstract
        raise NotImplementedError


class LibsvmParser(Parser):
    """``label idx:val idx:val ...`` -> [Feature(-1, label), Feature(idx, val), ...]."""

    def parse(self, line: str) -> List[Feature]:
        parts = line.split()
        if not parts:
            return []
        out = [Feature(-1, float(parts[0]))]
        for p in parts[1:]:
            i, v = p.split(":", 1)
            out.append(Feature(int(i), float(v)))
        return out


class CsvParser(Parser):
    """``label,v1,...`` (the MNIST CSV of src/main/resources/mnist_test.csv)."""

    def parse(self, line: str) -> List[Feature]:
        vals = line.split(",")
        return [Feature(-1, float(vals[0]))] + [Feature(i, float(v)) for i, v in enumerate(vals[1:])]


class DataSet:
    """Threaded prefetch of parsed batches into a bounded queue."""

    _END = object()

    def __init__(self, source: DataSource, parser: Parser, batch_size: int, threads: int = 1,
                 queue_depth: Optional[int] = None, drop_last: bool = False):
        self.source, self.parser, self.batch_size = source, parser, int(batch_size)
        self.threads = max(1, threads)
        self.q: "queue.Queue" = queue.Queue(maxsize=queue_depth or self.threads * 2)
        self.drop_last = drop_last
        self._workers: List[threading.Thread] = []
        self._done = 0
        self._lock = threading.Lock()
        self.start()

    def parse_feature(self, rows: List[List[Feature]]) -> Dict[str, torch.Tensor]:  # pragma: no cover
        raise NotImplementedError

    def start(self) -> None:
        self._done = 0
        self._stop = False
        self._peek = None
        for _ in range(self.threads):
            t = threading.Thread(target=self._run, daemon=True)
            t.start()
            self._workers.append(t)

    def _run(self):
        while not self._stop:
            rows = []
            while len(rows) < self.batch_size:
                line = self.source.read_line()
                if line is None:
                    break
                if line.strip():
                    rows.append(self.parser.parse(line))
            if rows and (len(rows) == self.batch_size or not self.drop_last):
                self.q.put(self.parse_feature(rows))
            if len(rows) < self.batch_size:
                break
        with self._lock:
            self._done += 1
            if self._done == self.threads:
                self.q.put(self._END)

    def next(self, timeout: float = 3.0) -> Optional[Dict[str, torch.Tensor]]:
        if self._peek is not None:
            b, self._peek = self._peek, None
            return b
        try:
            b = self.q.get(timeout=timeout)
        except queue.Empty:
            return None
        if b is self._END:
            self.q.put(self._END)
            return None
        return b

    def has_next(self, timeout: float = 60.0) -> bool:
        if self._peek is None:
            self._peek = self.next(timeout)
        return self._peek is not None

    def reset(self) -> None:
        self._stop = True
        for t in self._workers:
            while t.is_alive():
                try:
                    self.q.get_nowait()
                except queue.Empty:
                    pass
                t.join(timeout=0.05)
        self._workers = []
        self.q = queue.Queue(maxsize=self.q.maxsize)
        self.source.reset()
        self.start()

    def __iter__(self) -> Iterator[Dict[str, torch.Tensor]]:
        while True:
            b = self.next()
            if b is None:
                return
            yield b


class MnistDataSet(DataSet):
    """MNIST CSV -> X [B, 784] scaled to [0,1], Y [B] (Mnist.java:45-73)."""

    def __init__(self, path: str, batch_size: int, **kw):
        super().__init__(FileSource(path, kw.pop("offset", None), kw.pop("step", None)), CsvParser(), batch_size, **kw)

    def parse_feature(self, rows):
        y = torch.tensor([r[0].value for r in rows], dtype=torch.long)
        x = torch.tensor([[f.value for f in r[1:]] for r in rows], dtype=torch.float32) / 255.0
        return {"X": x, "Y": y}


class NativeBatchDataSet:
    """DataSet contract on the C++ reader (ps_amd._native.BatchReader)."""

    def __init__(self, path: str, fmt: str, batch_size: int, dims: int = 0, fields: int = 0, threads: int = 2,
                 depth: int = 4, offset: Optional[int] = None, step: Optional[int] = None, drop_last: bool = False,
                 x_scale: float = 1.0, label_dtype=torch.float32):
        from .. import _native  # type: ignore

        r, w = _rank_world()
        self.r = _native.BatchReader(path, fmt, batch_size, dims, fields, r if offset is None else offset,
                                     w if step is None else step, threads, depth, drop_last)
        self.fmt, self.x_scale, self.label_dtype = fmt, x_scale, label_dtype

    def next(self, timeout: float = 3.0) -> Optional[Dict[str, torch.Tensor]]:
        b = self.r.next(timeout)
        if b is None:
            return None
        out = {"Y": torch.from_numpy(b["Y"]).to(self.label_dtype)}
        if "X" in b:
            out["X"] = torch.from_numpy(b["X"]) * self.x_scale
        if "I" in b:
            out["E" if self.fmt == "ctr" else "I"] = torch.from_numpy(b["I"])
        if "V" in b:
            out["V"] = torch.from_numpy(b["V"])
        return out

    def has_next(self) -> bool:
        return self.r.has_next()

    def reset(self) -> None:
        self.r.reset()

    def __iter__(self):
        while True:
            b = self.next()
            if b is None:
                return
            yield b


# ---------------------------------------------------------------------------- synthetic
def synthetic_ctr(n: int, fields: int = 23, numeric: int = 45, ids_per_field: int = 1000, wide_k: int = 0,
                  wide_size: int = 100000, seed: int = 0, device=None) -> Dict[str, torch.Tensor]:
    """CTR-shaped batch with a known logistic ground truth (labels are learnable)."""
    g = torch.Generator().manual_seed(seed)
    E = torch.randint(0, ids_per_field, (n, fields), generator=g)
    X = torch.randn(n, numeric, generator=g)
    gt = torch.Generator().manual_seed(12345)  # fixed "true model" across seeds
    emb_w = torch.randn(fields, ids_per_field, generator=gt) * 0.8
    xw = torch.randn(numeric, generator=gt) * 0.3
    logit = emb_w.gather(1, E.t()).t().sum(1) / fields ** 0.5 + X @ xw
    Y = (torch.rand(n, generator=g) < torch.sigmoid(logit)).float()
    out = {"E": E, "X": X, "Y": Y}
    if wide_k:
        out["W"] = torch.randint(0, 1 << 30, (n, wide_k), generator=g) % wide_size
    if device is not None:
        out = {k: v.to(device) for k, v in out.items()}
    return out


def synthetic_images(n: int, c: int = 3, hw: int = 224, classes: int = 1000, seed: int = 0, device=None,
                     dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, c, hw, hw, generator=g).to(dtype)
    y = torch.randint(0, classes, (n,), generator=g)
    if device is not None:
        x, y = x.to(device), y.to(device)
    return {"X": x, "Y": y}


def load_reference_mnist(path: Optional[str] = None) -> Dict[str, torch.Tensor]:
    """The 1000-row MNIST CSV bundled with the reference (src/main/resources/mnist_test.csv):
    a plain-text fixture, read with numpy (no pickle)."""
    if path is None:
        import os

        # the reference checkout, else a local copy (data_cache/ is git-ignored: the fixture is
        # not committed, it only travels with the working tree to a GPU box)
        ref = "/root/reference/src/main/resources/mnist_test.csv"
        local = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                             "data_cache", "mnist_test.csv")
        path = os.environ.get("PS_AMD_MNIST_CSV") or (ref if os.path.exists(ref) else local)
    arr = np.loadtxt(path, delimiter=",", dtype=np.float32)
    return {"X": torch.from_numpy(arr[:, 1:] / 255.0), "Y": torch.from_numpy(arr[:, 0]).long()}
