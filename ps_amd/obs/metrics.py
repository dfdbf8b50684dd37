"""Metric emission (reference: visual/UiClient.java ``plot(id, x, y)``, async, fire-and-forget).

``plot(id, y, x)`` records a point in-process, appends a JSON line to ``PS_AMD_METRICS_PATH``
(one file per rank) and, when a UI server address is configured, hands the point to a
background sender thread (never blocks the training step -- same contract as the
reference's gzip'd async gRPC stub).  The address comes from the reference flags
``-DuiHost`` / ``-DuiPort`` (context/Context.java:81-82, visual/UiClient.java:25-27) or
``PS_AMD_UI_ADDR``; only the reporting replica sends -- replica 0 of a ``-DisMajor=1`` worker
(``ctx.is_report_ui()``, context/Context.java:94-100).  Structured step records (``log_step``) carry
samples/s, push/pull bytes, staleness and server-update time.
"""
from __future__ import annotations

import json
import os
import queue
import threading
import time
from collections import defaultdict
from typing import Dict, List, Optional, Tuple

_series: Dict[str, List[Tuple[float, float]]] = defaultdict(list)
_lock = threading.Lock()
_file = None
_file_path: Optional[str] = None
_client = None


def _rank() -> int:
    return int(os.environ.get("RANK", "0"))


def _open():
    global _file, _file_path
    p = os.environ.get("PS_AMD_METRICS_PATH", "")
    if p != _file_path:
        if _file is not None:
            _file.close()
        _file = None
        _file_path = p
        if p:
            root, ext = os.path.splitext(p)
            os.makedirs(os.path.dirname(os.path.abspath(p)), exist_ok=True)
            _file = open(f"{root}.rank{_rank()}{ext or '.jsonl'}", "a", buffering=1)
    return _file


def plot(name: str, y: float, x: float) -> None:
    """Record point (x, y) of series ``name`` (reference argument order: plot(id, y, step))."""
    y, x = float(y), float(x)
    with _lock:
        _series[name].append((x, y))
        f = _open()
        if f is not None:
            f.write(json.dumps({"t": time.time(), "series": name, "x": x, "y": y}) + "\n")
    c = _client or _auto_client()
    if c is not None and _report_ui():
        c.send(name, x, y)


def _report_ui() -> bool:
    from ..context import ctx

    return ctx.is_report_ui()


def log_step(**fields) -> None:
    with _lock:
        f = _open()
        if f is not None:
            f.write(json.dumps({"t": time.time(), "kind": "step", **fields}) + "\n")


def series(name: str) -> List[Tuple[float, float]]:
    with _lock:
        return list(_series.get(name, []))


def names() -> List[str]:
    with _lock:
        return list(_series)


def reset() -> None:
    with _lock:
        _series.clear()


class UiClient:
    """Async point sender to a UiServer (http POST /plot), bounded queue, drops on overflow."""

    def __init__(self, host: str, port: int, maxsize: int = 10000):
        self.url = f"http://{host}:{port}/plot"
        self.q: "queue.Queue" = queue.Queue(maxsize=maxsize)
        self.dropped = 0
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def send(self, name: str, x: float, y: float) -> None:
        try:
            self.q.put_nowait((name, x, y))
        except queue.Full:
            self.dropped += 1

    def _run(self):
        import urllib.request

        while True:
            batch = [self.q.get()]
            try:
                while len(batch) < 256:
                    batch.append(self.q.get_nowait())
            except queue.Empty:
                pass
            body = json.dumps([{"id": n, "x": x, "y": y} for n, x, y in batch]).encode()
            try:
                req = urllib.request.Request(self.url, data=body, headers={"Content-Type": "application/json"})
                urllib.request.urlopen(req, timeout=2).read()
            except Exception:
                self.dropped += len(batch)

    def flush(self, timeout: float = 2.0) -> None:
        t0 = time.time()
        while not self.q.empty() and time.time() - t0 < timeout:
            time.sleep(0.01)


_auto: Dict[Tuple[str, int], "UiClient"] = {}


def _auto_client():
    """The UI client of the configured address (one sender thread per address)."""
    addr = os.environ.get("PS_AMD_UI_ADDR", "")
    if addr:
        host, port = addr.rsplit(":", 1)
        key = (host, int(port))
    else:
        from ..context import ctx

        key = ctx.cfg.ui_address()
        if key is None:
            return None
    c = _auto.get(key)
    if c is None:
        c = _auto[key] = UiClient(*key)
    return c


def set_client(c: Optional[UiClient]) -> None:
    global _client
    _client = c
