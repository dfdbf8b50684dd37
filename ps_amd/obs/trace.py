"""Tracing: roctx ranges + a per-step timer breakdown (the reference has none).

``range("push")`` emits a roctx range (visible in ``rocprofv3 --marker-trace`` timelines)
through librocprofiler-sdk-roctx / libroctx64 loaded with ctypes; when neither is present
it is a no-op.  ``StepTimer`` accumulates wall-clock phases (fwd_bwd, push, server_update,
pull_wait, exposed_comm) and publishes them to the metrics stream.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from collections import defaultdict
from typing import Dict

_lib = None
_tried = False


def _roctx():
    global _lib, _tried
    if _tried:
        return _lib
    _tried = True
    if os.environ.get("PS_AMD_ROCTX", "1") == "0":
        return None
    for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so"):
        for base in ("", "/opt/rocm/lib/"):
            try:
                lib = ctypes.CDLL(base + name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _lib = lib
                return _lib
            except (OSError, AttributeError):
                continue
    return None


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


class StepTimer:
    def __init__(self):
        self.acc: Dict[str, float] = defaultdict(float)
        self.n = 0

    @contextlib.contextmanager
    def phase(self, name: str, sync=None):
        with range(name):
            t0 = time.perf_counter()
            try:
                yield
            finally:
                if sync is not None:
                    sync()
                self.acc[name] += (time.perf_counter() - t0) * 1e3

    def step_done(self) -> None:
        self.n += 1

    def summary(self) -> Dict[str, float]:
        return {k: v / max(1, self.n) for k, v in self.acc.items()}
