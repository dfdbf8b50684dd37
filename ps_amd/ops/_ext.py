"""Loader for the in-tree HIP extension ``ps_amd._C``.

Policy (matches the round-end "native code loaded" check):
  * a tensor on the GPU ALWAYS runs the HIP kernel.  If the extension is missing or fails
    to load on a machine with a GPU, the op raises -- there is no silent eager fallback.
  * a tensor on the CPU runs the plain-torch reference implementation (used by the CPU
    test-suite and the gloo plumbing configs).
"""
from __future__ import annotations

import importlib
import os

import torch

_C = None
_ERR: Exception | None = None


def _load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return _C
    try:
        _C = importlib.import_module("ps_amd._C")
    except Exception as e:  # pragma: no cover - exercised on broken installs only
        _ERR = e
        if os.environ.get("PS_AMD_AUTOBUILD", "0") == "1":
            from .. import _build

            _build.build()
            _ERR = None
            _C = importlib.import_module("ps_amd._C")
    return _C


def native():
    """Return the extension module or raise a loud error."""
    m = _load()
    if m is None:
        raise RuntimeError(
            f"ps_amd._C HIP extension is not available ({_ERR!r}); build it with "
            "`python -m ps_amd._build` (hipcc --offload-arch=gfx950)"
        )
    return m


def available() -> bool:
    return _load() is not None


def use_native(*tensors: torch.Tensor) -> bool:
    """True if the op must run the HIP kernel (any operand lives on the GPU)."""
    on_gpu = any(t is not None and t.is_cuda for t in tensors)
    if on_gpu:
        native()  # raise if missing
    return on_gpu
