"""Tensor utilities (reference: util/MatrixUtil.java).

  rand_uniform(rows, cols, max)  uniform in [-max, max)        MatrixUtil.rand(row,col,max) :62-74
  rand_gaussian(rows, cols)      N(0, 1)                        MatrixUtil.rand(row,col)     :48-60
  rand_bernoulli(rows, cols, p)  1 with prob p                  MatrixUtil.randBernoulli     :35-47
  hash_ids(x, size)              non-negative x mod size        MatrixUtil.hash              :27-33
  append_rows(offset, dst, src)  dst[offset:offset+len(src)]    MatrixUtil.appendRows        :76-82
  pretty(t)                      compact string                 MatrixUtil.pretty            :14-25
  to_bytes / from_bytes          raw little-endian wire format  FloatMatrix_2_ProtoMatrix   :84-109
                                 (replaces per-element boxed protobuf floats)
  xavier_bound(fan_in, fan_out)  4*sqrt(6/(in+out))             layer/FcLayer.java:39
"""
from __future__ import annotations

import math
import struct
from typing import Optional

import torch


def xavier_bound(fan_in: int, fan_out: int) -> float:
    return float(4.0 * math.sqrt(6.0) / math.sqrt(fan_in + fan_out))


def rand_uniform(rows: int, cols: int, max_abs: float, generator: Optional[torch.Generator] = None,
                 device=None) -> torch.Tensor:
    t = torch.rand(rows, cols, generator=generator, device=device)
    return (t * 2.0 - 1.0) * max_abs


def rand_gaussian(rows: int, cols: int, generator: Optional[torch.Generator] = None, device=None) -> torch.Tensor:
    return torch.randn(rows, cols, generator=generator, device=device)


def rand_bernoulli(rows: int, cols: int, p: float, generator: Optional[torch.Generator] = None,
                   device=None) -> torch.Tensor:
    return (torch.rand(rows, cols, generator=generator, device=device) < p).float()


def hash_ids(x: torch.Tensor, size: int) -> torch.Tensor:
    """Non-negative modulo (the reference's ``x % size`` is negative for negative ids)."""
    return torch.remainder(x.long(), size)


def append_rows(offset: int, dst: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    dst[offset:offset + src.shape[0]] = src
    return dst


def pretty(t: torch.Tensor, max_items: int = 8) -> str:
    flat = t.detach().reshape(-1)[:max_items].tolist()
    more = "..." if t.numel() > max_items else ""
    return f"{tuple(t.shape)}[" + ", ".join(f"{v:.4g}" for v in flat) + more + "]"


_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int64: 3, torch.int32: 4, torch.uint8: 5}
_DT_INV = {v: k for k, v in _DT.items()}


def to_bytes(t: torch.Tensor) -> bytes:
    """Header (dtype, ndim, shape...) + raw contiguous bytes."""
    t = t.detach().contiguous().cpu()
    hdr = struct.pack("<BB", _DT[t.dtype], t.dim()) + struct.pack(f"<{t.dim()}q", *t.shape)
    raw = t.view(torch.uint8).numpy().tobytes() if t.numel() else b""
    return hdr + raw


def from_bytes(b: bytes) -> torch.Tensor:
    dt, nd = struct.unpack_from("<BB", b, 0)
    shape = struct.unpack_from(f"<{nd}q", b, 2)
    off = 2 + 8 * nd
    dtype = _DT_INV[dt]
    buf = bytearray(b[off:])
    t = torch.frombuffer(buf, dtype=torch.uint8) if buf else torch.empty(0, dtype=torch.uint8)
    return t.view(dtype).reshape(shape).clone()
