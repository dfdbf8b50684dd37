"""Weight gradients on a second HIP stream, overlapped with the data-gradient chain.

In a ResNet backward the data gradients form one serial chain (block i's dx feeds block i-1),
while every weight gradient is a leaf: nothing but the optimizer reads it.  The chain is mostly
HBM-bound (BN applies, 1x1 data grads at 5+ TB/s), the weight gradients are MFMA-bound split-K
GEMMs, so running them on their own stream lets the CU dispatcher fill the MFMA-idle cycles of
the HBM-bound kernels with weight-gradient workgroups (two hardware queues feeding one chip).

Protocol (``Fork``):
  * ``fork()`` records an event on the compute stream after the operands of the next weight
    gradients were enqueued; the side stream waits on it;
  * ``run(fn, *inputs)`` enqueues ``fn`` on the side stream; every input tensor is
    ``record_stream``-ed so the caching allocator does not hand its memory to the compute
    stream before the side stream is done with it; outputs are allocated on the side stream
    and laid out like their parameter (so AccumulateGrad adopts them without a copy kernel on
    the compute stream);
  * the first fork of each ``Fork`` queues an autograd end-of-backward callback that makes
    the compute stream wait for the side stream -- whatever runs after ``loss.backward()``
    (an optimizer, a checkpoint) sees finished gradients;
  * consumers that read gradients DURING backward (the parameter-server bucket hooks,
    parallel/colocated.py ``_launch``) call ``join(stream)`` before reading.

Policy (``enabled``): on for batches up to 512 per GPU (ResNet-50 bs256 +0.6 / +2.4 %: the
layer-3/4 grids leave CUs idle) and, for a rank that owns its GPU, at any batch (bs1024 +0.35 %, where
the compute stream's HBM-bound kernels stretch by nearly as much as the weight gradients hide --
round 3's kernels lost 1.5 % there, profiles/r3_wgrad_side_stream_ab.txt; round 4:
profiles/r4_wgrad_stream_policy.txt).  ``PS_AMD_WGRAD_STREAM=1`` / ``0`` forces it,
``PS_AMD_WGRAD_STREAM_MAX_IMAGES`` sets the batch cap.  Also off on CPU, under graph capture, and when a
parameter already holds a gradient (micro-batch accumulation would make AccumulateGrad add on the
compute stream).
"""
from __future__ import annotations

import os
import threading
from typing import Callable, Dict, Optional

import torch

_STREAMS: Dict[int, torch.cuda.Stream] = {}
_lock = threading.Lock()
# storage of the gradients produced on a side stream during the current backward (cleared by the
# end-of-backward join): the parameter server lands a bucket from the side stream only when one of
# its gradients is among them -- a cross-queue hop costs ~0.1-0.6 ms at the step boundary
_SIDE_PTRS: set = set()
# side-stream work enqueued / joined so far, per side stream: every Fork of a backward queues an
# end-of-backward callback, but only the first one that finds unjoined work makes the compute stream
# wait (16 fused blocks queued 16 waits -- 16 barrier packets, a 0.09 ms bubble before the next
# forward: profiles/r6_step_boundary_gap.txt)
_WORK: Dict[int, int] = {}
_JOINED: Dict[int, int] = {}


def produced_on_side(t: Optional[torch.Tensor]) -> bool:
    """Whether ``t`` (a gradient) was written by a side-stream weight gradient of this backward."""
    return t is not None and t.device.type == "cuda" and t.data_ptr() in _SIDE_PTRS


def _ranks_per_device() -> int:
    from ..parallel.transport import ranks_per_device

    return ranks_per_device()


def enabled(images: Optional[int] = None) -> bool:
    """PS_AMD_WGRAD_STREAM=1: always, 0: never; unset / auto: for batches of at most
    PS_AMD_WGRAD_STREAM_MAX_IMAGES images per GPU -- by default any batch when this rank owns its
    GPU (``ranks_per_device() == 1``: a single process, or one rank per GPU on a node) and 512
    when several ranks share one GPU.  ResNet-50 bs256 +0.6 / +2.4 % on two boxes, bs1024 +0.35 % over three
    interleaved pairs on one box (profiles/r4_wgrad_stream_policy.txt); per-layer row thresholds
    (layers 3-4 only, or 2-4) measured below all layers.  With peers the large batches stay on
    one stream only where ranks SHARE a device: four bs1024 ranks on one GPU ran 4x slower with the
    side stream (profiles/r4_wgrad_stream_policy.txt), while a rank that owns its GPU is exactly
    the measured single-process case, whatever WORLD_SIZE is."""
    mode = os.environ.get("PS_AMD_WGRAD_STREAM", "auto")
    if mode in ("0", "1"):
        return mode == "1"
    if images is None:
        return False
    cap = os.environ.get("PS_AMD_WGRAD_STREAM_MAX_IMAGES")
    if cap is None:
        return images <= 512 or _ranks_per_device() == 1
    return images <= int(cap)


def side_stream(device: torch.device) -> torch.cuda.Stream:
    """The device's weight-gradient side stream (created on first use).  A CU-masked variant
    (hipExtStreamCreateWithCUMask) was measured and removed: no gain (README, round-6 prune)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    with _lock:
        s = _STREAMS.get(idx)
        if s is None:
            s = torch.cuda.Stream(device=idx)
            _STREAMS[idx] = s
        return s


def active(device: torch.device) -> Optional[torch.cuda.Stream]:
    """The device's side stream if weight gradients were ever put on it, else None."""
    if not _STREAMS or device.type != "cuda":
        return None
    return _STREAMS.get(device.index if device.index is not None else torch.cuda.current_device())


def join(stream: Optional[torch.cuda.Stream] = None, device: Optional[torch.device] = None) -> None:
    """Make ``stream`` (default: the current stream) wait for every weight gradient enqueued
    on the side stream so far."""
    if not _STREAMS:
        return
    stream = stream if stream is not None else torch.cuda.current_stream(device)
    side = _STREAMS.get(stream.device_index)
    if side is not None and side is not stream:
        stream.wait_stream(side)


def _match_layout(g: torch.Tensor, like: torch.Tensor) -> torch.Tensor:
    """``g`` with ``like``'s strides (a copy on the current -- side -- stream if they differ)."""
    if g.shape != like.shape:
        g = g.reshape(like.shape) if g.is_contiguous() else g.contiguous().reshape(like.shape)
    if all(gs == ls for gs, ls, n in zip(g.stride(), like.stride(), like.shape) if n != 1):
        return g
    out = torch.empty_strided(like.shape, like.stride(), dtype=g.dtype, device=g.device)
    out.copy_(g)
    return out


class Fork:
    """Per-backward helper (see module docstring)."""

    def __init__(self, device: torch.device, params=(), images: Optional[int] = None):
        self.on = (enabled(images) and device.type == "cuda" and not torch.cuda.is_current_stream_capturing()
                   and all(p is None or p.grad is None for p in params))
        self.queued = False
        if self.on:
            self.main = torch.cuda.current_stream(device)
            self.side = side_stream(device)

    def fork(self) -> None:
        if not self.on:
            return
        ev = torch.cuda.Event()
        ev.record(self.main)
        self.side.wait_event(ev)
        if not self.queued:  # one end-of-backward join per Fork (no state across passes)
            self.queued = True
            main, side = self.main, self.side

            def _join():
                k = id(side)
                if _JOINED.get(k, 0) < _WORK.get(k, 0):
                    main.wait_stream(side)
                    _JOINED[k] = _WORK[k]
                _SIDE_PTRS.clear()

            torch.autograd.Variable._execution_engine.queue_callback(_join)

    def run(self, fn: Callable, *inputs: torch.Tensor, like: Optional[torch.Tensor] = None):
        """``fn()`` on the side stream (inputs protected from reuse); with ``like`` the result is
        returned in ``like``'s layout."""
        if not self.on:
            out = fn()
            return _match_layout(out, like) if like is not None else out
        for t in inputs:
            if t is not None:
                t.record_stream(self.side)
        with torch.cuda.stream(self.side):
            out = fn()
            if like is not None:
                out = _match_layout(out, like)
        if isinstance(out, torch.Tensor):
            _SIDE_PTRS.add(out.data_ptr())
        _WORK[id(self.side)] = _WORK.get(id(self.side), 0) + 1
        return out
