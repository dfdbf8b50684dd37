"""1-bit sign compression with error feedback (K26)."""
from __future__ import annotations

import torch

from ._ext import native, use_native

CHUNK = 1024


def packed_sizes(n: int) -> tuple[int, int]:
    """(number of int64 words, number of chunk scales) for an n-element gradient."""
    return (n + 63) // 64, (n + CHUNK - 1) // CHUNK


def onebit_pack(g: torch.Tensor, err: torch.Tensor, words: torch.Tensor, scales: torch.Tensor,
                mom: torch.Tensor = None, beta1: float = 0.0) -> None:
    """Compress ``g + err`` into sign bits ``words`` (int64) and per-chunk ``scales``; update ``err``.
    With ``mom`` (1-bit Adam): first ``mom = beta1 mom + (1 - beta1) g`` (stored in mom's dtype), then
    compress ``mom + err`` -- the worker's momentum, not its gradient, crosses the wire."""
    n = g.numel()
    if use_native(g, err):
        native().onebit_pack(g.contiguous(), err, words, scales, mom, float(beta1))
        return
    x = g.float().reshape(-1)
    if mom is not None:
        x = beta1 * mom.float().reshape(-1) + (1.0 - beta1) * x
        mom.reshape(-1).copy_(x)
    c = x + err.float().reshape(-1)
    nw, ns = packed_sizes(n)
    pad = ns * CHUNK - n
    cp = torch.nn.functional.pad(c, (0, pad))
    counts = torch.full((ns,), CHUNK, dtype=torch.float32)
    if pad:
        counts[-1] = CHUNK - pad
    sc = cp.abs().reshape(ns, CHUNK).sum(1) / counts
    scales[:ns].copy_(sc)
    pos = c >= 0
    elem_scale = sc.repeat_interleave(CHUNK)[:n]
    err.reshape(-1).copy_(c - torch.where(pos, elem_scale, -elem_scale))
    bits = torch.nn.functional.pad(pos.to(torch.int64), (0, nw * 64 - n)).reshape(nw, 64)
    shifts = torch.arange(64, dtype=torch.int64)
    # assemble 64-bit words; bit 63 wraps into the sign bit like the device word does
    w = torch.zeros(nw, dtype=torch.int64)
    for b in range(64):
        w |= bits[:, b] << shifts[b]
    words[:nw].copy_(w)


def onebit_momentum(g: torch.Tensor, mom: torch.Tensor, beta1: float) -> None:
    """mom = beta1 mom + (1 - beta1) g: the 1-bit Adam worker momentum during full-precision rounds."""
    if use_native(g, mom):
        native().onebit_momentum(g.contiguous(), mom, float(beta1))
        return
    mom.copy_((beta1 * mom.float() + (1.0 - beta1) * g.float().reshape(mom.shape)).to(mom.dtype))


def onebit_unpack_reduce(words: torch.Tensor, scales: torch.Tensor, out: torch.Tensor, mult: float = 1.0,
                         accumulate: bool = False) -> None:
    """out (+)= mult * sum_w decode(words[w], scales[w])."""
    if use_native(words, out):
        native().onebit_unpack_reduce(words, scales, out, float(mult), bool(accumulate))
        return
    n = out.numel()
    acc = torch.zeros(n, dtype=torch.float32)
    idx = torch.arange(n)
    for w in range(words.shape[0]):
        word = words[w][idx // 64]
        bit = (word >> (idx % 64)) & 1
        sc = scales[w][idx // CHUNK]
        acc += torch.where(bit == 1, sc, -sc)
    acc *= mult
    if accumulate:
        acc += out.float().reshape(-1)
    out.copy_(acc.reshape(out.shape))
