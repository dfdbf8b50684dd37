"""Sparse-row ops for embedding / wide tables (HIP on GPU, torch on CPU).

``dedup_rows`` is the worker side of push_rows: it turns per-occurrence gradient rows into
(unique ids, reduced rows).  The sort/unique step uses torch (rocPRIM radix sort on the
GPU); the reduction itself is the deterministic ``segment_reduce_rows`` HIP kernel.
"""
from __future__ import annotations

import torch

from ._ext import native, use_native

ACT_NONE, ACT_RELU, ACT_LEAKY, ACT_SIGMOID = 0, 1, 2, 3


def _act_ref(x: torch.Tensor, act: int) -> torch.Tensor:
    if act == ACT_RELU:
        return torch.relu(x)
    if act == ACT_LEAKY:
        return torch.where(x > 0, x, 0.01 * x)
    if act == ACT_SIGMOID:
        return 0.001 + 0.998 * torch.sigmoid(x)
    return x


def gather_rows(table: torch.Tensor, rows: torch.Tensor, out: torch.Tensor | None = None, out_off: int = 0,
                act: int = ACT_NONE) -> torch.Tensor:
    """out[:, out_off:out_off+dim] = act(table[rows])."""
    dim = table.shape[1]
    if out is None:
        out = torch.empty(rows.numel(), dim, dtype=table.dtype, device=table.device)
    if use_native(table, rows):
        native().gather_rows(table, rows.contiguous(), out, int(out_off), int(act))
        return out
    out[:, out_off:out_off + dim] = _act_ref(table[rows].float(), act).to(out.dtype)
    return out


def segment_reduce_rows(src: torch.Tensor, perm: torch.Tensor, seg_off: torch.Tensor, out: torch.Tensor,
                        mean: bool = False) -> torch.Tensor:
    if use_native(src, perm):
        native().segment_reduce_rows(src, perm, seg_off, out, bool(mean))
        return out
    srt = src[perm].float()
    cnt = (seg_off[1:] - seg_off[:-1])
    seg_ids = torch.repeat_interleave(torch.arange(cnt.numel()), cnt)
    acc = torch.zeros(out.shape, dtype=torch.float32)
    acc.index_add_(0, seg_ids, srt)
    if mean:
        acc /= cnt.clamp(min=1).float()[:, None]
    out.copy_(acc.to(out.dtype))
    return out


def dedup_rows(ids: torch.Tensor, grads: torch.Tensor, mean: bool = False, out_dtype=None):
    """(unique_ids, reduced_grads[u]) where reduced = sum (or mean) over occurrences."""
    ids = ids.reshape(-1)
    grads = grads.reshape(ids.numel(), -1)
    uniq, inverse, counts = torch.unique(ids, sorted=True, return_inverse=True, return_counts=True)
    perm = torch.argsort(inverse, stable=True)
    seg_off = torch.zeros(uniq.numel() + 1, dtype=torch.int64, device=ids.device)
    torch.cumsum(counts, 0, out=seg_off[1:])
    out = torch.empty(uniq.numel(), grads.shape[1], dtype=out_dtype or grads.dtype, device=grads.device)
    segment_reduce_rows(grads.contiguous(), perm, seg_off, out, mean)
    return uniq, out


def scatter_add_rows(src: torch.Tensor, rows: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    if use_native(src, table):
        native().scatter_add_rows(src.contiguous(), rows.contiguous(), table)
        return table
    table.index_add_(0, rows, src.float())
    return table


def embedding_bag_fwd(table: torch.Tensor, ids: torch.Tensor, out: torch.Tensor, out_off: int = 0,
                      act: int = ACT_NONE) -> torch.Tensor:
    """out[b, off + f*dim + d] = act(table[ids[b, f], d]) -- fused field lookup + concat."""
    if use_native(table, ids):
        native().embedding_bag_fwd(table, ids.contiguous(), out, int(out_off), int(act))
        return out
    b, f = ids.shape
    dim = table.shape[1]
    out[:, out_off:out_off + f * dim] = _act_ref(table[ids].reshape(b, f * dim), act).to(out.dtype)
    return out


def sparse_lr_fwd(w: torch.Tensor, ids: torch.Tensor, bias: torch.Tensor | None, out: torch.Tensor) -> torch.Tensor:
    """out[b] = sum_f w[ids[b,f] mod H] + bias (wide part)."""
    if use_native(w, ids):
        native().sparse_lr_fwd(w, ids.contiguous(), bias, out)
        return out
    h = w.numel()
    idx = torch.remainder(ids, h)
    z = w.reshape(-1)[idx].sum(1)
    if bias is not None:
        z = z + bias.reshape(())
    out.copy_(z.reshape(out.shape))
    return out


_M32 = 0xFFFFFFFF


def philox_u01(seed: int, ctr: torch.Tensor, ctr_hi: torch.Tensor | None = None) -> torch.Tensor:
    """uniform [0, 1) from the 4 words of Philox-4x32-10(seed, ctr) -> [n, 4] -- bit-identical
    to ``Philox::gen`` + ``u01`` in csrc/include/psamd_device.h (and the host copy in the native
    server), computed with int64 torch ops so the CPU oracle initialises rows exactly like the
    HIP kernel."""
    ctr = ctr.long()
    c0, c1 = ctr & _M32, (ctr >> 32) & _M32
    if ctr_hi is None:
        c2 = torch.zeros_like(c0)
        c3 = torch.zeros_like(c0)
    else:  # 128-bit counter: high 64 bits
        hi = ctr_hi.long().expand_as(ctr)
        c2, c3 = hi & _M32, (hi >> 32) & _M32
    k0, k1 = int(seed) & _M32, (int(seed) >> 32) & _M32
    for _ in range(10):
        p0 = 0xD2511F53 * c0  # < 2^64: wraps in int64 with the same low bits
        p1 = 0xCD9E8D57 * c2
        hi0, lo0 = (p0 >> 32) & _M32, p0 & _M32
        hi1, lo1 = (p1 >> 32) & _M32, p1 & _M32
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + 0x9E3779B9) & _M32
        k1 = (k1 + 0xBB67AE85) & _M32
    return torch.stack([(c >> 8).float() * (1.0 / 16777216.0) for c in (c0, c1, c2, c3)], dim=-1)


def init_values(seed: int, keys: torch.Tensor, dim: int, lo: float, hi: float) -> torch.Tensor:
    """Deterministic first-touch values of rows ``keys`` ([n] int64 global keys) -> [n, dim]:
    element c is word c % 4 of Philox(seed, counter = (c // 4, key)) -- a 128-bit counter, so
    keys that differ only in their high (field) bits still get independent rows."""
    q = torch.arange((dim + 3) // 4, dtype=torch.int64, device=keys.device)
    ctr = q[None, :].expand(keys.numel(), -1)
    khi = keys.long()[:, None].expand_as(ctr)
    u = philox_u01(seed, ctr.reshape(-1), khi.reshape(-1)).reshape(keys.numel(), -1)[:, :dim]
    return lo + (hi - lo) * u


def lazy_init_rows(table: torch.Tensor, rows: torch.Tensor, flags: torch.Tensor, seed: int, row_base: int,
                   lo: float, hi: float, keys: torch.Tensor | None = None) -> None:
    """Initialise rows not yet touched (flags==0) deterministically from (seed, global key);
    the key is ``keys[r]`` when given, else ``rows[r] + row_base``.  Negative rows skipped."""
    if use_native(table, rows):
        native().lazy_init_rows(table, rows.contiguous(), flags, int(seed), int(row_base), float(lo), float(hi),
                                None if keys is None else keys.contiguous())
        return
    rows = rows.long()
    k = rows + row_base if keys is None else keys.long()
    ok = rows >= 0
    rows, k = rows[ok], k[ok]
    new = flags[rows] == 0
    rows, k = rows[new], k[new]
    if rows.numel():
        table[rows] = init_values(seed, k, table.shape[1], lo, hi).to(table.dtype)
        flags[rows] = 1


def hash_slots(hkeys: torch.Tensor, ids: torch.Tensor, insert: bool, status: torch.Tensor) -> torch.Tensor:
    """Slots of ``ids`` in the device open-addressing map ``hkeys`` (HIP kernel, GPU only)."""
    out = torch.empty_like(ids)
    native().hash_slots(hkeys, ids.contiguous(), out, bool(insert), status)
    return out


class _GatherUnique(torch.autograd.Function):
    """out[k] = leaf[inv[k]] (cast to out_dtype); backward = deterministic segment sum of the
    output gradient per unique row (sorted-order perm + seg_off), no atomics, no sort."""

    @staticmethod
    def forward(ctx, leaf, inv, perm, seg_off, out_dtype):
        out = torch.empty(inv.numel(), leaf.shape[1], dtype=out_dtype, device=leaf.device)
        native().gather_rows(leaf, inv, out, 0, ACT_NONE)
        ctx.save_for_backward(perm, seg_off)
        ctx.nrows, ctx.ldtype = leaf.shape[0], leaf.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        perm, seg_off = ctx.saved_tensors
        dleaf = torch.empty(ctx.nrows, dout.shape[1], dtype=ctx.ldtype, device=dout.device)
        native().segment_reduce_rows(dout.contiguous(), perm, seg_off, dleaf, False)
        return dleaf, None, None, None, None


def unique_with_segments(ids: torch.Tensor):
    """(uniq, inv, counts, perm, seg_off) of a flat id vector: perm lists positions in sorted-id
    order (stable), seg_off[u]..seg_off[u+1] the occurrences of uniq[u] within perm."""
    ids = ids.reshape(-1)
    srt, perm = torch.sort(ids, stable=True)
    uniq, inv_sorted, counts = torch.unique_consecutive(srt, return_inverse=True, return_counts=True)
    inv = torch.empty_like(inv_sorted)
    inv[perm] = inv_sorted
    seg_off = torch.zeros(uniq.numel() + 1, dtype=torch.int64, device=ids.device)
    torch.cumsum(counts, 0, out=seg_off[1:])
    return uniq, inv, counts, perm, seg_off


def gather_unique(leaf: torch.Tensor, inv: torch.Tensor, perm: torch.Tensor, seg_off: torch.Tensor,
                  out_dtype=None) -> torch.Tensor:
    """leaf[inv] (optionally cast) with a segment-sum backward; GPU path = HIP gather_rows /
    segment_reduce_rows, CPU = torch indexing."""
    out_dtype = out_dtype or leaf.dtype
    if use_native(leaf, inv):
        return _GatherUnique.apply(leaf, inv.reshape(-1), perm, seg_off, out_dtype)
    return leaf[inv.reshape(-1)].to(out_dtype)
