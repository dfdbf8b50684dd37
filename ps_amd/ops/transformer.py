"""Fused transformer row / elementwise ops (csrc/kernels/transformer.hip) with autograd.

  rms_norm(x, w, eps, residual=None)         -> y  |  (s = x + residual, y = RMSNorm(s))
  layer_norm_residual(x, o, g, b, eps, p)    -> LN(x + dropout_p(o))        (BERT post-LN)
  swiglu(gu)                                  -> silu(gu[..., :F]) * gu[..., F:]
  rope_split(qkv, cs, H, KV)                  -> q, k, v  (RoPE + head split + transpose)
  attention_qkv(qkv, H, p, mask)              -> dropout_p(softmax(q k^T / 8)) v over the fused qkv
                                                 projection (csrc/kernels/attention.hip, S <= 128)
  attention_causal_gqa(q, k, v)               -> causal GQA flash attention, heads merged
                                                 (csrc/kernels/flash_attn.hip, head dim 128)

GPU bf16 tensors (row length <= 4096, multiple of 8) take the HIP kernels; everything else
runs the plain torch composition, which is also the numerics oracle in the GPU tests.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from .. import knobs
from ._ext import native


def _hip(*ts) -> bool:
    return all(t is not None and t.is_cuda and t.dtype == torch.bfloat16 for t in ts)


def _seed() -> int:
    # host RNG (no device sync); deterministic under torch.manual_seed
    return int(torch.randint(0, 2 ** 62, (1,)).item())


# ------------------------------------------------------------------------------ RMSNorm
def _rms_ref(x, w, eps):
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype) * w


class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        x = x.contiguous()
        _, y, rstd = native().rmsnorm_fwd(x, None, w.contiguous(), float(eps))
        ctx.save_for_backward(x, w, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, rstd = ctx.saved_tensors
        dx, dw = native().rmsnorm_bwd(dy.contiguous(), x, w, rstd, None)
        return dx, dw.to(w.dtype), None


class _AddRMSNorm(torch.autograd.Function):
    """s = x + r (the residual stream, returned) and y = RMSNorm(s) in one pass; backward
    folds the stream gradient ds into the norm backward (one pass, dx = dr)."""

    @staticmethod
    def forward(ctx, x, r, w, eps):
        s, y, rstd = native().rmsnorm_fwd(x.contiguous(), r.contiguous(), w.contiguous(), float(eps))
        ctx.save_for_backward(s, w, rstd)
        # an unused stream output (the final norm discards s) arrives as None, not as a zero-filled
        # [B, S, D] tensor autograd would write first (2.6 ms per Llama step beside the serve)
        ctx.set_materialize_grads(False)
        return s, y

    @staticmethod
    def backward(ctx, ds, dy):
        s, w, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(s)
        dsum, dw = native().rmsnorm_bwd(dy.contiguous(), s, w, rstd,
                                        ds.contiguous() if ds is not None else None)
        return dsum, dsum, dw.to(w.dtype), None


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None):
    D = x.shape[-1]
    ok = _hip(x) and D % 8 == 0 and D <= 4096 and w.is_cuda and w.dtype in (torch.bfloat16, torch.float32)
    if residual is None:
        return _RMSNorm.apply(x, w, eps) if ok else _rms_ref(x, w, eps)
    if ok and _hip(residual):
        return _AddRMSNorm.apply(x, residual, w, eps)
    s = x + residual
    return s, _rms_ref(s, w, eps)


# ------------------------------------------------------------------------------ LayerNorm
class _LNResidual(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, o, gamma, beta, eps, p):
        seed = _seed()
        s, y, mean, rstd = native().layernorm_fwd(x.contiguous(), o.contiguous(), gamma.contiguous(),
                                                  beta.contiguous(), float(eps), float(p), seed)
        ctx.save_for_backward(s, gamma, mean, rstd)
        ctx.p, ctx.seed = float(p), seed
        return y

    @staticmethod
    def backward(ctx, dy):
        s, gamma, mean, rstd = ctx.saved_tensors
        dx, do, dg, db = native().layernorm_bwd(dy.contiguous(), s, gamma, mean, rstd, ctx.p, ctx.seed)
        return dx, do, dg.to(gamma.dtype), db.to(gamma.dtype), None, None


def layer_norm_residual(x: torch.Tensor, o: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float,
                        p: float = 0.0, training: bool = True) -> torch.Tensor:
    """LayerNorm(x + dropout_p(o)) -- the BERT sublayer epilogue in one pass each way."""
    p = float(p) if training else 0.0
    D = x.shape[-1]
    if _hip(x, o) and D % 8 == 0 and D <= 4096 and gamma.dtype in (torch.bfloat16, torch.float32):
        return _LNResidual.apply(x, o, gamma, beta, eps, p)
    return F.layer_norm(x + F.dropout(o, p, training), (D,), gamma, beta, eps)


# ------------------------------------------------------------------------------ SwiGLU
class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        return native().swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dh):
        (gu,) = ctx.saved_tensors
        return native().swiglu_bwd(dh.contiguous(), gu)


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    if _hip(gu) and gu.shape[-1] % 16 == 0:
        return _SwiGLU.apply(gu)
    g, u = gu.chunk(2, dim=-1)
    return F.silu(g) * u


# ------------------------------------------------------------------------------ RoPE
def rope_table(seq: int, hd: int, theta: float, device) -> torch.Tensor:
    """[S, hd/2, 2] fp32 (cos, sin) -- rotate-halves convention (Llama / HF)."""
    inv = 1.0 / (theta ** (torch.arange(0, hd, 2, device=device).float() / hd))
    f = torch.outer(torch.arange(seq, device=device).float(), inv)
    return torch.stack([torch.cos(f), torch.sin(f)], dim=-1).contiguous()


def _rope_ref(x, cs):
    d = x.shape[-1]
    c, s = cs[..., 0][None, None].to(x.dtype), cs[..., 1][None, None].to(x.dtype)
    x1, x2 = x[..., : d // 2], x[..., d // 2:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


class _RopeSplit(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cs, H, KV):
        q, k, v = native().rope_split_fwd(qkv.contiguous(), cs, int(H), int(KV))
        ctx.save_for_backward(cs)
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        (cs,) = ctx.saved_tensors
        dq = dq if dq is not None else None
        return native().rope_split_bwd(dq.contiguous(), dk.contiguous(), dv.contiguous(), cs), None, None, None


def rope_split(qkv: torch.Tensor, cs: torch.Tensor, H: int, KV: int):
    """qkv [B, S, H + 2 KV, hd] -> q [B, H, S, hd], k/v [B, KV, S, hd] with RoPE on q and k."""
    if _hip(qkv) and qkv.shape[-1] % 16 == 0:
        return _RopeSplit.apply(qkv, cs, H, KV)
    x = qkv.transpose(1, 2)
    q, k, v = x.split([H, KV, KV], dim=1)
    return _rope_ref(q, cs), _rope_ref(k, cs), v


# ------------------------------------------------------------------------------ attention
def attention_qkv_ok(qkv: torch.Tensor, heads: int, mask) -> bool:
    """The fused kernel's domain: GPU bf16, head dim 64, S a multiple of 32 up to 128, no mask."""
    return (mask is None and _hip(qkv) and qkv.dim() == 3 and qkv.shape[2] == 3 * heads * 64
            and qkv.shape[1] % 32 == 0 and 0 < qkv.shape[1] <= 128
            and knobs.enabled("fused_attn"))


class _FusedAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, heads, p):
        qkv = qkv.contiguous()
        seed = _seed() if p > 0 else 0
        out, lse = native().attn_fwd(qkv, heads, float(p), seed)
        ctx.save_for_backward(qkv, out, lse)
        ctx.heads, ctx.p, ctx.seed = heads, float(p), seed
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        return native().attn_bwd(qkv, out, dout.contiguous(), lse, ctx.heads, ctx.p, ctx.seed), None, None


def attention_qkv(qkv: torch.Tensor, heads: int, p: float = 0.0, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Multi-head self-attention over the fused projection ``qkv`` [B, S, 3 * H * D] (q | k | v,
    heads inner) -> [B, S, H * D], dropout ``p`` on the probabilities.  On the fused kernel the
    heads are never split into separate q / k / v tensors and the output is already merged."""
    if attention_qkv_ok(qkv, heads, mask):
        return _FusedAttention.apply(qkv, heads, float(p))
    b, s, _ = qkv.shape
    q, k, v = qkv.view(b, s, 3, heads, -1).permute(2, 0, 3, 1, 4)
    a = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, dropout_p=p)
    return a.transpose(1, 2).reshape(b, s, -1)


# ------------------------------------------------------------------------------ causal GQA flash attention
def flash_ok(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> bool:
    """The in-house causal GQA flash kernels are the default for head dim 128 (PS_AMD_DISABLE=flash_attn
    falls back to SDPA): on the Llama-3-8B shape they beat SDPA's library kernels forward and
    backward (profiles/r3_flash_v3_probe.jsonl) and end to end (profiles/r3_llama_flash_vs_sdpa.jsonl)."""
    return (_hip(q, k, v) and q.dim() == 4 and q.shape[3] == 128 and k.shape == v.shape and q.shape[2] % 128 == 0
            and q.shape[1] % k.shape[1] == 0 and knobs.enabled("flash_attn"))


class _FlashCausal(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        out, lse = native().fa_fwd(q, k, v)
        ctx.save_for_backward(q, k, v, out, lse)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        return tuple(native().fa_bwd(q, k, v, out, dout.contiguous(), lse))


def attention_causal_gqa(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """Causal attention with grouped KV heads: q [B, H, S, D], k / v [B, KV, S, D] -> [B, S, H * D]
    (heads merged, the output projection's input layout)."""
    if flash_ok(q, k, v):
        return _FlashCausal.apply(q, k, v)
    b, _, s, _ = q.shape
    a = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
    return a.transpose(1, 2).reshape(b, s, -1)


# ------------------------------------------------------------------------------ fused LM-head cross-entropy
class _FusedXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, labels, ignore):
        lse, rows = native().xent_fwd(x, labels, int(ignore))
        # the kernels' rule for a scored row (xent.hip: y != ignore and 0 <= y < V): an out-of-range
        # label scores 0 and is not in the mean's denominator either (F.cross_entropy raises on
        # one; checking here would cost a host sync per step)
        V = x.shape[1]
        count = ((labels != ignore) & (labels >= 0) & (labels < V)).sum().float().reshape(1)
        ctx.save_for_backward(x, labels, lse, count)
        ctx.ignore = int(ignore)
        return (rows.sum() / count.clamp(min=1.0)).reshape(())

    @staticmethod
    def backward(ctx, go):
        x, labels, lse, count = ctx.saved_tensors
        dx = native().xent_bwd(x, labels, lse, go.float().reshape(1).contiguous(), count, ctx.ignore)
        return dx, None, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Mean softmax cross-entropy of ``logits`` [..., V] against ``labels`` [...] (ignore_index rows
    excluded), as F.cross_entropy.  GPU bf16 logits take the fused HIP kernels (csrc/kernels/xent.hip):
    the forward reads the logits once (per-row log-sum-exp), the backward reads them once and writes
    the bf16 gradient -- no fp32 copy of the vocab-sized activations.  PS_AMD_DISABLE=fused_xent falls back."""
    V = logits.shape[-1]
    if _hip(logits) and logits.dtype == torch.bfloat16 and knobs.enabled("fused_xent"):
        x = logits.reshape(-1, V)
        x = x if x.is_contiguous() else x.contiguous()
        return _FusedXent.apply(x, labels.reshape(-1).long().contiguous(), int(ignore_index))
    return F.cross_entropy(logits.float().reshape(-1, V), labels.reshape(-1), ignore_index=ignore_index)
