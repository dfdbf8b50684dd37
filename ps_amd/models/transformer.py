"""BERT-base and Llama-3 models for the BASELINE.json north-star configs (random init, no
checkpoints, no network).

Compact in-repo definitions (transformers is not needed on the hot path): parameter shapes
and counts match the published architectures -- BERT-base 110M (12 x 768, 12 heads, FFN
3072, vocab 30522), Llama-3-8B 8.03B (32 x 4096, 32 q / 8 kv heads, FFN 14336, vocab
128256, RoPE theta 500000).  BERT attention (S <= 128) runs the fused MFMA kernel of
csrc/kernels/attention.hip, Llama's causal GQA attention the flash kernel of flash_attn.hip;
everything is bf16 on the GPU with fp32 masters on the parameter-server shards.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.checkpoint import checkpoint

from ..ops.dense import SplitKLinear
from ..ops.linear import PsLinear
from ..ops.transformer import (attention_causal_gqa, attention_qkv, cross_entropy, layer_norm_residual, rms_norm, rope_split,
                              rope_table, swiglu)


# ------------------------------------------------------------------------------------ BERT
@dataclass
class BertConfig:
    vocab: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    max_pos: int = 512
    type_vocab: int = 2
    eps: float = 1e-12
    dropout: float = 0.1


class BertLayer(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.c = c
        # split-K weight gradients (ops/dense.py SplitKLinear): 32K tokens into small dW
        self.qkv = SplitKLinear(c.hidden, 3 * c.hidden)
        self.proj = SplitKLinear(c.hidden, c.hidden)
        self.ln1 = nn.LayerNorm(c.hidden, eps=c.eps)
        self.fc1 = SplitKLinear(c.hidden, c.ffn)
        self.fc2 = SplitKLinear(c.ffn, c.hidden)
        self.ln2 = nn.LayerNorm(c.hidden, eps=c.eps)

    def forward(self, x, mask: Optional[torch.Tensor] = None):
        p = self.c.dropout if self.training else 0.0
        # fused MFMA attention over the qkv projection for S <= 128 (ops/transformer.py), SDPA else
        # fork: x's residual gradient is added inside the qkv / fc1 data-gradient GEMM (ops/dense.py)
        qkv, xr = self.qkv.fork(x)
        a = attention_qkv(qkv, self.c.heads, p, mask)
        # post-LN epilogues: LN(x + dropout(sublayer)) as one fused HIP pass each way
        x = layer_norm_residual(xr, self.proj(a), self.ln1.weight, self.ln1.bias, self.c.eps, p, self.training)
        h, xr = self.fc1.fork(x)
        f = self.fc2(F.gelu(h))
        return layer_norm_residual(xr, f, self.ln2.weight, self.ln2.bias, self.c.eps, p, self.training)


class BertForMLM(nn.Module):
    """BERT-base with the masked-LM head (decoder tied to the word embeddings)."""

    def __init__(self, c: BertConfig = BertConfig()):
        super().__init__()
        self.c = c
        self.word = nn.Embedding(c.vocab, c.hidden)
        self.pos = nn.Embedding(c.max_pos, c.hidden)
        self.tok_type = nn.Embedding(c.type_vocab, c.hidden)
        self.ln = nn.LayerNorm(c.hidden, eps=c.eps)
        self.layers = nn.ModuleList(BertLayer(c) for _ in range(c.layers))
        self.head_dense = nn.Linear(c.hidden, c.hidden)
        self.head_ln = nn.LayerNorm(c.hidden, eps=c.eps)
        self.head_bias = nn.Parameter(torch.zeros(c.vocab))
        self.apply(self._init)

    @staticmethod
    def _init(m):
        if isinstance(m, (nn.Linear, nn.Embedding)):
            nn.init.normal_(m.weight, std=0.02)
        if isinstance(m, nn.Linear) and m.bias is not None:
            nn.init.zeros_(m.bias)

    def forward(self, ids, labels=None, positions=None):
        """``positions`` [B, P] (the masked-LM positions of the original BERT pretraining input
        format, ``masked_lm_positions``): the LM head runs only on those B*P rows -- the vocab
        projection and its softmax are 1/(S/P) of the dense-head cost.  Without positions the
        head runs on every token (labels -100 are ignored)."""
        b, s = ids.shape
        pos = torch.arange(s, device=ids.device)
        x = self.word(ids) + self.pos(pos)[None] + self.tok_type.weight[0]
        x = F.dropout(self.ln(x), self.c.dropout, self.training)
        for layer in self.layers:
            x = layer(x)
        if positions is not None:
            flat = (positions + torch.arange(b, device=ids.device)[:, None] * s).reshape(-1)
            x = x.reshape(b * s, -1).index_select(0, flat)
            if labels is not None:
                labels = labels.reshape(-1).index_select(0, flat)
        h = self.head_ln(F.gelu(self.head_dense(x)))
        logits = h @ self.word.weight.t() + self.head_bias
        if labels is None:
            return logits
        return cross_entropy(logits.view(-1, self.c.vocab), labels.reshape(-1), ignore_index=-100)


def mlm_batch(batch: int, seq: int, vocab: int = 30522, mask_prob: float = 0.15, seed: int = 0, device=None,
              with_positions: bool = False):
    """Synthetic MLM batch in the BERT pretraining format: exactly round(mask_prob * seq)
    masked positions per sequence (create_pretraining_data's num_to_predict), replaced by
    [MASK]; labels -100 elsewhere.  ``with_positions`` also returns masked_lm_positions [B, P]."""
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(min(1000, vocab // 2), vocab, (batch, seq), generator=g)
    npred = max(1, int(round(mask_prob * seq)))
    positions = torch.rand(batch, seq, generator=g).argsort(dim=1)[:, :npred].sort(dim=1).values
    labels = torch.full_like(ids, -100)
    labels.scatter_(1, positions, ids.gather(1, positions))
    ids = ids.scatter(1, positions, 103)  # [MASK]
    if device is not None:
        ids, labels, positions = ids.to(device), labels.to(device), positions.to(device)
    return (ids, labels, positions) if with_positions else (ids, labels)


# ----------------------------------------------------------------------------------- Llama
@dataclass
class LlamaConfig:
    vocab: int = 128256
    hidden: int = 4096
    layers: int = 32
    heads: int = 32
    kv_heads: int = 8
    ffn: int = 14336
    rope_theta: float = 500000.0
    eps: float = 1e-5
    max_seq: int = 8192

    @staticmethod
    def llama3_8b() -> "LlamaConfig":
        return LlamaConfig()

    @staticmethod
    def tiny() -> "LlamaConfig":
        return LlamaConfig(vocab=512, hidden=64, layers=2, heads=4, kv_heads=2, ffn=128, max_seq=128)


class RMSNorm(nn.Module):
    def __init__(self, d, eps):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        self.eps = eps

    def forward(self, x):
        return rms_norm(x, self.weight, self.eps)  # fused HIP kernel on GPU bf16 (ops/transformer.py)


class LlamaBlock(nn.Module):
    """Pre-norm decoder block.  Q/K/V and gate/up projections are single fused GEMMs
    (``wqkv`` [(H + 2 KV) * hd, D], ``w13`` [2 F, D] -- same parameter count as separate
    matrices, one hipBLASLt launch each); attention is the causal GQA flash kernel
    (csrc/kernels/flash_attn.hip; no K/V replication, output already head-merged)."""

    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.c = c
        hd = c.hidden // c.heads
        self.attn_norm = RMSNorm(c.hidden, c.eps)
        # PsLinear: the weight gradient lands straight in the PS gradient bucket (ops/linear.py)
        self.wqkv = PsLinear(c.hidden, (c.heads + 2 * c.kv_heads) * hd, bias=False)
        self.wo = PsLinear(c.heads * hd, c.hidden, bias=False)
        self.mlp_norm = RMSNorm(c.hidden, c.eps)
        self.w13 = PsLinear(c.hidden, 2 * c.ffn, bias=False)
        self.w2 = PsLinear(c.ffn, c.hidden, bias=False)

    def forward(self, x, r, cs):
        """Residual stream = x + r (r: the previous block's pending MLP output, None for the
        first block) -- the add is fused into this block's first RMSNorm, and this block's
        MLP output is returned pending for the next one."""
        b, s, _ = x.shape
        c = self.c
        hd = c.hidden // c.heads
        if r is None:
            h = self.attn_norm(x)
        else:
            x, h = rms_norm(x, self.attn_norm.weight, c.eps, residual=r)
        qkv = self.wqkv(h).view(b, s, c.heads + 2 * c.kv_heads, hd)
        q, k, v = rope_split(qkv, cs, c.heads, c.kv_heads)  # RoPE + split + transpose, one pass
        o = self.wo(attention_causal_gqa(q, k, v))  # flash kernel (heads merged) or SDPA
        x, h = rms_norm(x, self.mlp_norm.weight, c.eps, residual=o)
        return x, self.w2(swiglu(self.w13(h)))


class LlamaForCausalLM(nn.Module):
    def __init__(self, c: LlamaConfig = LlamaConfig(), checkpointing: bool = False):
        super().__init__()
        self.c = c
        self.checkpointing = checkpointing
        self.embed = nn.Embedding(c.vocab, c.hidden)
        self.layers = nn.ModuleList(LlamaBlock(c) for _ in range(c.layers))
        self.norm = RMSNorm(c.hidden, c.eps)
        self.lm_head = PsLinear(c.hidden, c.vocab, bias=False)
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, std=0.02)

    def forward(self, ids, labels=None):
        s = ids.shape[1]
        cs = rope_table(s, self.c.hidden // self.c.heads, self.c.rope_theta, ids.device)
        x, r = self.embed(ids), None
        for layer in self.layers:
            if self.checkpointing and self.training:
                x, r = checkpoint(layer, x, r, cs, use_reentrant=False)
            else:
                x, r = layer(x, r, cs)
        _, h = rms_norm(x, self.norm.weight, self.c.eps, residual=r)
        logits = self.lm_head(h)
        if labels is None:
            return logits
        # next-token targets; the last position has none (ignored) -- no sliced copy of the logits
        tgt = torch.cat([labels[:, 1:], torch.full_like(labels[:, :1], -100)], dim=1)
        return cross_entropy(logits, tgt, ignore_index=-100)


def param_count(m: nn.Module) -> int:
    seen, n = set(), 0
    for p in m.parameters():
        if id(p) not in seen:
            seen.add(id(p))
            n += p.numel()
    return n
