"""Causal GQA flash attention (csrc/kernels/flash_attn.hip) vs a plain-torch fp32 reference (B * KV a
multiple of 8 takes the XCD-aware block order, other shapes the plain one):
output, log-sum-exp, dq / dk / dv (the GQA dk / dv sum over the q heads of each KV group)."""
import pytest
import torch

from ps_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def _ref(q, k, v):
    B, H, S, D = q.shape
    G = H // k.shape[1]
    kk, vv = k.repeat_interleave(G, 1), v.repeat_interleave(G, 1)
    sc = q @ kk.transpose(-1, -2) / D ** 0.5
    mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
    sc = sc.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(sc, -1)
    o = torch.softmax(sc, -1) @ vv
    return o.transpose(1, 2).reshape(B, S, H * D), lse


@pytest.mark.parametrize("B,H,KV,S", [(1, 4, 1, 128), (2, 4, 2, 256), (1, 8, 2, 384), (1, 8, 2, 2048), (1, 4, 1, 4096), (1, 16, 8, 256), (2, 8, 8, 512)])
def test_flash_causal_gqa(B, H, KV, S):
    g = torch.Generator().manual_seed(B * 100 + H * 10 + S)
    q = torch.randn(B, H, S, 128, generator=g).bfloat16().to(DEV)
    k = torch.randn(B, KV, S, 128, generator=g).bfloat16().to(DEV)
    v = torch.randn(B, KV, S, 128, generator=g).bfloat16().to(DEV)
    dout = torch.randn(B, S, H * 128, generator=g).bfloat16().to(DEV)
    out, lse = native().fa_fwd(q, k, v)
    qf, kf, vf = (t.float().requires_grad_() for t in (q, k, v))
    ro, rl = _ref(qf, kf, vf)
    assert _rel(out, ro) < 1e-2
    torch.testing.assert_close(lse, rl, rtol=1e-3, atol=2e-3)
    ro.backward(dout.float())
    dq, dk, dv = native().fa_bwd(q, k, v, out, dout, lse)
    assert _rel(dq, qf.grad) < 2e-2
    assert _rel(dk, kf.grad) < 2e-2
    assert _rel(dv, vf.grad) < 2e-2


def test_llama_block_flash_matches_sdpa(monkeypatch):
    from ps_amd.models.transformer import LlamaBlock, LlamaConfig
    from ps_amd.ops.transformer import rope_table

    torch.manual_seed(0)
    c = LlamaConfig(hidden=512, layers=1, heads=4, kv_heads=2, ffn=1024, vocab=128)
    blk = LlamaBlock(c).to(DEV).bfloat16()
    x = torch.randn(2, 256, 512, device=DEV).bfloat16()
    wl = torch.randn(2, 256, 512, device=DEV)
    cs = rope_table(256, 128, c.rope_theta, x.device)
    outs = []
    for flag in ("1", "0"):  # flash kernel (the default) vs SDPA
        monkeypatch.setenv("PS_AMD_DISABLE", "" if flag == "1" else "flash_attn")
        blk.zero_grad()
        xi = x.clone().requires_grad_()
        y, r = blk(xi, None, cs)
        ((y.float() + r.float()) * wl).sum().backward()
        outs.append((r.detach(), xi.grad.clone(), blk.wqkv.weight.grad.clone()))
    for a, b in zip(outs[0], outs[1]):
        assert _rel(a, b) < 2e-2
