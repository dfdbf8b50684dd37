"""Fused short-sequence attention (csrc/kernels/attention.hip) vs a plain-torch fp32 reference
of the same op: forward output, log-sum-exp and the dq / dk / dv gradient, with and without the
attention-probability dropout (the reference applies the kernel's own keep mask, fetched with
attn_dropout_mask for the same seed)."""
import pytest
import torch

from ps_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(qkv, heads, keep=None, p=0.0):
    b, s, _ = qkv.shape
    q, k, v = qkv.float().view(b, s, 3, heads, 64).permute(2, 0, 3, 1, 4)
    sc = q @ k.transpose(-1, -2) * 0.125
    lse = torch.logsumexp(sc, -1)
    pr = torch.softmax(sc, -1)
    if keep is not None:
        pr = pr * keep.view(b, heads, s, s).float() / (1 - p)
    o = (pr @ v).transpose(1, 2).reshape(b, s, heads * 64)
    return o, lse


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("B,S,H", [(3, 32, 2), (2, 64, 3), (2, 96, 2), (2, 128, 12)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_fused_attention_fwd_bwd(B, S, H, p):
    g = torch.Generator(device="cpu").manual_seed(S * 7 + H + int(p * 10))
    qkv = (torch.randn(B, S, 3 * H * 64, generator=g) * 0.8).to(DEV).bfloat16()
    dout = torch.randn(B, S, H * 64, generator=g).to(DEV).bfloat16()
    seed = 12345 + S
    out, lse = native().attn_fwd(qkv, H, p, seed)
    keep = native().attn_dropout_mask(qkv, B * H, S, p, seed) if p > 0 else None
    if keep is not None:
        assert abs(keep.float().mean().item() - (1 - p)) < 0.01
    x = qkv.float().requires_grad_()
    ro, rl = _ref(x, H, keep, p)
    assert _rel(out, ro) < 1e-2
    torch.testing.assert_close(lse, rl, rtol=1e-3, atol=2e-3)
    ro.backward(dout.float())
    dqkv = native().attn_bwd(qkv, out, dout, lse, H, p, seed)
    ref = x.grad.view(B, S, 3, H, 64)
    got = dqkv.view(B, S, 3, H, 64)
    for i, name in enumerate("qkv"):
        assert _rel(got[:, :, i], ref[:, :, i]) < 2e-2, name


def test_bert_layer_fused_attention_matches_sdpa(monkeypatch):
    """BertLayer (p = 0) with the fused kernel vs the SDPA path: output and parameter grads."""
    from ps_amd.models.transformer import BertConfig, BertLayer

    torch.manual_seed(0)
    c = BertConfig(hidden=256, heads=4, ffn=512, dropout=0.0)
    layer = BertLayer(c).to(DEV).bfloat16()
    x = torch.randn(4, 128, 256, device=DEV).bfloat16()
    wl = torch.randn(4, 128, 256, device=DEV)  # (mean(y^2) after a LayerNorm has zero gradient)
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("PS_AMD_DISABLE", "" if flag == "1" else "fused_attn")
        layer.zero_grad()
        xi = x.clone().requires_grad_()
        y = layer(xi)
        (y.float() * wl).sum().backward()
        outs.append((y.detach(), xi.grad.clone(), layer.qkv.weight.grad.clone()))
    for a, b in zip(outs[0], outs[1]):
        assert _rel(a, b) < 2e-2


@pytest.mark.parametrize("R,V,ign", [(300, 30522, 7), (64, 1000, 0), (33, 517, 5)])
def test_fused_cross_entropy_matches_fp32(R, V, ign):
    """LM-head cross-entropy on bf16 logits (csrc/kernels/xent.hip) vs F.cross_entropy in fp32:
    loss and gradient, with ignored rows (label -100) and a non-multiple-of-8 vocab."""
    from ps_amd.ops.transformer import cross_entropy

    torch.manual_seed(R + V)
    x = (torch.randn(R, V, device="cuda") * 3).bfloat16()
    lab = torch.randint(0, V, (R,), device="cuda")
    lab[torch.randperm(R, device="cuda")[:ign]] = -100
    xf = x.float().requires_grad_()
    ref = torch.nn.functional.cross_entropy(xf, lab, ignore_index=-100)
    (ref * 0.7).backward()
    xg = x.clone().requires_grad_()
    loss = cross_entropy(xg, lab)
    (loss * 0.7).backward()
    torch.testing.assert_close(loss.float(), ref.detach(), rtol=1e-4, atol=1e-4)
    rel = ((xg.grad.float() - xf.grad).norm() / xf.grad.norm()).item()
    assert rel < 1e-2, rel
    assert bool((xg.grad[lab == -100] == 0).all())


def test_fused_cross_entropy_out_of_range_labels_are_not_counted():
    """a label outside [0, V) that is not ignore_index scores 0 in the kernels and is
    left out of the mean's denominator too -- the loss equals F.cross_entropy over the in-range
    rows only, and those rows get zero gradient."""
    from ps_amd.ops.transformer import cross_entropy

    torch.manual_seed(3)
    R, V = 40, 517
    x = (torch.randn(R, V, device="cuda") * 2).bfloat16()
    lab = torch.randint(0, V, (R,), device="cuda")
    lab[:3] = V + 4
    lab[3:5] = -7
    lab[5] = -100
    ok = (lab >= 0) & (lab < V)
    ref = torch.nn.functional.cross_entropy(x.float()[ok], lab[ok])
    xg = x.clone().requires_grad_()
    loss = cross_entropy(xg, lab)
    loss.backward()
    torch.testing.assert_close(loss.float(), ref, rtol=1e-4, atol=1e-4)
    assert bool((xg.grad[~ok] == 0).all())
