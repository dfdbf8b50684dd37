"""Fused transformer HIP kernels (csrc/kernels/transformer.hip) vs plain torch fp32 references."""
import pytest
import torch
import torch.nn.functional as F

from ps_amd.ops import transformer as T

pytestmark = pytest.mark.gpu


def _close(a, b, tol=2e-2):
    a, b = a.float(), b.float()
    err = (a - b).norm() / b.norm().clamp_min(1e-12)
    assert err < tol, float(err)


@pytest.mark.parametrize("R,D", [(300, 4096), (64, 768), (17, 104)])
@pytest.mark.parametrize("wdtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("residual", [False, True])
def test_rmsnorm_fwd_bwd(R, D, wdtype, residual):
    torch.manual_seed(0)
    x = torch.randn(R, D, device="cuda").bfloat16().requires_grad_(True)
    r = torch.randn(R, D, device="cuda").bfloat16().requires_grad_(True)
    w = (1 + 0.1 * torch.randn(D, device="cuda")).to(wdtype).requires_grad_(True)
    xr, rr, wr = (t.detach().float().requires_grad_(True) for t in (x, r, w))
    if residual:
        s, y = T.rms_norm(x, w, 1e-5, residual=r)
        sr = xr + rr
        yr = sr * torch.rsqrt(sr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
        _close(s, sr, 1e-2)
        ds = torch.randn_like(sr)
    else:
        y = T.rms_norm(x, w, 1e-5)
        yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    _close(y, yr)
    dy = torch.randn_like(yr)
    if residual:
        torch.autograd.backward([s, y], [ds.bfloat16(), dy.bfloat16()])
        torch.autograd.backward([sr, yr], [ds.bfloat16().float(), dy.bfloat16().float()])
        _close(r.grad, rr.grad)
    else:
        y.backward(dy.bfloat16())
        yr.backward(dy.bfloat16().float())
    _close(x.grad, xr.grad)
    _close(w.grad, wr.grad)


@pytest.mark.parametrize("used", ["y", "s"])
def test_rmsnorm_residual_one_output_used(used):
    """Only one of (stream s, normed y) feeds the loss (the final norm drops s): autograd hands the
    backward None for the other (no zero-filled tensor) and the gradients match the reference."""
    torch.manual_seed(3)
    R, D = 96, 1024
    x = torch.randn(R, D, device="cuda").bfloat16().requires_grad_(True)
    r = torch.randn(R, D, device="cuda").bfloat16().requires_grad_(True)
    w = (1 + 0.1 * torch.randn(D, device="cuda")).requires_grad_(True)
    xr, rr, wr = (t.detach().float().requires_grad_(True) for t in (x, r, w))
    s, y = T.rms_norm(x, w, 1e-5, residual=r)
    sr = xr + rr
    yr = sr * torch.rsqrt(sr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    g = torch.randn(R, D, device="cuda").bfloat16()
    (y if used == "y" else s).backward(g)
    (yr if used == "y" else sr).backward(g.float())
    _close(x.grad, xr.grad)
    _close(r.grad, rr.grad)
    if used == "y":
        _close(w.grad, wr.grad)


@pytest.mark.parametrize("R,D", [(512, 768), (33, 1024), (8, 64)])
@pytest.mark.parametrize("wdtype", [torch.float32, torch.bfloat16])
def test_layernorm_residual_no_dropout(R, D, wdtype):
    torch.manual_seed(1)
    x = torch.randn(R, D, device="cuda").bfloat16().requires_grad_(True)
    o = torch.randn(R, D, device="cuda").bfloat16().requires_grad_(True)
    g = (1 + 0.1 * torch.randn(D, device="cuda")).to(wdtype).requires_grad_(True)
    b = (0.1 * torch.randn(D, device="cuda")).to(wdtype).requires_grad_(True)
    y = T.layer_norm_residual(x, o, g, b, 1e-12, 0.0, True)
    xr, orr, gr, br = (t.detach().float().requires_grad_(True) for t in (x, o, g, b))
    yr = F.layer_norm(xr + orr, (D,), gr, br, 1e-12)
    _close(y, yr)
    dy = torch.randn_like(yr).bfloat16()
    y.backward(dy)
    yr.backward(dy.float())
    for a, c in ((x, xr), (o, orr), (g, gr), (b, br)):
        _close(a.grad, c.grad)


def test_layernorm_residual_dropout_mask_consistent():
    """The backward regenerates exactly the forward's dropout mask (Philox, never stored)."""
    torch.manual_seed(2)
    R, D, p = 256, 768, 0.1
    x = torch.zeros(R, D, device="cuda").bfloat16().requires_grad_(True)
    o = torch.ones(R, D, device="cuda").bfloat16().requires_grad_(True)
    g = torch.ones(D, device="cuda")
    b = torch.zeros(D, device="cuda")
    y = T.layer_norm_residual(x, o, g, b, 1e-5, p, True)
    kept_fwd = y > y.min(dim=1, keepdim=True).values  # s = mask * 1/(1-p): LN is monotone per row
    dy = torch.randn(R, D, device="cuda").bfloat16()
    y.backward(dy)
    kept_bwd = o.grad != 0
    assert torch.equal(kept_fwd, kept_bwd)
    frac = 1 - kept_bwd.float().mean().item()
    assert abs(frac - p) < 0.01
    # kept elements: d(o) = d(s) / (1 - p) and d(x) = d(s)
    torch.testing.assert_close(o.grad[kept_bwd].float(), x.grad[kept_bwd].float() / (1 - p), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("R,F", [(100, 1024), (7, 14336)])
def test_swiglu_fwd_bwd(R, F):
    torch.manual_seed(3)
    gu = torch.randn(R, 2 * F, device="cuda").bfloat16().requires_grad_(True)
    gr = gu.detach().float().requires_grad_(True)
    h = T.swiglu(gu)
    a, u = gr.chunk(2, dim=-1)
    hr = F_silu(a) * u
    _close(h, hr)
    dh = torch.randn_like(hr).bfloat16()
    h.backward(dh)
    hr.backward(dh.float())
    _close(gu.grad, gr.grad)


def test_swiglu_saturated_inputs_stay_finite():
    """the fast sigmoid (bare exp2 + reciprocal) at |g| up to 120: exp overflows to inf and the
    reciprocal to 0 -- silu and its gradient must still match the fp32 reference, no NaN."""
    F = 1024
    g = torch.linspace(-120, 120, 2 * F, device="cuda").reshape(2, F)
    gu = torch.cat([g, torch.ones_like(g)], dim=-1).bfloat16().requires_grad_(True)
    gr = gu.detach().float().requires_grad_(True)
    h = T.swiglu(gu)
    a, u = gr.chunk(2, dim=-1)
    hr = F_silu(a) * u
    assert torch.isfinite(h.float()).all()
    _close(h, hr)
    dh = torch.ones_like(hr).bfloat16()
    h.backward(dh)
    hr.backward(dh.float())
    assert torch.isfinite(gu.grad.float()).all()
    _close(gu.grad, gr.grad)


def F_silu(t):
    return t * torch.sigmoid(t)


@pytest.mark.parametrize("B,S,H,KV,hd", [(1, 64, 8, 2, 128), (2, 33, 4, 4, 64)])
def test_rope_split_fwd_bwd(B, S, H, KV, hd):
    torch.manual_seed(4)
    qkv = torch.randn(B, S, H + 2 * KV, hd, device="cuda").bfloat16().requires_grad_(True)
    cs = T.rope_table(S, hd, 500000.0, "cuda")
    q, k, v = T.rope_split(qkv, cs, H, KV)
    qr_in = qkv.detach().float().requires_grad_(True)
    x = qr_in.transpose(1, 2)
    qr, kr, vr = x[:, :H], x[:, H:H + KV], x[:, H + KV:]
    qr, kr = T._rope_ref(qr, cs), T._rope_ref(kr, cs)
    for a, c in ((q, qr), (k, kr), (v, vr)):
        assert a.shape == c.shape and a.is_contiguous()
        _close(a, c, 1e-2)
    gq, gk, gv = (torch.randn_like(t).bfloat16() for t in (qr, kr, vr))
    torch.autograd.backward([q, k, v], [gq, gk, gv])
    torch.autograd.backward([qr, kr, vr], [gq.float(), gk.float(), gv.float()])
    _close(qkv.grad, qr_in.grad, 1e-2)
