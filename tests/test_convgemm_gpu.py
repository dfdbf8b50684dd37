"""Implicit-GEMM convolution kernels (csrc/kernels/convgemm.hip) vs plain-torch fp32 references
of the same op, and the fused ResNet bottleneck vs the module-by-module path.

Pixel counts are not multiples of the 128-row tile, both 64- and 128-channel tile widths are
used, stride-2 gathers run on odd map sizes, and the 3x3 geometry (padding taps) is checked
against F.conv2d."""
import copy

import pytest
import torch
import torch.nn.functional as F

from ps_amd.ops import native
from ps_amd.ops.convgemm import geo

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bf(t):
    return t.bfloat16().to(DEV).contiguous()


def _close(out, ref, tol=1e-2, amax=0.05):
    out = out.float().cpu()
    ref = ref.float().cpu()
    err = ((out - ref).norm() / ref.norm().clamp_min(1e-12)).item()
    assert err < tol, f"relative error {err:.3g}"
    assert (out - ref).abs().max().item() <= amax * ref.abs().max().item() + 1e-3


def _close_flips(out, ref, tol, amax, frac=5e-4):
    """_close with the max-abs bound on all but a fraction ``frac`` of the elements."""
    out = out.float().cpu()
    ref = ref.float().cpu()
    err = ((out - ref).norm() / ref.norm().clamp_min(1e-12)).item()
    assert err < tol, f"relative error {err:.3g}"
    bad = ((out - ref).abs() > amax * ref.abs().max() + 1e-3).float().mean().item()
    assert bad <= frac, f"{bad:.2e} of the elements off by more than {amax} x max"


def _gen(seed):
    return torch.Generator().manual_seed(seed)


def _coef(k, g):
    return torch.cat([torch.rand(k, generator=g) + 0.5, torch.randn(k, generator=g) * 0.5])


def _bn_relu(a, coef):
    k = a.shape[-1]
    return torch.relu(a * coef[:k] + coef[k:]).bfloat16().float()


def _rnd(*shape, g, scale=1.0):
    return (torch.randn(*shape, generator=g) * scale).bfloat16().float()


SHAPES = [(300, 64, 64), (1000, 128, 256), (128, 256, 128), (4099, 512, 64), (517, 1024, 128)]


@pytest.mark.parametrize("M,K,N", SHAPES)
@pytest.mark.parametrize("pro", [False, True])
def test_conv1x1_forward_with_bn_statistics(M, K, N, pro):
    g = _gen(M * 7 + K + N)
    a, b = _rnd(M, K, g=g), _rnd(N, K, g=g, scale=K ** -0.5)
    coef = _coef(K, g) if pro else None
    ref = (_bn_relu(a, coef) if pro else a) @ b.t()
    kshift = torch.randn(N, generator=g) * 0.1
    c, part = native().conv_gemm(_bf(a), _bf(b), [M, 1, M, 1, 1, 1, 0], coef.to(DEV) if pro else None, 1, None,
                                 kshift.to(DEV))
    _close(c, ref)
    cb = c.float().cpu() - kshift
    torch.testing.assert_close(part[0].sum(0).cpu(), cb.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part[1].sum(0).cpu(), (cb * cb).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("M,K,N", SHAPES[:3])
def test_conv1x1_residual_epilogue(M, K, N):
    g = _gen(M + 1)
    a, b, r = _rnd(M, K, g=g), _rnd(N, K, g=g, scale=K ** -0.5), _rnd(M, N, g=g)
    c, _ = native().conv_gemm(_bf(a), _bf(b), [M, 1, M, 1, 1, 1, 0], None, 2, _bf(r))
    _close(c, a @ b.t() + r)
    # epilogue 5: residual masked by ReLU bits
    keep = torch.rand(M, N, generator=g) > 0.5
    bits = (keep.view(-1, 8).int() << torch.arange(8)).sum(1).to(torch.uint8)
    c5, _ = native().conv_gemm(_bf(a), _bf(b), [M, 1, M, 1, 1, 1, 0], None, 5, _bf(r), bits=bits.to(DEV))
    _close(c5, a @ b.t() + r * keep)


@pytest.mark.parametrize("M,K,N", SHAPES[:4])
def test_conv1x1_bn_backward_epilogue(M, K, N):
    g = _gen(M + 2)
    a, b, z = _rnd(M, K, g=g), _rnd(N, K, g=g, scale=K ** -0.5), _rnd(M, N, g=g)
    mc = _coef(N, g)
    mean, invstd = torch.randn(N, generator=g) * 0.1, torch.rand(N, generator=g) + 0.5
    c, part = native().conv_gemm(_bf(a), _bf(b), [M, 1, M, 1, 1, 1, 0], None, 3, _bf(z), None, mc.to(DEV),
                                 mean.to(DEV), invstd.to(DEV))
    mask = (z * mc[:N] + mc[N:]) > 0
    _close(c, (a @ b.t()) * mask)
    cg = c.float().cpu()
    torch.testing.assert_close(part[0].sum(0).cpu(), cg.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part[1].sum(0).cpu(), (cg * ((z - mean) * invstd)).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("M,K,N", [(300, 256, 64), (1000, 512, 128), (4099, 256, 64), (517, 1024, 256),
                                   (333, 2048, 512)])
def test_bn_backward_prologue_matches_apply_then_gemm(M, K, N):
    """conv_gemm(a=d, a2=z, bwd=coef) == bn_bwd_partials(d, z) then conv_gemm on its output: the
    data gradient of the previous BN computed while staging A (and stored as a third output),
    then the GEMM with epilogue 3 (ReLU mask + the next BN's backward sums)."""
    g = _gen(M + K)
    d, z = _rnd(M, K, g=g), _rnd(M, K, g=g)
    gamma, mean, invstd = torch.rand(K, generator=g) + 0.5, torch.randn(K, generator=g) * 0.1, torch.rand(K) + 0.5
    xhat = (z - mean) * invstd
    part = torch.stack([d.sum(0, keepdim=True), (d * xhat).sum(0, keepdim=True)]).to(DEV).contiguous()
    b, z2 = _rnd(N, K, g=g, scale=K ** -0.5), _rnd(M, N, g=g)
    mc = _coef(N, g)
    m2, i2 = torch.randn(N, generator=g) * 0.1, torch.rand(N, generator=g) + 0.5
    args = (_bf(b), [M, 1, M, 1, 1, 1, 0], None, 3, _bf(z2), None, mc.to(DEV), m2.to(DEV), i2.to(DEV))
    dz_ref, dg_ref, db_ref = native().bn_bwd_partials(_bf(d), _bf(z), part, gamma.to(DEV), mean.to(DEV), invstd.to(DEV))
    c_ref, p_ref = native().conv_gemm(dz_ref, *args)
    dg, db, coef = native().bn_bwd_coef(part, gamma.to(DEV), mean.to(DEV), invstd.to(DEV), M)
    torch.testing.assert_close(dg, dg_ref)
    torch.testing.assert_close(db, db_ref)
    c, p, dz = native().conv_gemm(_bf(d), *args, a2=_bf(z), bwd=coef)
    # same formula, FMA contraction may differ by one bf16 ulp
    assert (dz != dz_ref).float().mean().item() < 1e-2
    torch.testing.assert_close(dz.float(), dz_ref.float(), rtol=8e-3, atol=1e-3)
    ref_dz = gamma * invstd * (d - d.mean(0) - xhat * (d * xhat).mean(0))
    _close(dz, ref_dz)
    _close(c, c_ref, tol=1e-2, amax=0.05)
    torch.testing.assert_close(p.sum(1), p_ref.sum(1), rtol=2e-3, atol=2e-2)


def test_conv1x1_stride2_gather_and_strided_residual():
    n, h, w, K, N = 3, 13, 11, 128, 64
    g = _gen(3)
    a, b = _rnd(n * h * w, K, g=g), _rnd(N, K, g=g, scale=K ** -0.5)
    gg = geo(h, w, 1, 2)
    oh, ow = gg[2], gg[3]
    c, _ = native().conv_gemm(_bf(a), _bf(b), gg)
    _close(c, a.view(n, h, w, K)[:, ::2, ::2].reshape(-1, K) @ b.t())
    # data gradient of a stride-2 downsample added into the full-resolution map (epilogue 4)
    a2, b2 = _rnd(n * h * w, 64, g=g), _rnd(K, 64, g=g, scale=0.125)
    t = _rnd(n * oh * ow, K, g=g)
    c2, _ = native().conv_gemm(_bf(a2), _bf(b2), geo(h, w), None, 4, _bf(t))
    ref = a2 @ b2.t()
    ref.view(n, h, w, K)[:, ::2, ::2] += t.view(n, oh, ow, K)
    _close(c2, ref)


@pytest.mark.parametrize("n,cin,cout,hw,stride", [(2, 64, 64, 56, 1), (3, 128, 128, 28, 1), (1, 128, 64, 28, 1),
                                                  (2, 64, 192, 56, 1), (2, 128, 128, 56, 2), (1, 64, 128, 56, 2)])
def test_conv3x3_patch_wgrad(n, cin, cout, hw, stride):
    """The 3x3 patch weight-gradient kernel (stride 1, 56- / 28-wide maps, <= 128 channels; the
    image borders are the patch halo) vs fp32 autograd, and vs the im2col kernels it replaces
    (PS_AMD_WGRAD_PATCH_MAX_C is read once per process, so the comparison goes through the
    ResNet-wide shapes here and the generic 14-wide path above)."""
    g = _gen(n + cin + cout + hw)
    x = _rnd(n, hw, hw, cin, g=g)
    oh = hw // stride
    dz = _rnd(n * oh * oh, cout, g=g)
    wv = torch.zeros(cout, cin, 3, 3, requires_grad=True)
    yr = F.conv2d(x.permute(0, 3, 1, 2), wv, None, stride, 1)
    dw_ref = torch.autograd.grad(yr, wv, dz.view(n, oh, oh, cout).permute(0, 3, 1, 2))[0]
    dw = native().conv_wgrad(_bf(dz), _bf(x.reshape(-1, cin)), geo(hw, hw, 3, stride, 1))
    _close(dw, dw_ref.permute(0, 2, 3, 1).reshape(cout, 9 * cin))


@pytest.mark.parametrize("cin,cout,hw,stride", [(64, 64, 14, 1), (128, 128, 9, 2), (64, 128, 7, 1)])
@pytest.mark.parametrize("pro", [False, True])
def test_conv3x3_implicit_gemm_forward_and_wgrad(cin, cout, hw, stride, pro):
    n = 3
    g = _gen(cin + cout + hw + stride)
    x = _rnd(n, hw, hw, cin, g=g)
    wt = _rnd(cout, cin, 3, 3, g=g, scale=(9 * cin) ** -0.5)
    coef = _coef(cin, g) if pro else None
    xin = _bn_relu(x, coef) if pro else x
    ref = F.conv2d(xin.permute(0, 3, 1, 2), wt, None, stride, 1).permute(0, 2, 3, 1).reshape(-1, cout)
    gg = geo(hw, hw, 3, stride, 1)
    wmat = wt.permute(0, 2, 3, 1).reshape(cout, 9 * cin)  # channels_last weight order
    c, _ = native().conv_gemm(_bf(x.reshape(-1, cin)), _bf(wmat), gg, coef.to(DEV) if pro else None)
    _close(c, ref)
    dz = _rnd(n * gg[2] * gg[3], cout, g=g)
    wv = wt.clone().requires_grad_()
    yr = F.conv2d(xin.permute(0, 3, 1, 2), wv, None, stride, 1)
    dw_ref = torch.autograd.grad(yr, wv, dz.view(n, gg[2], gg[3], cout).permute(0, 3, 1, 2))[0]
    dw = native().conv_wgrad(_bf(dz), _bf(x.reshape(-1, cin)), gg, coef.to(DEV) if pro else None)
    _close(dw, dw_ref.permute(0, 2, 3, 1).reshape(cout, 9 * cin))


@pytest.mark.parametrize("ks,cin,cout,hw,stride,pro", [
    (1, 256, 256, 9, 1, False), (1, 256, 256, 9, 1, True), (1, 128, 512, 7, 1, True), (1, 512, 128, 7, 1, False),
    (1, 256, 512, 11, 2, False), (3, 256, 256, 7, 1, False), (3, 256, 256, 9, 2, False), (3, 512, 256, 5, 1, False),
    (3, 128, 128, 9, 1, False), (3, 128, 128, 11, 2, False)])
def test_wide_wgrad_kernel(ks, cin, cout, hw, stride, pro):
    """conv_wgrad on the 8-wave 256 x 256 / 256 x 128 / 128 x 256 tiles (4-deep LDS-DMA ring,
    32-pixel stages, BN prologue on the X fragments for 1x1) vs fp32 autograd; pixel counts
    are not multiples of the 32-pixel stage."""
    n = 5
    g = _gen(ks * 1000 + cin + cout + hw + stride + pro)
    x = _rnd(n, hw, hw, cin, g=g)
    coef = _coef(cin, g) if pro else None
    xin = _bn_relu(x, coef) if pro else x
    gg = geo(hw, hw, ks, stride, ks // 2)
    dz = _rnd(n * gg[2] * gg[3], cout, g=g)
    wv = torch.zeros(cout, cin, ks, ks, requires_grad=True)
    yr = F.conv2d(xin.permute(0, 3, 1, 2), wv, None, stride, ks // 2)
    dw_ref = torch.autograd.grad(yr, wv, dz.view(n, gg[2], gg[3], cout).permute(0, 3, 1, 2))[0]
    dw = native().conv_wgrad(_bf(dz), _bf(x.reshape(-1, cin)), gg, coef.to(DEV) if pro else None)
    _close(dw, dw_ref.permute(0, 2, 3, 1).reshape(cout, ks * ks * cin))


@pytest.mark.parametrize("N", [256, 64])
@pytest.mark.parametrize("epi", [0, 1, 2, 3, 4, 5])
def test_deep_k_lds_dma_path_all_epilogues(epi, N):
    """K % 256 == 0, no prologue: the LDS-DMA kernel (128-channel tiles; N = 64: the tall
    256 x 64 tile) with the weight given as a strided transposed view, as the block backward
    passes it."""
    n, h, w, K = 2, 13, 11, 512
    M = n * h * w
    g = _gen(40 + epi)
    a, bt = _rnd(M, K, g=g), _rnd(K, N, g=g, scale=K ** -0.5)
    ref = a @ bt
    args = [None] * 6
    if epi == 1:
        args = [None, (torch.randn(N, generator=g) * 0.1).to(DEV), None, None, None, None]
    elif epi in (2, 5):
        r = _rnd(M, N, g=g)
        keep = torch.rand(M, N, generator=g) > 0.5
        bits = (keep.view(-1, 8).int() << torch.arange(8)).sum(1).to(torch.uint8)
        args = [_bf(r), None, None, None, None, bits.to(DEV) if epi == 5 else None]
        ref = ref + (r * keep if epi == 5 else r)
    elif epi == 3:
        z = _rnd(M, N, g=g)
        mc = _coef(N, g)
        mean, invstd = torch.randn(N, generator=g) * 0.1, torch.rand(N, generator=g) + 0.5
        args = [_bf(z), None, mc.to(DEV), mean.to(DEV), invstd.to(DEV), None]
        ref = ref * ((z * mc[:N] + mc[N:]) > 0)
    elif epi == 4:
        oh, ow = (h + 1) // 2, (w + 1) // 2
        t = _rnd(n * oh * ow, N, g=g)
        args = [_bf(t), None, None, None, None, None]
        ref.view(n, h, w, N)[:, ::2, ::2] += t.view(n, oh, ow, N)
    aux, kshift, mc, mean, invstd, bits = args
    c, part = native().conv_gemm(_bf(a), _bf(bt).t(), geo(h, w), None, epi, aux, kshift, mc, mean, invstd, bits)
    _close(c, ref)
    if epi == 1:
        cb = c.float().cpu() - kshift.cpu()
        torch.testing.assert_close(part[0].sum(0).cpu(), cb.sum(0), rtol=1e-4, atol=1e-2)
        torch.testing.assert_close(part[1].sum(0).cpu(), (cb * cb).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("cin,cout", [(256, 128), (64, 64)])
@pytest.mark.parametrize("stride", [1, 2])
def test_conv3x3_deep_k_lds_dma_path(stride, cin, cout):
    """3x3, C = 256 (K = 2304) / C = 64 (K = 576, the tall 256 x 64 tile): padding taps of the
    LDS-DMA kernel come from its zero page."""
    n, hw = 2, 9
    g = _gen(50 + stride)
    x = _rnd(n, hw, hw, cin, g=g)
    wt = _rnd(cout, cin, 3, 3, g=g, scale=(9 * cin) ** -0.5)
    ref = F.conv2d(x.permute(0, 3, 1, 2), wt, None, stride, 1).permute(0, 2, 3, 1).reshape(-1, cout)
    c, _ = native().conv_gemm(_bf(x.reshape(-1, cin)), _bf(wt.permute(0, 2, 3, 1).reshape(cout, 9 * cin)),
                              geo(hw, hw, 3, stride, 1))
    _close(c, ref)


@pytest.mark.parametrize("M,N,K", [(300, 64, 64), (5000, 256, 64), (1000, 128, 512), (777, 512, 128)])
@pytest.mark.parametrize("pro", [False, True])
def test_conv1x1_weight_grad(M, N, K, pro):
    g = _gen(M + N + K)
    dz, x = _rnd(M, N, g=g), _rnd(M, K, g=g)
    coef = _coef(K, g) if pro else None
    ref = dz.t() @ (_bn_relu(x, coef) if pro else x)
    dw = native().conv_wgrad(_bf(dz), _bf(x), [M, 1, M, 1, 1, 1, 0], coef.to(DEV) if pro else None)
    _close(dw, ref)


def test_conv1x1_weight_grad_stride2():
    n, h, w = 4, 14, 13
    gg = geo(h, w, 1, 2)
    g = _gen(11)
    dz, x = _rnd(n * gg[2] * gg[3], 256, g=g), _rnd(n * h * w, 128, g=g)
    dw = native().conv_wgrad(_bf(dz), _bf(x), gg)
    _close(dw, dz.t() @ x.view(n, h, w, 128)[:, ::2, ::2].reshape(-1, 128))


def test_bn_apply_coef_and_backward_from_partials():
    from ps_amd.ops.bn import bn_act  # noqa: F401  (module import check)

    g = _gen(5)
    R, C = 999, 192
    x, r = _rnd(R, C, g=g), _rnd(R, C, g=g)
    cf, rcf = _coef(C, g), _coef(C, g)
    y, bits = native().bn_apply_coef(_bf(x), cf.to(DEV), _bf(r), rcf.to(DEV), 1, True)
    _close(y, torch.relu(x * cf[:C] + cf[C:] + r * rcf[:C] + rcf[C:]))
    # 1 bit per element: bit j of byte v is y[8 v + j] > 0
    unpacked = ((bits.cpu()[:, None].int() >> torch.arange(8)) & 1).reshape(R, C).bool()
    assert torch.equal(unpacked, y.cpu().float() > 0)
    y0 = native().bn_apply_coef(_bf(x), cf.to(DEV), None, None, 0)[0]
    _close(y0, x * cf[:C] + cf[C:])
    # BN backward with the ReLU mask from the bits == with the mask from y
    dy = _rnd(R, C, g=g)
    gam = torch.rand(C, generator=g) + 0.5
    mu, istd = torch.randn(C, generator=g) * 0.1, torch.rand(C, generator=g) + 0.5
    ref = native().bn_act_bwd(_bf(dy), y, _bf(x), gam.to(DEV), mu.to(DEV), istd.to(DEV), 1, True, True, None)
    got = native().bn_act_bwd(_bf(dy), None, _bf(x), gam.to(DEV), mu.to(DEV), istd.to(DEV), 3, True, True, None, bits)
    for u, v in zip(ref, got):  # same masks; FMA contraction may differ by one bf16 ulp per template
        assert (u != v).float().mean().item() < 1e-3
        torch.testing.assert_close(u.float(), v.float(), rtol=8e-3, atol=1e-5)
    # backward from partial sums == backward with its own reduce pass
    gr = _rnd(R, C, g=g)
    gamma, mean, invstd = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.1, torch.rand(C) + 0.5
    xhat = (x - mean) * invstd
    part = torch.stack([gr.sum(0, keepdim=True), (gr * xhat).sum(0, keepdim=True)])
    dx, dg, db = native().bn_bwd_partials(_bf(gr), _bf(x), part.to(DEV).contiguous(), gamma.to(DEV), mean.to(DEV),
                                          invstd.to(DEV))
    ref_dx = gamma * invstd * (gr - gr.mean(0) - xhat * (gr * xhat).mean(0))
    _close(dx, ref_dx)
    torch.testing.assert_close(db.cpu(), gr.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(dg.cpu(), (gr * xhat).sum(0), rtol=1e-4, atol=1e-3)
    # strided slabs (slabs 0 and 2 of an epilogue-9 [3, G, C] part, as the downsample BN gets
    # them) == the same slabs stacked contiguously -- bitwise, also through the tall-partials fold
    for G in (1, 3000):
        p3 = torch.randn(3, G, C, generator=g).to(DEV)
        want = native().bn_bwd_partials(_bf(gr), _bf(x), p3[0::2].contiguous(), gamma.to(DEV), mean.to(DEV),
                                        invstd.to(DEV))
        got = native().bn_bwd_partials(_bf(gr), _bf(x), p3[0::2], gamma.to(DEV), mean.to(DEV), invstd.to(DEV))
        for u, v in zip(want, got):
            assert torch.equal(u, v)


@pytest.mark.parametrize("conv3x3", ["1", "0"])
@pytest.mark.parametrize("inplanes,planes,stride", [(256, 64, 1), (64, 64, 1), (256, 128, 2), (512, 128, 1)])
def test_fused_bottleneck_matches_module_path(inplanes, planes, stride, conv3x3, monkeypatch):
    """Fused block (3x3 conv on our GEMMs or, PS_AMD_DISABLE=conv3x3, on MIOpen) vs module path."""
    import torch.nn as nn

    from ps_amd.models.resnet import Bottleneck, prepare_for_mi355x
    from ps_amd.ops.bn import BatchNormAct2d
    from ps_amd.ops.convgemm import fused_block_ok

    monkeypatch.setenv("PS_AMD_DISABLE", "" if conv3x3 == "1" else "conv3x3")
    torch.manual_seed(0)
    ds = None
    if stride != 1 or inplanes != planes * 4:
        ds = nn.Sequential(nn.Conv2d(inplanes, planes * 4, 1, stride=stride, bias=False),
                           BatchNormAct2d(planes * 4, act="none"))
    a = Bottleneck(inplanes, planes, stride, ds)
    for m in a.modules():
        if isinstance(m, nn.BatchNorm2d):
            nn.init.uniform_(m.weight, 0.5, 1.5)
            nn.init.uniform_(m.bias, -0.2, 0.2)
    b = copy.deepcopy(a)
    b.fuse_block = False
    a, b = prepare_for_mi355x(a.cuda()), prepare_for_mi355x(b.cuda())
    x = torch.randn(4, inplanes, 15, 15, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    assert fused_block_ok(a, x) and not fused_block_ok(b, x)
    xa, xb = x.clone().requires_grad_(), x.clone().requires_grad_()
    ya, yb = a(xa), b(xb)
    _close(ya.detach(), yb.detach(), tol=2e-2, amax=0.1)
    gout = torch.randn_like(ya)
    ya.backward(gout)
    yb.backward(gout)
    # bf16 ReLU-mask flips near 0 differ per path (and per MIOpen solver choice): a flipped
    # element may differ by O(its own magnitude), so the max-abs bound is on all but 0.05 %
    _close_flips(xa.grad, xb.grad, tol=3e-2, amax=0.25)
    for (name, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        assert p.grad is not None, name
        _close(p.grad, q.grad, tol=3e-2, amax=0.25)
    for (name, t), (_, u) in zip(a.named_buffers(), b.named_buffers()):
        torch.testing.assert_close(t.float(), u.float(), rtol=2e-3, atol=2e-3, msg=name)


def test_tall_partials_fold_into_bn_finalize():
    """G > 2048 partial rows (per-tile partials of a non-persistent conv GEMM) take a first-level
    fold (partials_fold_kernel) before the finalize kernels; sums vs fp64."""
    G, C, R = 5000, 64, 100000
    g = _gen(77)
    part = torch.stack([torch.randn(G, C, generator=g), torch.rand(G, C, generator=g) * 40])
    kshift = torch.randn(C, generator=g)
    mean, invstd, coef = native().bn_finalize_sums(part.to(DEV), kshift.to(DEV), R, None, None, None, None, 0.1, 1e-5)
    s1, s2 = part[0].double().sum(0), part[1].double().sum(0)
    dm = s1 / R
    torch.testing.assert_close(mean.cpu().double(), kshift.double() + dm, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(invstd.cpu().double(), (s2 / R - dm * dm + 1e-5).rsqrt(), rtol=1e-4, atol=1e-5)
    x = _rnd(3000, C, g=g)
    gr = _rnd(3000, C, g=g)
    m, i = torch.randn(C, generator=g) * 0.1, torch.rand(C, generator=g) + 0.5
    _, dgamma, dbeta = native().bn_bwd_partials(_bf(gr), _bf(x), part.to(DEV), None, m.to(DEV), i.to(DEV))
    torch.testing.assert_close(dbeta.cpu().double(), s1, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(dgamma.cpu().double(), s2, rtol=1e-5, atol=1e-2)


@pytest.mark.parametrize("epi", [6, 7, 8])
@pytest.mark.parametrize("K", [64, 512])
def test_fold_epilogues_previous_block_bn3_reduce(epi, K):
    """Epilogues 6/7/8 (= 5/2/4 + the previous block's bn3 backward reduce): output masked by
    the previous block's output bits, partial sums of g and g * (z3 - mean) * invstd."""
    n, h, w, N = 2, 13, 11, 256
    M = n * h * w
    g = _gen(90 + epi + K)
    a, bt = _rnd(M, K, g=g), _rnd(K, N, g=g, scale=K ** -0.5)
    ref = a @ bt
    bits = None
    if epi == 6:
        r = _rnd(M, N, g=g)
        keep = torch.rand(M, N, generator=g) > 0.5
        bits = (keep.view(-1, 8).int() << torch.arange(8)).sum(1).to(torch.uint8).to(DEV)
        aux = r
        ref = ref + r * keep
    elif epi == 7:
        aux = _rnd(M, N, g=g)
        ref = ref + aux
    else:
        oh, ow = (h + 1) // 2, (w + 1) // 2
        aux = _rnd(n * oh * ow, N, g=g)
        ref.view(n, h, w, N)[:, ::2, ::2] += aux.view(n, oh, ow, N)
    ref = ref.bfloat16().float()
    z3 = _rnd(M, N, g=g)
    keep2 = torch.rand(M, N, generator=g) > 0.4
    bits2 = (keep2.view(-1, 8).int() << torch.arange(8)).sum(1).to(torch.uint8)
    mean, invstd = torch.randn(N, generator=g) * 0.1, torch.rand(N, generator=g) + 0.5
    c, part = native().conv_gemm(_bf(a), _bf(bt).t(), geo(h, w), None, epi, _bf(aux), None, None, mean.to(DEV),
                                 invstd.to(DEV), bits, _bf(z3), bits2.to(DEV))
    gref = ref * keep2
    _close(c, gref)
    gc = c.float().cpu()
    assert torch.all(gc[~keep2] == 0)
    torch.testing.assert_close(part[0].sum(0).cpu(), gc.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part[1].sum(0).cpu(), (gc * (z3 - mean) * invstd).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("extra_consumer,wide", [(False, False), (True, False), (False, True)])
def test_chained_blocks_fold_bn3_backward(extra_consumer, wide, monkeypatch):
    """Three fused bottlenecks (downsample first) inside the ResNet forward context: block i's
    conv1 data-grad epilogue reduces block i-1's bn3 backward.  Checked against the same fused
    chain with the fold disabled (PS_AMD_DISABLE=fold_bn3: every block runs its own reduce pass).
    With a second consumer of a block output autograd sums the gradients and that block must
    fall back to its own reduce.  (Fused vs module path per block: the test above.)"""
    import torch.nn as nn

    from ps_amd.models.resnet import Bottleneck, prepare_for_mi355x
    from ps_amd.ops import convgemm as cg
    from ps_amd.ops.bn import BatchNormAct2d

    torch.manual_seed(1)
    # wide: 1024-channel block outputs -- the deep-K (LDS-DMA) two-source prologues
    cin, pl = (512, 256) if wide else (128, 64)
    ds = nn.Sequential(nn.Conv2d(cin, 4 * pl, 1, stride=2, bias=False), BatchNormAct2d(4 * pl, act="none"))
    a = nn.Sequential(Bottleneck(cin, pl, 2, ds), Bottleneck(4 * pl, pl), Bottleneck(4 * pl, pl))
    for m in a.modules():
        if isinstance(m, nn.BatchNorm2d):
            nn.init.uniform_(m.weight, 0.5, 1.5)
            nn.init.uniform_(m.bias, -0.2, 0.2)
    a = prepare_for_mi355x(a.cuda())
    x = torch.randn(4, cin, 17, 17, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    gw = torch.randn(4, 4 * pl, 9, 9, device=DEV)
    gw1 = torch.randn(4, 4 * pl, 9, 9, device=DEV)
    state = copy.deepcopy(a.state_dict())

    def run(defer=False):
        a.load_state_dict(state)
        a.zero_grad()
        a[0]._defer_out = a[1]._defer_out = defer  # (set by ResNet.forward on the model path)
        xi = x.clone().requires_grad_()
        with cg.deferred_bn_counters():
            y1 = a[0](xi)
            y3 = a[2](a[1](y1))
        loss = (y3.float() * gw).sum()
        if extra_consumer:
            loss = loss + (y1.float() * gw1).sum()
        loss.backward()
        return xi.grad.clone(), {n: p.grad.clone() for n, p in a.named_parameters()}

    before, before_ds = cg.FOLD_STATS["used"], cg.FOLD_STATS["ds"]
    ga, pa = run()
    assert cg.FOLD_STATS["used"] - before == (1 if extra_consumer else 2)
    # the downsample block's BN sum rides in block 1's epilogue 9 unless y1 has a second consumer
    assert cg.FOLD_STATS["ds"] - before_ds == (0 if extra_consumer else 1)
    monkeypatch.setenv("PS_AMD_DISABLE", "fold_bn_ds")  # bn3 folded, the downsample BN reduced on its own
    gc, pc = run()
    _close(ga, gc, tol=1e-2, amax=0.05)
    for n in pc:
        _close(pa[n], pc[n], tol=1e-2, amax=0.05)
    monkeypatch.delenv("PS_AMD_DISABLE")
    # block outputs applied in the next block's conv1 prologue (PRO 3): same gradients, and the
    # forward outputs / ReLU bits they store equal the apply pass's
    before = cg.FOLD_STATS["resp"]
    gr, pr = run(defer=True)
    assert cg.FOLD_STATS["resp"] - before == 2
    _close(ga, gr, tol=1e-2, amax=0.05)
    for n in pr:
        _close(pa[n], pr[n], tol=1e-2, amax=0.05)
    monkeypatch.setenv("PS_AMD_DISABLE", "fold_bn3")
    before = cg.FOLD_STATS["used"]
    gb, pb = run()
    assert cg.FOLD_STATS["used"] == before
    _close(ga, gb, tol=1e-2, amax=0.05)
    for n in pb:
        _close(pa[n], pb[n], tol=1e-2, amax=0.05)


@pytest.mark.parametrize("n,h,w,C1,C2", [(3, 15, 13, 64, 64), (2, 9, 9, 128, 256)])
def test_conv3x3_data_grad_with_bn_backward_sums(n, h, w, C1, C2):
    """Stride-1 3x3 data gradient as the forward GEMM over dz with the flipped / transposed
    weight (ops/convgemm._mat3_dgrad), epilogue 3: the ReLU mask of the bn1 output recomputed
    from z1 and bn1's backward sums -- vs fp32 torch (conv2d_input)."""
    from ps_amd.ops.convgemm import _mat3_dgrad

    g = _gen(n * h + C1 + C2)
    wt = _rnd(C2, C1, 3, 3, g=g, scale=(9 * C1) ** -0.5)
    dz = _rnd(n, h, w, C2, g=g)
    z1 = _rnd(n, h, w, C1, g=g)
    coef = _coef(C1, g)
    mean, invstd = torch.randn(C1, generator=g) * 0.1, torch.rand(C1, generator=g) + 0.5
    dy = torch.nn.grad.conv2d_input((n, C1, h, w), wt, dz.permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    on = (z1 * coef[:C1] + coef[C1:]) > 0
    gref = (dy.bfloat16().float() * on).reshape(-1, C1)
    wd = _mat3_dgrad(_bf(wt))
    c, part = native().conv_gemm(_bf(dz).reshape(-1, C2), wd, geo(h, w, 3, 1, 1), None, 3,
                                 _bf(z1).reshape(-1, C1), None, coef.to(DEV), mean.to(DEV), invstd.to(DEV))
    _close(c, gref)
    gc = c.float().cpu()
    xhat = (z1.reshape(-1, C1) - mean) * invstd
    torch.testing.assert_close(part[0].sum(0).cpu(), gc.sum(0), rtol=1e-4, atol=2e-2)
    torch.testing.assert_close(part[1].sum(0).cpu(), (gc * xhat).sum(0), rtol=1e-4, atol=2e-2)


@pytest.mark.parametrize("n,h,w,C1,C2,epi", [(2, 14, 10, 128, 128, 3), (3, 8, 8, 64, 256, 0), (1, 28, 28, 256, 64, 3),
                                             (2, 6, 12, 512, 128, 0)])
def test_conv3x3_stride2_data_grad_phases(n, h, w, C1, C2, epi):
    """Stride-2 3x3 data gradient as four stride-1 phase GEMMs over dz (csrc conv_dgrad_s2), each
    writing every other dx row; epilogue 3: bn1's ReLU mask from z1 and its backward sums over
    the concatenated phase partials -- vs fp32 torch (conv2d_input)."""
    from ps_amd.ops.convgemm import _phase_weights

    g = _gen(7 * n + h + C1 + C2 + epi)
    oh, ow = h // 2, w // 2
    wt = _rnd(C2, C1, 3, 3, g=g, scale=(9 * C1) ** -0.5)
    dz = _rnd(n, oh, ow, C2, g=g)
    dy = torch.nn.grad.conv2d_input((n, C1, h, w), wt, dz.permute(0, 3, 1, 2), stride=2, padding=1)
    dy = dy.permute(0, 2, 3, 1).reshape(-1, C1)
    if epi == 0:
        c, _ = native().conv_dgrad_s2(_bf(dz).reshape(-1, C2), _phase_weights(_bf(wt)), h, w)
        _close(c, dy)
        return
    z1 = _rnd(n, h, w, C1, g=g).reshape(-1, C1)
    coef = _coef(C1, g)
    mean, invstd = torch.randn(C1, generator=g) * 0.1, torch.rand(C1, generator=g) + 0.5
    on = (z1 * coef[:C1] + coef[C1:]) > 0
    gref = dy.bfloat16().float() * on
    c, part = native().conv_dgrad_s2(_bf(dz).reshape(-1, C2), _phase_weights(_bf(wt)), h, w, 3, _bf(z1),
                                     coef.to(DEV), mean.to(DEV), invstd.to(DEV))
    _close(c, gref)
    gc = c.float().cpu()
    xhat = (z1 - mean) * invstd
    torch.testing.assert_close(part[0].sum(0).cpu(), gc.sum(0), rtol=1e-4, atol=2e-2)
    torch.testing.assert_close(part[1].sum(0).cpu(), (gc * xhat).sum(0), rtol=1e-4, atol=2e-2)


def test_weight_prep_matches_reference_layouts(monkeypatch):
    """csrc weight_prep (one launch for every fused block) == the per-weight torch layouts the data
    gradients used before; and a ResNet-tiny backward is bitwise the same with and without it."""
    from ps_amd.models.resnet import prepare_for_mi355x, resnet_tiny
    from ps_amd.ops import convgemm as cg

    torch.manual_seed(3)
    m = prepare_for_mi355x(resnet_tiny(num_classes=10).cuda())
    blocks = m._blocks()
    cg.prepare_backward_weights(blocks)
    prep = cg._tls.prep
    cg._tls.prep = None
    for b in blocks:
        w1t, w3t, w2d, wdt, _ = prep[id(b)]
        assert torch.equal(w1t, cg._mat(b.conv1.weight).t())
        assert torch.equal(w3t, cg._mat(b.conv3.weight).t())
        if b.conv2.stride[0] == 1:
            assert torch.equal(w2d, cg._mat3_dgrad(b.conv2.weight))
        else:
            for u, v in zip(w2d, cg._phase_weights(b.conv2.weight)):
                assert torch.equal(u, v)
        if b.downsample is not None:
            assert torch.equal(wdt, cg._mat(b.downsample[0].weight).t())
    monkeypatch.setattr(cg, "WGRAD3X3_MIN_C", 64)  # in-house weight gradients: deterministic
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(8, 3, 64, 64, device=DEV, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=DEV, generator=g)
    grads = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PS_AMD_DISABLE", "" if flag == "1" else "weight_prep")
        mm = copy.deepcopy(m)
        F.cross_entropy(mm(x).float(), y).backward()
        grads[flag] = {n: p.grad.clone() for n, p in mm.named_parameters()}
    for n, gr in grads["0"].items():
        assert torch.equal(grads["1"][n], gr), n


@pytest.mark.parametrize("n,hw,cin,cout", [(2, 56, 64, 64), (10, 56, 64, 64), (20, 56, 64, 64), (3, 28, 128, 128),
                                           (2, 14, 256, 256), (2, 28, 64, 128)])
def test_conv3x3_patch_forward_statistics_and_data_grad(n, hw, cin, cout):
    """3x3 stride-1 forward on the patch-staged tiles (PS_AMD_CONV_PATCH, default on: the tile's
    input rows staged once per 64-channel chunk, tiles straddling two images) with the BN
    statistics epilogue, and the data gradient (flipped weight) with epilogue 3 -- vs fp32 torch.
    n = 10 / 20 at 56 x 56: tiles crossing image boundaries and grids of several waves."""
    from ps_amd.ops.convgemm import _mat3_dgrad

    g = _gen(n * hw + cin + cout)
    x = _rnd(n, hw, hw, cin, g=g)
    wt = _rnd(cout, cin, 3, 3, g=g, scale=(9 * cin) ** -0.5)
    ref = F.conv2d(x.permute(0, 3, 1, 2), wt, None, 1, 1).permute(0, 2, 3, 1).reshape(-1, cout)
    ks = torch.randn(cout, generator=g) * 0.1
    c, part = native().conv_gemm(_bf(x.reshape(-1, cin)), _bf(wt.permute(0, 2, 3, 1).reshape(cout, 9 * cin)),
                                 geo(hw, hw, 3, 1, 1), None, 1, None, ks.to(DEV))
    _close(c, ref)
    cf = c.float().cpu()
    torch.testing.assert_close(part[0].sum(0).cpu(), (cf - ks).sum(0), rtol=1e-4, atol=5e-2)
    torch.testing.assert_close(part[1].sum(0).cpu(), ((cf - ks) ** 2).sum(0), rtol=1e-4, atol=5e-2)
    # data gradient: dz [n, hw, hw, cout] -> dy [.., cin], ReLU mask + bn sums over z1
    dz = _rnd(n, hw, hw, cout, g=g)
    z1 = _rnd(n, hw, hw, cin, g=g)
    coef = _coef(cin, g)
    mean, invstd = torch.randn(cin, generator=g) * 0.1, torch.rand(cin, generator=g) + 0.5
    dy = torch.nn.grad.conv2d_input((n, cin, hw, hw), wt, dz.permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    on = (z1 * coef[:cin] + coef[cin:]) > 0
    gref = (dy.bfloat16().float() * on).reshape(-1, cin)
    c2, p2 = native().conv_gemm(_bf(dz).reshape(-1, cout), _mat3_dgrad(_bf(wt)), geo(hw, hw, 3, 1, 1), None, 3,
                                _bf(z1).reshape(-1, cin), None, coef.to(DEV), mean.to(DEV), invstd.to(DEV))
    _close(c2, gref)
    gc = c2.float().cpu()
    xhat = (z1.reshape(-1, cin) - mean) * invstd
    torch.testing.assert_close(p2[0].sum(0).cpu(), gc.sum(0), rtol=1e-4, atol=5e-2)
    torch.testing.assert_close(p2[1].sum(0).cpu(), (gc * xhat).sum(0), rtol=1e-4, atol=5e-2)


@pytest.mark.parametrize("M,K,N", [(3000, 64, 256), (1000, 128, 512), (517, 512, 256)])
def test_epilogue9_downsample_bn_sum(M, K, N):
    """Epilogue 9 = epilogue 6 (+ residual masked by bits, output masked by the previous block's
    bits, bn3 sums) + the third partial sum(g * (zd - mean2) * invstd2) of the previous block's
    downsample BN: same output and first two slabs as epilogue 6, third slab vs fp32.  K = 64 / 128
    run the persistent register-staged tiles (the third sum lives in LDS), K = 512 the LDS-DMA one."""
    g = _gen(M + K + N)
    a, b = _rnd(M, K, g=g), _rnd(N, K, g=g, scale=K ** -0.5)
    r, z3, zd = _rnd(M, N, g=g), _rnd(M, N, g=g), _rnd(M, N, g=g)

    def bits_of(keep):
        return (keep.view(-1, 8).int() << torch.arange(8)).sum(1).to(torch.uint8).to(DEV)

    k1, k2 = torch.rand(M, N, generator=g) > 0.5, torch.rand(M, N, generator=g) > 0.4
    m3, i3 = torch.randn(N, generator=g) * 0.1, torch.rand(N, generator=g) + 0.5
    md, idd = torch.randn(N, generator=g) * 0.1, torch.rand(N, generator=g) + 0.5
    common = dict(bits=bits_of(k1), aux2=_bf(z3), bits2=bits_of(k2), mean=m3.to(DEV), invstd=i3.to(DEV))
    geo1 = [M, 1, M, 1, 1, 1, 0]
    c6, p6 = native().conv_gemm(_bf(a), _bf(b), geo1, None, 6, _bf(r), **common)
    c9, p9 = native().conv_gemm(_bf(a), _bf(b), geo1, None, 9, _bf(r), aux3=_bf(zd), mean2=md.to(DEV),
                                invstd2=idd.to(DEV), **common)
    assert p9.shape[0] == 3 and torch.equal(c6, c9)
    torch.testing.assert_close(p9[:2], p6, rtol=0, atol=0)
    gv = c9.float().cpu()
    torch.testing.assert_close(p9[2].sum(0).cpu(), (gv * ((zd - md) * idd)).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("M,C,N,dual", [(300, 256, 64, False), (4099, 256, 128, True), (1000, 64, 64, False),
                                        (517, 512, 256, True), (700, 1024, 128, False), (129, 2048, 512, False)])
def test_block_output_prologue_matches_apply_then_gemm(M, C, N, dual):
    """conv_gemm(z3, pro=bn3 coef, a2=r[, pro2=downsample coef], aout, abits) == bn_apply_coef
    (the block output relu(bn3(z3) + r) and its ReLU bits) then conv_gemm on that output with
    the BN-statistics epilogue: the consumer block's conv1 applies the previous block's output
    while staging A and stores it (rows + bits) for the residual and the backward.  K >= 320 runs
    the LDS-DMA two-source variant (both row sources DMA'd, one in-place pass per stage), below
    the register-staged one."""
    g = _gen(M + C + N)
    z3, r = _rnd(M, C, g=g), _rnd(M, C, g=g)
    cf3 = _coef(C, g).to(DEV)
    cfd = _coef(C, g).to(DEV) if dual else None
    b = _rnd(N, C, g=g, scale=C ** -0.5)
    ks = (torch.randn(N, generator=g) * 0.1).to(DEV)
    geo = [M, 1, M, 1, 1, 1, 0]
    y_ref, bits_ref = native().bn_apply_coef(_bf(z3), cf3, _bf(r), cfd, 1, True)
    c_ref, p_ref = native().conv_gemm(y_ref, _bf(b), geo, None, 1, None, ks)
    y = torch.full_like(y_ref, float("nan"))
    bits = torch.zeros_like(bits_ref)
    c, p = native().conv_gemm(_bf(z3), _bf(b), geo, cf3, 1, None, ks, a2=_bf(r), pro2=cfd, aout=y, abits=bits)
    torch.cuda.synchronize()
    # same arithmetic as the apply kernels; FMA contraction may move a value by one bf16 ulp
    assert (y != y_ref).float().mean().item() < 1e-2
    torch.testing.assert_close(y.float(), y_ref.float(), rtol=8e-3, atol=1e-3)
    assert (bits != bits_ref).float().mean().item() < 1e-2
    _close(c, c_ref, tol=1e-2, amax=0.05)
    assert p.shape[0] == 2 and p.shape[2] == N
    torch.testing.assert_close(p.sum(1), p_ref.sum(1), rtol=2e-3, atol=2e-2)


def test_layer1_chain_single_pass_backwards_match_unfused(monkeypatch):
    """Layer-1 shapes (64 -> 256, stride 1): conv3's backward and the downsample branch's backward
    each run as ONE pass with the BN backward in the prologue (conv_bwd_fused.hip, normal and PLAIN
    modes).  Against the same chain with both passes split back into apply + two GEMMs."""
    import torch.nn as nn

    from ps_amd.models.resnet import Bottleneck, prepare_for_mi355x
    from ps_amd.ops import convgemm as cg
    from ps_amd.ops.bn import BatchNormAct2d

    torch.manual_seed(2)
    ds = nn.Sequential(nn.Conv2d(64, 256, 1, bias=False), BatchNormAct2d(256, act="none"))
    a = nn.Sequential(Bottleneck(64, 64, 1, ds), Bottleneck(256, 64), Bottleneck(256, 64))
    for m in a.modules():
        if isinstance(m, nn.BatchNorm2d):
            nn.init.uniform_(m.weight, 0.5, 1.5)
            nn.init.uniform_(m.bias, -0.2, 0.2)
    a = prepare_for_mi355x(a.cuda())
    x = torch.randn(4, 64, 19, 19, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    gw = torch.randn(4, 256, 19, 19, device=DEV)
    state = copy.deepcopy(a.state_dict())

    def run():
        a.load_state_dict(state)
        a.zero_grad()
        xi = x.clone().requires_grad_()
        with cg.deferred_bn_counters():
            y = a(xi)
        (y.float() * gw).sum().backward()
        return xi.grad.clone(), {n: p.grad.clone() for n, p in a.named_parameters()}

    c3, dsf = cg.FOLD_STATS.get("conv3_fused", 0), cg.FOLD_STATS.get("ds_fused", 0)
    ga, pa = run()
    assert cg.FOLD_STATS.get("conv3_fused", 0) - c3 == 2  # blocks 0 and 1 (block 2 has no consumer)
    assert cg.FOLD_STATS.get("ds_fused", 0) - dsf == 1
    monkeypatch.setenv("PS_AMD_DISABLE", "ds_bwd_fused,conv3_bwd_fused")
    gb, pb = run()
    _close(ga, gb, tol=1e-2, amax=0.05)
    for n in pb:
        _close(pa[n], pb[n], tol=1e-2, amax=0.05)
