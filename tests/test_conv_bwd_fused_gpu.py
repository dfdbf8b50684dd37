"""conv3's fused backward (csrc/kernels/conv_bwd_fused.hip) vs fp32 torch and vs the two-kernel
chain it replaces (conv_gemm with the BN-backward prologue storing dz3, then conv_wgrad re-reading
it).  Pixel counts leave partial tiles and give blocks one to several tiles each."""
import pytest
import torch

from ps_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bf(t):
    return t.bfloat16().to(DEV).contiguous()


def _rnd(*shape, g, scale=1.0):
    return (torch.randn(*shape, generator=g) * scale).bfloat16().float()


def _close(out, ref, tol=1e-2, amax=0.05):
    out, ref = out.float().cpu(), ref.float().cpu()
    err = ((out - ref).norm() / ref.norm().clamp_min(1e-12)).item()
    assert err < tol, f"relative error {err:.3g}"
    assert (out - ref).abs().max().item() <= amax * ref.abs().max().item() + 1e-3


def _problem(M, CI, CO, seed):
    g = torch.Generator().manual_seed(seed)
    d, z3 = _rnd(M, CO, g=g), _rnd(M, CO, g=g)
    gamma, mean, invstd = torch.rand(CO, generator=g) + 0.5, torch.randn(CO, generator=g) * 0.1, torch.rand(CO) + 0.5
    xhat = (z3 - mean) * invstd
    part = torch.stack([d.sum(0, keepdim=True), (d * xhat).sum(0, keepdim=True)]).to(DEV).contiguous()
    dg, db, coef = native().bn_bwd_coef(part, gamma.to(DEV), mean.to(DEV), invstd.to(DEV), M)
    w3 = _rnd(CO, CI, g=g, scale=CO ** -0.5)  # conv3 weight [CO, CI]
    z2 = _rnd(M, CI, g=g)
    cf2 = torch.cat([torch.rand(CI, generator=g) + 0.5, torch.randn(CI, generator=g) * 0.5])
    m2, i2 = torch.randn(CI, generator=g) * 0.1, torch.rand(CI, generator=g) + 0.5
    return d, z3, coef, w3, z2, cf2, m2, i2


@pytest.mark.parametrize("M,CI,CO", [(300, 64, 256), (4099, 64, 256), (100003, 64, 256), (38401, 64, 256)])
def test_conv3_fused_backward_matches_fp32_and_two_kernel_chain(M, CI, CO):
    d, z3, coef, w3, z2, cf2, m2, i2 = _problem(M, CI, CO, M + CO)
    assert native().conv11_bwd_fused_supported(CI, CO)
    w3t = _bf(w3.t())
    gy, part, dw = native().conv11_bwd_fused(_bf(d), _bf(z3), coef, w3t, _bf(z2), cf2.to(DEV), m2.to(DEV), i2.to(DEV))
    torch.cuda.synchronize()
    # fp32 reference of the same op (dz3 rounded to bf16 as the kernel stages it)
    c = coef.cpu()
    dz3 = (c[:CO] * d + c[CO:2 * CO] * z3 + c[2 * CO:]).bfloat16().float()
    on = (z2 * cf2[:CI] + cf2[CI:]) > 0
    gy_ref = (dz3 @ w3) * on
    _close(gy, gy_ref)
    a2 = torch.relu((z2 * cf2[:CI] + cf2[CI:]).bfloat16().float())
    _close(dw, dz3.t() @ a2)
    gyf = gy.float().cpu()
    torch.testing.assert_close(part[0].sum(0).cpu(), gyf.sum(0), rtol=2e-3, atol=3e-2)
    torch.testing.assert_close(part[1].sum(0).cpu(), (gyf * ((z2 - m2) * i2)).sum(0), rtol=2e-3, atol=3e-2)
    assert part.shape[0] == 2 and part.shape[2] == CI
    # the chain it replaces: prologue GEMM (stores dz3) + weight-gradient GEMM
    geo = [M, 1, M, 1, 1, 1, 0]
    c_ref, p_ref, dz_ref = native().conv_gemm(_bf(d), w3t, geo, None, 3, _bf(z2), None, cf2.to(DEV), m2.to(DEV),
                                              i2.to(DEV), a2=_bf(z3), bwd=coef)
    dw_ref = native().conv_wgrad(dz_ref, _bf(z2), geo, cf2.to(DEV))
    _close(gy, c_ref, tol=5e-3, amax=0.03)
    _close(dw, dw_ref, tol=5e-3, amax=0.03)
    torch.testing.assert_close(part.sum(1), p_ref.sum(1), rtol=2e-3, atol=3e-2)


@pytest.mark.parametrize("CI,CO", [(64, 256)])
def test_conv3_fused_backward_deterministic(CI, CO):
    M = 70001
    d, z3, coef, w3, z2, cf2, m2, i2 = _problem(M, CI, CO, 5)
    args = (_bf(d), _bf(z3), coef, _bf(w3.t()), _bf(z2), cf2.to(DEV), m2.to(DEV), i2.to(DEV))
    a = native().conv11_bwd_fused(*args)
    b = native().conv11_bwd_fused(*args)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("M", [300, 4099, 100003])
def test_downsample_plain_backward_matches_fp32(M):
    """PLAIN mode (the block's downsample branch): z2 is the weight gradient's operand as is and the
    data gradient leaves unmasked, with no partial sums."""
    CI, CO = 64, 256
    d, zd, coef, wd, x, _, _, _ = _problem(M, CI, CO, M + 7)
    assert native().conv11_bwd_fused_supported(CI, CO, True)
    t, part, dw = native().conv11_bwd_fused(_bf(d), _bf(zd), coef, _bf(wd.t()), _bf(x))
    torch.cuda.synchronize()
    assert part.numel() == 0
    c = coef.cpu()
    dzd = (c[:CO] * d + c[CO:2 * CO] * zd + c[2 * CO:]).bfloat16().float()
    _close(t, dzd @ wd)
    _close(dw, dzd.t() @ x)
    # against the chain it replaces: apply pass + data-gradient GEMM + weight-gradient GEMM
    geo = [M, 1, M, 1, 1, 1, 0]
    t_ref = native().conv_gemm(_bf(dzd), _bf(wd.t()), geo)[0]
    dw_ref = native().conv_wgrad(_bf(dzd), _bf(x), geo)
    _close(t, t_ref, tol=5e-3, amax=0.03)
    _close(dw, dw_ref, tol=5e-3, amax=0.03)
