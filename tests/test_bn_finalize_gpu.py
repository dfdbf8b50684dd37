"""One-launch BN finalize (csrc/kernels/bn_act.hip bn_fin3_kernel) straight from producer partial sums
[2, G, C]: the forward statistics (bn_finalize_sums) and the backward coefficients (bn_bwd_coef) vs
an fp64 torch reference, at partial-row counts from 1 to past the chunk cap, bitwise repeatable."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _native():
    from ps_amd.ops._ext import native

    return native()


SHAPES = [(1, 64), (37, 64), (256, 128), (257, 64), (3136, 256), (25088, 64), (40000, 64), (196, 2048), (784, 1024)]


@pytest.mark.parametrize("G,C", SHAPES)
def test_forward_statistics_match_fp64(G, C):
    g = torch.Generator(device=DEV).manual_seed(G + C)
    part = torch.randn(2, G, C, device=DEV, generator=g)
    part[1] = part[1].abs() * 3 + 1  # sum((x - k)^2) > 0
    R = G * 128
    ks = torch.randn(C, device=DEV, generator=g) * 0.1
    gamma, beta = torch.rand(C, device=DEV, generator=g) + 0.5, torch.randn(C, device=DEV, generator=g)
    rm, rv = torch.randn(C, device=DEV, generator=g), torch.rand(C, device=DEV, generator=g) + 0.5
    rm0, rv0 = rm.clone(), rv.clone()
    mean, invstd, coef = _native().bn_finalize_sums(part, ks, R, gamma, beta, rm, rv, 0.1, 1e-5)
    s1, s2 = part[0].double().sum(0), part[1].double().sum(0)
    dm = s1 / R
    var = (s2 / R - dm * dm).clamp_min(0)
    want_mean = ks.double() + dm
    want_is = (var + 1e-5).rsqrt()
    torch.testing.assert_close(mean.double(), want_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(invstd.double(), want_is, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(coef[:C].double(), gamma.double() * want_is, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(coef[C:].double(), beta.double() - want_mean * gamma.double() * want_is,
                               rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rm.double(), 0.9 * rm0.double() + 0.1 * want_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv.double(), 0.9 * rv0.double() + 0.1 * var * R / (R - 1), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("G,C", SHAPES)
def test_backward_coefficients_match_fp64_and_repeat(G, C):
    g = torch.Generator(device=DEV).manual_seed(7 * G + C)
    part = torch.randn(2, G, C, device=DEV, generator=g)
    R = G * 128
    gamma = torch.rand(C, device=DEV, generator=g) + 0.5
    mean, invstd = torch.randn(C, device=DEV, generator=g) * 0.1, torch.rand(C, device=DEV, generator=g) + 0.5
    dg, db, coef = _native().bn_bwd_coef(part, gamma, mean, invstd, R)
    sd, sx = part[0].double().sum(0), part[1].double().sum(0)
    torch.testing.assert_close(db.double(), sd, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(dg.double(), sx, rtol=1e-5, atol=1e-3)
    k = gamma.double() * invstd.double()
    md, mx = sd / R, sx / R
    torch.testing.assert_close(coef[:C].double(), k, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(coef[C:2 * C].double(), -k * invstd.double() * mx, rtol=1e-4, atol=1e-8)
    torch.testing.assert_close(coef[2 * C:].double(), -k * md + k * invstd.double() * mx * mean.double(),
                               rtol=1e-4, atol=1e-8)
    for _ in range(3):  # fixed-order sums: identical whichever block of a group arrives last
        dg2, db2, coef2 = _native().bn_bwd_coef(part, gamma, mean, invstd, R)
        assert torch.equal(dg, dg2) and torch.equal(db, db2) and torch.equal(coef, coef2)
