"""One-launch BN finalize (csrc/kernels/bn_act.hip bn_fin2_kernel): the statistics / backward
coefficients from [2, G, C] producer partials, chunk sums published agent-coherently and added in
chunk order by the last block of each 64-channel group -- vs a float64 torch reference of the same
math, bitwise repeatable, and the arrival counters back at zero (a second call on the same stream
gives the same answer)."""
import os

import pytest
import torch

from ps_amd.ops import native

# the switch is read once per process: these tests pin the kernel only when the run opts in
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(os.environ.get("PS_AMD_BN_FIN2") != "1",
                                                  reason="one-launch finalize is opt-in (PS_AMD_BN_FIN2=1)")]
DEV = "cuda"


def _part(G, C, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(2, G, C, generator=g, device=DEV) * 3 + 1, g


@pytest.mark.parametrize("G,C", [(1, 64), (7, 128), (196, 2048), (785, 256), (12544, 64), (3136, 512)])
def test_fin2_forward_statistics(G, C):
    part, g = _part(G, C, G + C)
    part[1] = part[1].abs() * 50  # sum of squares: positive, variance > 0
    R = G * 256
    kshift = torch.randn(C, generator=g, device=DEV)
    gamma, beta = torch.rand(C, generator=g, device=DEV) + 0.5, torch.randn(C, generator=g, device=DEV)
    rmean, rvar = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    rm0, rv0 = rmean.clone(), rvar.clone()
    mean, invstd, coef = native().bn_finalize_sums(part, kshift, R, gamma, beta, rmean, rvar, 0.1, 1e-5)
    s1, s2 = part[0].double().sum(0), part[1].double().sum(0)
    dm = s1 / R
    var = (s2 / R - dm * dm).clamp_min(0)
    m_ref = kshift.double() + dm
    i_ref = (var + 1e-5).rsqrt()
    torch.testing.assert_close(mean.double(), m_ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(invstd.double(), i_ref, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(coef[:C].double(), gamma.double() * i_ref, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(coef[C:].double(), beta.double() - m_ref * gamma.double() * i_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rmean.double(), 0.9 * rm0.double() + 0.1 * m_ref, rtol=1e-5, atol=1e-5)
    unb = var * R / (R - 1)
    torch.testing.assert_close(rvar.double(), 0.9 * rv0.double() + 0.1 * unb, rtol=1e-4, atol=1e-5)
    again = native().bn_finalize_sums(part, kshift, R, gamma, beta, None, None, 0.1, 1e-5)
    assert torch.equal(again[0], mean) and torch.equal(again[1], invstd) and torch.equal(again[2], coef)


@pytest.mark.parametrize("G,C", [(1, 64), (33, 256), (196, 2048), (12544, 64), (3136, 512)])
def test_fin2_backward_coefficients(G, C):
    part, g = _part(G, C, 7 * G + C)
    R = G * 256
    gamma = torch.rand(C, generator=g, device=DEV) + 0.5
    mean, invstd = torch.randn(C, generator=g, device=DEV), torch.rand(C, generator=g, device=DEV) + 0.5
    dg, db, coef = native().bn_bwd_coef(part, gamma, mean, invstd, R)
    sd, sx = part[0].double().sum(0), part[1].double().sum(0)
    torch.testing.assert_close(db.double(), sd, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(dg.double(), sx, rtol=1e-5, atol=1e-3)
    k = gamma.double() * invstd.double()
    torch.testing.assert_close(coef[:C].double(), k, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(coef[C:2 * C].double(), -k * invstd.double() * sx / R, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(coef[2 * C:].double(), -k * sd / R + k * invstd.double() * (sx / R) * mean.double(),
                               rtol=1e-4, atol=1e-6)
    for _ in range(3):  # counters reset: repeated calls agree bitwise
        dg2, db2, coef2 = native().bn_bwd_coef(part, gamma, mean, invstd, R)
        assert torch.equal(dg2, dg) and torch.equal(db2, db) and torch.equal(coef2, coef)


def test_fin2_strided_epilogue9_slabs():
    """Slabs 0 and 2 of a [3, G, C] part (the epilogue-9 view) reach the finalize without a copy."""
    G, C = 1568, 1024
    p3, g = _part(G, C, 5)
    p3 = torch.cat([p3, p3[:1] * 0.5])
    view = p3[0::2]
    R = G * 128
    gamma = torch.rand(C, generator=g, device=DEV) + 0.5
    mean, invstd = torch.randn(C, generator=g, device=DEV), torch.rand(C, generator=g, device=DEV) + 0.5
    dg, db, _ = native().bn_bwd_coef(view, gamma, mean, invstd, R)
    torch.testing.assert_close(db.double(), p3[0].double().sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(dg.double(), p3[2].double().sum(0), rtol=1e-5, atol=1e-3)
