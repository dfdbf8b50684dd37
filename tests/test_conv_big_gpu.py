"""256 x 256-tile conv GEMM (csrc/kernels/conv_big.hip: deep-K 1x1 convolutions, epilogues 0 / 1 / 3,
stride 1 and the stride-2 downsample gather) vs plain-torch fp32 references of the same op.

Shapes are chosen so the planner routes them to the big tiles (>= 256 blocks; checked through
conv_gemm_plan) with partial last pixel tiles."""
import pytest
import torch

from ps_amd.ops import native
from ps_amd.ops.convgemm import geo

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rnd(*shape, g, scale=1.0):
    return (torch.randn(*shape, generator=g, device=DEV) * scale).bfloat16()


def _close(out, ref, tol=1e-2, amax=0.05):
    out, ref = out.float(), ref.float()
    err = ((out - ref).norm() / ref.norm().clamp_min(1e-12)).item()
    assert err < tol, f"relative error {err:.3g}"
    assert (out - ref).abs().max().item() <= amax * ref.abs().max().item() + 1e-3


def _gen(seed):
    return torch.Generator(device=DEV).manual_seed(seed)


def _assert_big(M, N, C, gg, epi):
    bm, bn, gm = native().conv_gemm_plan(M, N, C, gg, False, epi)
    assert (bm, bn) == (256, 256) and gm == (M + 255) // 256, (bm, bn, gm)


@pytest.mark.parametrize("M,K,N", [(65613, 256, 256), (33001, 1024, 512), (16411, 2048, 1024)])
@pytest.mark.parametrize("epi", [0, 1, 3])
def test_big_tile_1x1_epilogues(M, K, N, epi):
    g = _gen(M + K + N + epi)
    a, b = _rnd(M, K, g=g), _rnd(N, K, g=g, scale=K ** -0.5)
    gg = [M, 1, M, 1, 1, 1, 0]
    _assert_big(M, N, K, gg, epi)
    ref = a.float() @ b.float().t()
    if epi == 0:
        c, part = native().conv_gemm(a, b, gg)
        _close(c, ref)
        return
    if epi == 1:
        kshift = torch.randn(N, generator=g, device=DEV) * 0.1
        c, part = native().conv_gemm(a, b, gg, None, 1, None, kshift)
        _close(c, ref)
        cb = c.float() - kshift
        torch.testing.assert_close(part[0].sum(0), cb.sum(0), rtol=1e-4, atol=5e-2)
        torch.testing.assert_close(part[1].sum(0), (cb * cb).sum(0), rtol=1e-4, atol=5e-2)
        return
    z = _rnd(M, N, g=g)
    mc = torch.cat([torch.rand(N, generator=g, device=DEV) + 0.5, torch.randn(N, generator=g, device=DEV) * 0.5])
    mean, invstd = torch.randn(N, generator=g, device=DEV) * 0.1, torch.rand(N, generator=g, device=DEV) + 0.5
    c, part = native().conv_gemm(a, b, gg, None, 3, z, None, mc, mean, invstd)
    mask = (z.float() * mc[:N] + mc[N:]) > 0
    _close(c, ref * mask)
    cg = c.float()
    torch.testing.assert_close(part[0].sum(0), cg.sum(0), rtol=1e-4, atol=5e-2)
    torch.testing.assert_close(part[1].sum(0), (cg * ((z.float() - mean) * invstd)).sum(0), rtol=1e-3, atol=5e-2)


def test_big_tile_stride2_downsample_gather():
    n, h, K, N = 700, 14, 512, 512
    g = _gen(11)
    a, b = _rnd(n * h * h, K, g=g), _rnd(N, K, g=g, scale=K ** -0.5)
    gg = geo(h, h, 1, 2)
    M = n * gg[2] * gg[3]
    _assert_big(M, N, K, gg, 1)
    kshift = torch.zeros(N, device=DEV)
    c, part = native().conv_gemm(a, b, gg, None, 1, None, kshift)
    ref = a.view(n, h, h, K)[:, ::2, ::2].reshape(-1, K).float() @ b.float().t()
    _close(c, ref)
    torch.testing.assert_close(part[0].sum(0), c.float().sum(0), rtol=1e-4, atol=5e-2)


def test_big_tile_deterministic():
    M, K, N = 33001, 1024, 512
    g = _gen(3)
    a, b = _rnd(M, K, g=g), _rnd(N, K, g=g, scale=K ** -0.5)
    ks = torch.zeros(N, device=DEV)
    c1, p1 = native().conv_gemm(a, b, [M, 1, M, 1, 1, 1, 0], None, 1, None, ks)
    c2, p2 = native().conv_gemm(a, b, [M, 1, M, 1, 1, 1, 0], None, 1, None, ks)
    assert torch.equal(c1, c2) and torch.equal(p1, p2)
