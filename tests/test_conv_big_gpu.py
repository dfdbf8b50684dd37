"""256 x 256-tile conv GEMM (csrc/kernels/conv_big.hip: deep-K 1x1 convolutions, epilogues 0 / 1 / 3,
stride 1 and the stride-2 downsample gather) vs plain-torch fp32 references of the same op.

Shapes are chosen so the planner routes them to the big tiles (>= 1024 blocks, or K >= 1024 with
>= 256 blocks; checked through conv_gemm_plan) with partial last pixel tiles."""
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


@pytest.mark.parametrize("M,K,N", [(262213, 256, 256), (33001, 1024, 512), (16411, 2048, 1024)])
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
    n, h, K, N = 700, 14, 1024, 512
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


def _coef(k, g):
    return torch.cat([torch.rand(k, generator=g, device=DEV) + 0.5, torch.randn(k, generator=g, device=DEV) * 0.5])


def test_big_tile_bn_relu_prologue():
    """PRO 1: relu(bf16(a sc + sh)) applied by the in-LDS pass over each stage."""
    M, K, N = 33001, 1024, 512
    g = _gen(21)
    a, b = _rnd(M, K, g=g), _rnd(N, K, g=g, scale=K ** -0.5)
    coef = _coef(K, g)
    gg = [M, 1, M, 1, 1, 1, 0]
    bm, bn, _ = native().conv_gemm_plan(M, N, K, gg, True, 1, 0)
    assert (bm, bn) == (256, 256)
    ks = torch.zeros(N, device=DEV)
    c, part = native().conv_gemm(a, b, gg, coef, 1, None, ks)
    x = torch.relu((a.float() * coef[:K] + coef[K:]).bfloat16().float())
    _close(c, x @ b.float().t())
    torch.testing.assert_close(part[0].sum(0), c.float().sum(0), rtol=1e-4, atol=5e-2)


def test_big_tile_bn_backward_prologue_stores_dz():
    """PRO 2: dz = bf16(ca g + cb z + cc) from two row sources, stored once (channel tile 0) and fed
    to the data-gradient GEMM with epilogue 3 -- vs the apply pass + the same GEMM."""
    M, K, N = 33001, 1024, 512
    g = _gen(22)
    d, z = _rnd(M, K, g=g), _rnd(M, K, g=g)
    b = _rnd(N, K, g=g, scale=K ** -0.5)
    cb = torch.cat([torch.rand(K, generator=g, device=DEV) + 0.5, torch.randn(K, generator=g, device=DEV) * 0.1,
                    torch.randn(K, generator=g, device=DEV) * 0.1])
    z2 = _rnd(M, N, g=g)
    mc = _coef(N, g)
    m2, i2 = torch.randn(N, generator=g, device=DEV) * 0.1, torch.rand(N, generator=g, device=DEV) + 0.5
    gg = [M, 1, M, 1, 1, 1, 0]
    bm, bn, _ = native().conv_gemm_plan(M, N, K, gg, True, 3, 2)
    assert (bm, bn) == (256, 256)
    c, part, dz = native().conv_gemm(d, b, gg, None, 3, z2, None, mc, m2, i2, a2=z, bwd=cb)
    dz_ref = (cb[:K] * d.float() + cb[K:2 * K] * z.float() + cb[2 * K:]).bfloat16()
    assert (dz != dz_ref).float().mean().item() < 1e-2  # FMA contraction may differ by one ulp
    torch.testing.assert_close(dz.float(), dz_ref.float(), rtol=8e-3, atol=1e-3)
    mask = (z2.float() * mc[:N] + mc[N:]) > 0
    _close(c, (dz_ref.float() @ b.float().t()) * mask)
    cg = c.float()
    torch.testing.assert_close(part[0].sum(0), cg.sum(0), rtol=1e-4, atol=5e-2)
    torch.testing.assert_close(part[1].sum(0), (cg * ((z2.float() - m2) * i2)).sum(0), rtol=1e-3, atol=5e-2)


@pytest.mark.parametrize("dual", [False, True])
def test_big_tile_block_output_prologue(dual):
    """PRO 3: the previous block's output relu(z3 sc + sh + r) (r = the residual rows, or dual: the
    downsample BN's output) built while staging, stored with its ReLU bits, then the GEMM."""
    M, K, N = 33001, 1024, 512
    g = _gen(23 + dual)
    z3, r = _rnd(M, K, g=g), _rnd(M, K, g=g)
    b = _rnd(N, K, g=g, scale=K ** -0.5)
    cf3, cfd = _coef(K, g), _coef(K, g)
    gg = [M, 1, M, 1, 1, 1, 0]
    bm, bn, _ = native().conv_gemm_plan(M, N, K, gg, True, 1, 1)
    assert (bm, bn) == (256, 256)
    out = torch.empty(M, K, device=DEV, dtype=torch.bfloat16)
    bits = torch.empty(M * K // 8, device=DEV, dtype=torch.uint8)
    ks = torch.zeros(N, device=DEV)
    c, part = native().conv_gemm(z3, b, gg, cf3, 1, None, ks, a2=r, pro2=cfd if dual else None, aout=out, abits=bits)
    res = (r.float() * cfd[:K] + cfd[K:]) if dual else r.float()
    y = torch.relu(z3.float() * cf3[:K] + cf3[K:] + res).bfloat16()
    assert (out != y).float().mean().item() < 1e-2
    torch.testing.assert_close(out.float(), y.float(), rtol=8e-3, atol=1e-3)
    want_bits = ((out.float() > 0).view(-1, 8).int() << torch.arange(8, device=DEV)).sum(1).to(torch.uint8)
    assert torch.equal(bits, want_bits)
    _close(c, y.float() @ b.float().t())
    torch.testing.assert_close(part[0].sum(0), c.float().sum(0), rtol=1e-4, atol=5e-2)


def test_layer3_chain_on_big_tiles_matches_module_path():
    """Two layer-3 bottlenecks (1024 -> 256 -> 1024, 14 x 14) at a batch where the block-output,
    BN + ReLU and BN-backward prologues all run on the 256 x 256 tiles.  Against an fp32 run of the
    module path: at this depth bf16 rounding (ReLU-mask flips through two BN backwards) moves the
    input gradient by ~12 % for EVERY bf16 path (scripts/debug_big_chain.py), so the fused path is
    held to the bf16 module path's own error, not to a fixed tolerance."""
    import copy

    import torch.nn as nn

    from ps_amd.models.resnet import Bottleneck, prepare_for_mi355x
    from ps_amd.ops import convgemm as cg

    torch.manual_seed(4)
    n, h = 400, 14
    M = n * h * h
    assert cg.big_tile(M, 256, 1024, src2=1) and cg.big_tile(M, 256, 1024, src2=2, epi=3)
    assert cg.big_tile(M, 1024, 256, pro=True)
    a = nn.Sequential(Bottleneck(1024, 256), Bottleneck(1024, 256))
    for m in a.modules():
        if isinstance(m, nn.BatchNorm2d):
            nn.init.uniform_(m.weight, 0.5, 1.5)
            nn.init.uniform_(m.bias, -0.2, 0.2)
    b, f = copy.deepcopy(a), copy.deepcopy(a)
    for blk in list(b) + list(f):
        blk.fuse_block = False
    a, b, f = prepare_for_mi355x(a.cuda()), prepare_for_mi355x(b.cuda()), f.cuda()
    x = torch.randn(n, 1024, h, h, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    xa, xb, xf = x.clone().requires_grad_(), x.clone().requires_grad_(), x.float().requires_grad_()
    r0, u0 = cg.FOLD_STATS["resp"], cg.FOLD_STATS["used"]
    with cg.deferred_bn_counters():
        a[0]._defer_out = True
        ya = a(xa)
    assert cg.FOLD_STATS["resp"] - r0 == 1
    yb, yf = b(xb), f(xf)
    gout = torch.randn(yf.shape, device=DEV).bfloat16()
    ya.backward(gout.contiguous(memory_format=torch.channels_last))
    yb.backward(gout.contiguous(memory_format=torch.channels_last))
    yf.backward(gout.float().contiguous(memory_format=torch.channels_last))
    assert cg.FOLD_STATS["used"] - u0 == 1  # block 0's bn3 backward: the consumer's sums + BWD prologue

    def rel(u, v):
        return ((u.float() - v.float()).norm() / v.float().norm().clamp_min(1e-12)).item()

    pairs = [("y", ya.detach(), yb.detach(), yf.detach()), ("dx", xa.grad, xb.grad, xf.grad)]
    pairs += [(nm, p.grad, q.grad, r.grad) for (nm, p), (_, q), (_, r) in
              zip(a.named_parameters(), b.named_parameters(), f.named_parameters())]
    for nm, u, v, w in pairs:
        ef, eb = rel(u, w), rel(v, w)
        assert ef <= 1.25 * eb + 5e-3, (nm, ef, eb)


def _unpack(bits, M, N):
    return ((bits.view(-1, 1).int() >> torch.arange(8, device=DEV)) & 1).view(M, N).bool()


@pytest.mark.parametrize("epi", [2, 4, 5, 6, 7, 8, 9])
def test_big_tile_residual_and_fold_epilogues(epi):
    """The conv1 data-gradient epilogues on the 256 x 256 tiles: + residual rows (2), + the stride-2
    residual map at even (h, w) (4), + residual masked by the block output's bits (5); 6-8 = 5 / 2 / 4
    then the previous block's ReLU mask (bits2) and its bn3 backward sums, 9 = 6 + the downsample
    BN's sum (third partial slab)."""
    n, h, K, N = 700, 14, 256, 512
    M = n * h * h
    g = _gen(40 + epi)
    a, b = _rnd(M, K, g=g), _rnd(N, K, g=g, scale=K ** -0.5)
    gg = geo(h, h)
    _assert_big(M, N, K, gg, epi)
    base = {6: 5, 9: 5, 7: 2, 8: 4}.get(epi, epi)
    ref = (a.float() @ b.float().t()).bfloat16().float()
    kw = {}
    if base == 4:
        r = (h + 1) // 2
        aux = _rnd(n * r * r, N, g=g)
        full = torch.zeros(n, h, h, N, device=DEV)
        full[:, ::2, ::2] = aux.float().view(n, r, r, N)
        want = ref + full.view(M, N)
    else:
        aux = _rnd(M, N, g=g)
        want = ref + aux.float()
    if base == 5:
        bits = torch.randint(0, 256, (M * N // 8,), generator=g, device=DEV, dtype=torch.uint8)
        kw["bits"] = bits
        want = torch.where(_unpack(bits, M, N), want, ref)
    if epi >= 6:
        z3 = _rnd(M, N, g=g)
        bits2 = torch.randint(0, 256, (M * N // 8,), generator=g, device=DEV, dtype=torch.uint8)
        mean, invstd = torch.randn(N, generator=g, device=DEV) * 0.1, torch.rand(N, generator=g, device=DEV) + 0.5
        kw.update(aux2=z3, bits2=bits2, mean=mean, invstd=invstd)
        want = want * _unpack(bits2, M, N)
    if epi == 9:
        zd = _rnd(M, N, g=g)
        m2, i2 = torch.randn(N, generator=g, device=DEV) * 0.1, torch.rand(N, generator=g, device=DEV) + 0.5
        kw.update(aux3=zd, mean2=m2, invstd2=i2)
    c, part = native().conv_gemm(a, b, gg, None, epi, aux, **kw)
    _close(c, want)
    if epi < 6:
        assert part is None or part.numel() == 0
        return
    assert part.shape == (3 if epi == 9 else 2, (M + 255) // 256, N)
    cg = c.float()
    torch.testing.assert_close(part[0].sum(0), cg.sum(0), rtol=1e-4, atol=5e-2)
    torch.testing.assert_close(part[1].sum(0), (cg * ((z3.float() - mean) * invstd)).sum(0), rtol=1e-3, atol=5e-2)
    if epi == 9:
        torch.testing.assert_close(part[2].sum(0), (cg * ((zd.float() - m2) * i2)).sum(0), rtol=1e-3, atol=5e-2)
