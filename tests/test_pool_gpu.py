"""NHWC max pool HIP kernels (+ fused stem BN -> ReLU -> pool) vs plain torch fp32 references."""
import pytest
import torch
import torch.nn.functional as F

from ps_amd.ops.bn import BatchNormAct2d
from ps_amd.ops.pool import bn_relu_maxpool, max_pool2d

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,C,H,W,k,s,p", [(2, 64, 112, 112, 3, 2, 1), (3, 16, 9, 7, 2, 2, 0),
                                           (1, 24, 10, 10, 3, 1, 1), (2, 8, 15, 15, 3, 2, 1),
                                           (1, 32, 8, 12, 3, 2, 1), (2, 8, 6, 4, 3, 2, 1)])
def test_maxpool_nhwc_fwd_bwd(N, C, H, W, k, s, p):
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    xr = x.float().detach().requires_grad_(True)
    xh = x.detach().requires_grad_(True)
    y = max_pool2d(xh, k, s, p)
    yr = F.max_pool2d(xr, k, s, p)
    assert torch.equal(y.float(), yr)  # max of bf16 values is exact
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g.bfloat16().float())
    torch.testing.assert_close(xh.grad.float(), xr.grad, rtol=1e-2, atol=1e-2)


def test_bn_relu_maxpool_matches_unfused():
    torch.manual_seed(0)
    N, C, H, W = 4, 64, 56, 56
    x = (torch.randn(N, C, H, W, device="cuda") * 2 + 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
    bn = BatchNormAct2d(C).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    ref = torch.nn.BatchNorm2d(C).cuda()
    ref.load_state_dict(bn.state_dict())
    xh = x.detach().requires_grad_(True)
    xr = x.float().detach().requires_grad_(True)
    y = bn_relu_maxpool(xh, bn, 3, 2, 1)
    yr = F.max_pool2d(torch.relu(ref(xr)), 3, 2, 1)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-3, atol=1e-3)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    cos = torch.nn.functional.cosine_similarity
    assert cos(xh.grad.float().flatten(), xr.grad.flatten(), dim=0) > 0.99
    torch.testing.assert_close(bn.weight.grad, ref.weight.grad, rtol=5e-2, atol=0.5)
    torch.testing.assert_close(bn.bias.grad, ref.bias.grad, rtol=5e-2, atol=0.5)


@pytest.mark.parametrize("ci,co,h", [(256, 64, 14), (1024, 256, 7), (64, 256, 14), (2048, 512, 7)])
def test_conv1x1_routed_matches_conv2d(ci, co, h):
    from ps_amd.ops.conv import Conv1x1

    torch.manual_seed(0)
    m = Conv1x1(ci, co).cuda().bfloat16().to(memory_format=torch.channels_last)
    ref = torch.nn.Conv2d(ci, co, 1, bias=False).cuda()
    ref.weight.data.copy_(m.weight.float())
    x = torch.randn(4, ci, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    xh = x.detach().requires_grad_(True)
    xr = x.float().detach().requires_grad_(True)
    y, yr = m(xh), ref(xr)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g.bfloat16().float())
    torch.testing.assert_close(xh.grad.float(), xr.grad, rtol=2e-2, atol=5e-2)
    cos = torch.nn.functional.cosine_similarity
    assert cos(m.weight.grad.float().flatten(), ref.weight.grad.flatten(), dim=0) > 0.999


@pytest.mark.parametrize("N,H,W", [(2, 224, 224), (3, 30, 46), (1, 17, 9), (2, 256, 256)])
@pytest.mark.parametrize("cin", [3, 4])
def test_stem_conv_fwd_wgrad(N, H, W, cin):
    from ps_amd.ops.conv import StemConv

    torch.manual_seed(0)
    m = StemConv(cin).cuda().bfloat16().to(memory_format=torch.channels_last)
    ref = torch.nn.Conv2d(cin, 64, 7, 2, 3, bias=False).cuda()
    ref.weight.data.copy_(m.weight.float())
    x = torch.randn(N, cin, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = m(x)
    yr = ref(x.float())
    assert y.shape == yr.shape
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=3e-2)
    g = torch.randn_like(yr).bfloat16()
    y.backward(g)
    yr.backward(g.float())
    torch.testing.assert_close(m.weight.grad.float(), ref.weight.grad, rtol=2e-2, atol=2e-2 * ref.weight.grad.abs().max().item())


@pytest.mark.parametrize("N,H", [(4, 64), (2, 224)])
def test_stem_fused_block_matches_unfused(N, H):
    from ps_amd.ops.conv import StemConv, stem_bn_relu_maxpool

    torch.manual_seed(0)
    conv = StemConv(3).cuda().bfloat16().to(memory_format=torch.channels_last)
    bn = BatchNormAct2d(64).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-1, 1)  # the partial-sum shift; must not affect the result
    rconv = torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False).cuda()
    rconv.weight.data.copy_(conv.weight.float())
    rbn = torch.nn.BatchNorm2d(64).cuda()
    rbn.load_state_dict({k: v for k, v in bn.state_dict().items()})
    x = (torch.randn(N, 3, H, H, device="cuda") + 3.0).bfloat16().contiguous(memory_format=torch.channels_last)
    y = stem_bn_relu_maxpool(x, conv, bn)
    yr = F.max_pool2d(torch.relu(rbn(rconv(x.float()))), 3, 2, 1)
    rel = ((y.float() - yr).norm() / yr.norm()).item()
    assert rel < 1e-2, rel
    torch.testing.assert_close(bn.running_mean, rbn.running_mean, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(bn.running_var, rbn.running_var, rtol=1e-2, atol=1e-3)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    cos = torch.nn.functional.cosine_similarity
    for a, b in ((conv.weight.grad, rconv.weight.grad), (bn.weight.grad, rbn.weight.grad),
                 (bn.bias.grad, rbn.bias.grad)):
        assert cos(a.float().flatten(), b.flatten(), dim=0) > 0.99


@pytest.mark.parametrize("H,k,s,p", [(112, 3, 2, 1), (15, 3, 2, 1), (10, 3, 1, 1), (9, 2, 2, 0)])
def test_fused_bn_pool_value_and_first_argmax_exact(H, k, s, p):
    """BN-apply + ReLU + pool kernel vs the unfused semantics: the max of the bf16-rounded
    relu(x * scale + shift) (one fp32 rounding, as the kernel's fma) and the FIRST tap (kh, kw)
    order attaining it -- bitwise, including ties (many zeros after the ReLU)."""
    from ps_amd.ops import native

    torch.manual_seed(1)
    N, C = 2, 16
    x = torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    sc = torch.rand(C, device="cuda") + 0.5
    sh = torch.randn(C, device="cuda") * 0.5
    coef = torch.cat([sc, sh]).float().contiguous()
    xn = x.permute(0, 2, 3, 1).contiguous()
    y, idx = native().maxpool_nhwc_fwd(xn, coef, k, s, p)
    # reference: exact product-sum in fp64 -> one rounding to fp32 (= fma) -> bf16
    a = torch.relu(x.double() * sc.double().view(1, C, 1, 1) + sh.double().view(1, C, 1, 1)).float().bfloat16()
    ap = torch.nn.functional.pad(a.float(), (p, p, p, p), value=-1.0)  # padding never wins (a >= 0)
    cols = torch.nn.functional.unfold(ap, k, stride=s)  # [N, C*k*k, L], tap-major within a channel
    OH = (H + 2 * p - k) // s + 1
    cols = cols.view(N, C, k * k, OH, OH)
    ref = cols.max(dim=2).values
    first = (cols == ref.unsqueeze(2)).float().argmax(dim=2)  # first tap attaining the max
    yk = y.view(N, OH, OH, C).permute(0, 3, 1, 2).float()
    ik = idx.view(N, OH, OH, C).permute(0, 3, 1, 2).long()
    assert torch.equal(yk, ref)
    assert torch.equal(ik, first)


@pytest.mark.parametrize("N,H,C", [(2, 112, 64), (3, 16, 32)])
def test_pool_bn_bwd_fused_matches_unfused(N, H, C):
    """Stem backward with the pool scatter fused into both BN-backward passes (pool.hip
    pool_bn_bwd_kernel) vs the unfused chain maxpool_nhwc_bwd -> bn_act_bwd (relu mask from z):
    the same pool gradient (rounded to bf16 where the unfused path stores it), the same per-channel
    sums up to fp32 summation order -> dz within one bf16 ulp, dgamma / dbeta to 1e-4."""
    from ps_amd.ops import native

    torch.manual_seed(2)
    z = torch.randn(N, H, H, C, device="cuda").bfloat16()
    sc = torch.rand(C, device="cuda") + 0.5
    sh = torch.randn(C, device="cuda") * 0.3
    coef = torch.cat([sc, sh]).float().contiguous()
    zf = z.float()
    mean = zf.mean(dim=(0, 1, 2))
    invstd = 1.0 / (zf.var(dim=(0, 1, 2), unbiased=False) + 1e-5).sqrt()
    gamma = torch.rand(C, device="cuda") + 0.5
    y, idx = native().maxpool_nhwc_fwd(z, coef, 3, 2, 1)
    dy = torch.randn_like(y.float()).bfloat16()
    dz, dg, db = native().pool_bn_bwd(dy, idx, z, coef, gamma, mean, invstd)
    dpool = native().maxpool_nhwc_bwd(dy, idx, H, H, 3, 2, 1)
    dz_ref, _, dg_ref, db_ref = native().bn_act_bwd(dpool.view(-1, C), None, z.view(-1, C), gamma, mean, invstd, 1,
                                                    False, True, coef)
    torch.testing.assert_close(dg, dg_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(db, db_ref, rtol=1e-4, atol=1e-4)
    d = (dz.float() - dz_ref.view_as(dz).float()).abs()
    ulp = dz_ref.view_as(dz).float().abs() * 2.0 ** -7 + 1e-6
    assert bool((d <= ulp).all()), d.max().item()


@pytest.mark.parametrize("N,H,cin", [(2, 224, 3), (3, 64, 4), (2, 40, 3)])
def test_stem_bwd_fused_matches_apply_then_wgrad(N, H, cin):
    """Stem backward with the BN apply inside the weight gradient (stem.hip FUSED: each dz row is
    rebuilt from the pooled gradient, argmax and z) vs the apply pass writing dz + the plain weight
    gradient: dz is computed with the same arithmetic and accumulated in the same order, so the
    packed weight gradient matches to fp32 rounding and dgamma / dbeta exactly."""
    from ps_amd.ops import native
    from ps_amd.ops.conv import nhwc_in

    torch.manual_seed(5)
    x = torch.randn(N, cin, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    xin = nhwc_in(x)
    OH = (H - 1) // 2 + 1
    z = torch.randn(N, OH, OH, 64, device="cuda").bfloat16()
    coef = torch.cat([torch.rand(64, device="cuda") + 0.5, torch.randn(64, device="cuda") * 0.3]).float().contiguous()
    zf = z.float()
    mean = zf.mean(dim=(0, 1, 2))
    invstd = 1.0 / (zf.var(dim=(0, 1, 2), unbiased=False) + 1e-5).sqrt()
    gamma = torch.rand(64, device="cuda") + 0.5
    y, idx = native().maxpool_nhwc_fwd(z, coef, 3, 2, 1)
    dy = torch.randn_like(y.float()).bfloat16()
    dz, dg_ref, db_ref = native().pool_bn_bwd(dy, idx, z, coef, gamma, mean, invstd)
    dw_ref = native().stem_conv_wrw(xin, dz)
    dw, dg, db = native().stem_bwd_fused(xin, dy, idx, z, coef, gamma, mean, invstd)
    torch.cuda.synchronize()
    assert torch.equal(dg, dg_ref) and torch.equal(db, db_ref)
    torch.testing.assert_close(dw, dw_ref, rtol=1e-5, atol=1e-5 * dw_ref.abs().max().item())
