"""Fused NHWC BatchNorm(+residual)+ReLU HIP kernels vs a plain torch fp32 reference."""
import pytest
import torch
import torch.nn.functional as F

from ps_amd.ops.bn import BatchNormAct2d, bn_act

pytestmark = pytest.mark.gpu


def _ref(x, res, w, b, rm, rv, training, act):
    y = F.batch_norm(x.float(), rm, rv, w, b, training, 0.1, 1e-5)
    if res is not None:
        y = y + res.float()
    return torch.relu(y) if act == "relu" else y


@pytest.mark.parametrize("C,H", [(64, 14), (136, 7), (2048, 7), (256, 28)])
@pytest.mark.parametrize("act", ["relu", "none"])
@pytest.mark.parametrize("with_res", [False, True])
def test_bn_act_train_fwd_bwd(C, H, act, with_res):
    torch.manual_seed(C + H)
    N = 8
    x = (torch.randn(N, C, H, H) * 2 + 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
    res = torch.randn(N, C, H, H).bfloat16().contiguous(memory_format=torch.channels_last) if with_res else None
    w = torch.rand(C) + 0.5
    b = torch.randn(C) * 0.1
    dy = torch.randn(N, C, H, H).bfloat16().contiguous(memory_format=torch.channels_last)
    # reference (fp32 on CPU)
    xr = x.float().requires_grad_()
    rr = res.float().requires_grad_() if with_res else None
    wr, br = w.clone().requires_grad_(), b.clone().requires_grad_()
    rm, rv = torch.zeros(C), torch.ones(C)
    yr = _ref(xr, rr, wr, br, rm, rv, True, act)
    yr.backward(dy.float())
    # HIP
    xg = x.cuda().requires_grad_()
    rg = res.cuda().requires_grad_() if with_res else None
    wg, bg = w.cuda().requires_grad_(), b.cuda().requires_grad_()
    rmg, rvg = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    yg = bn_act(xg, wg, bg, rmg, rvg, True, 0.1, 1e-5, act, rg)
    assert yg.is_contiguous(memory_format=torch.channels_last)
    yg.backward(dy.cuda())
    torch.cuda.synchronize()
    torch.testing.assert_close(yg.float().cpu(), yr.detach(), rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(rmg.cpu(), rm, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rvg.cpu(), rv, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(xg.grad.float().cpu(), xr.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(wg.grad.cpu(), wr.grad, rtol=1e-2, atol=2e-1)
    torch.testing.assert_close(bg.grad.cpu(), br.grad, rtol=1e-2, atol=2e-1)
    if with_res:
        torch.testing.assert_close(rg.grad.float().cpu(), rr.grad, rtol=2e-2, atol=2e-2)


def test_bn_act_eval_mode_and_module():
    C = 128
    m = BatchNormAct2d(C).cuda()
    m.running_mean.normal_()
    m.running_var.uniform_(0.5, 2.0)
    m.eval()
    x = torch.randn(4, C, 8, 8, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = m(x)
    ref = torch.relu(F.batch_norm(x.float(), m.running_mean, m.running_var, m.weight, m.bias, False, 0.1, 1e-5))
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=3e-2)
    m.train()
    m(x)
    assert int(m.num_batches_tracked) == 1


def test_resnet_fused_matches_unfused_gpu():
    """End-to-end: bf16 fused-BN ResNet vs bf16 MIOpen-BN ResNet, both judged against an
    fp32 model -- the fused path must be at least as close to fp32 (per-parameter cosine)."""
    import copy

    from ps_amd.models.resnet import ResNet, prepare_for_mi355x

    torch.manual_seed(0)
    # zero_init_residual would zero every in-block gradient of a 1-block-per-stage net
    a = ResNet((1, 1, 1, 1), 10, zero_init_residual=False, fused_bn=True)
    b = ResNet((1, 1, 1, 1), 10, zero_init_residual=False, fused_bn=False)
    b.load_state_dict(a.state_dict())
    ref = copy.deepcopy(b).cuda().to(memory_format=torch.channels_last)
    a = prepare_for_mi355x(a.cuda())
    b = prepare_for_mi355x(b.cuda())
    x = torch.randn(8, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    ya, yb, yr = a(x), b(x), ref(x.float())
    rel = lambda u: ((u.float() - yr).norm() / yr.norm()).item()  # noqa: E731
    assert rel(ya) < 0.05 and rel(ya) < rel(yb) + 0.01, (rel(ya), rel(yb))
    g = torch.randn_like(yr)
    ya.float().backward(g)
    yb.float().backward(g)
    yr.backward(g)
    cos = torch.nn.functional.cosine_similarity
    for (n, p), (_, q), (_, r) in zip(a.named_parameters(), b.named_parameters(), ref.named_parameters()):
        ca = cos(p.grad.float().reshape(1, -1), r.grad.reshape(1, -1)).item()
        cb = cos(q.grad.float().reshape(1, -1), r.grad.reshape(1, -1)).item()
        assert ca > 0.9 and ca > cb - 0.05, (n, ca, cb)


@pytest.mark.gpu
def test_bn_stats_large_mean_offset():
    """Welford/Chan statistics: |mean| >> std must not lose the variance (E[x^2]-E[x]^2 would)."""
    from ps_amd.ops import native

    torch.manual_seed(0)
    N, H, W, C = 16, 28, 28, 64
    x64 = 50.0 + 0.05 * torch.randn(N, C, H, W, dtype=torch.float64)
    x = x64.cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    xr = x.double()
    g = torch.ones(C, device="cuda")
    b = torch.zeros(C, device="cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    x2 = x.permute(0, 2, 3, 1).reshape(-1, C)  # NHWC rows (a view: channels_last)
    y, mean, invstd, _ = native().bn_act_fwd(x2, None, g, b, rm, rv, True, 0.1, 1e-5, 0)
    mref = xr.mean((0, 2, 3))
    vref = xr.var((0, 2, 3), unbiased=False)
    torch.testing.assert_close(mean.double(), mref, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close((1 / invstd.double() ** 2 - 1e-5), vref, rtol=2e-3, atol=1e-7)


@pytest.mark.gpu
def test_resnet50_full_depth_training_trajectory_vs_fp32():
    """Full ResNet-50 (3, 4, 6, 3): 8 SGD steps of the bf16 production path (fused bottlenecks,
    cross-block bn3 fold, HIP stem / BN / pool, co-located PS with the fused HIP momentum kernel)
    against the same net in fp32 through plain torch modules and torch.optim -- the loss
    trajectories must agree step by step within bf16 tolerance, and both must learn the batch."""
    import copy

    import torch.nn.functional as F

    from ps_amd.models.resnet import prepare_for_mi355x, resnet50
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import MomentumUpdater

    torch.manual_seed(0)
    base = resnet50(num_classes=10, fused_bn=True)
    ref = copy.deepcopy(base)
    for mod in ref.modules():  # the fp32 oracle runs every block module by module
        if hasattr(mod, "fuse_block"):
            mod.fuse_block = False
    ref = ref.cuda().to(memory_format=torch.channels_last)
    net = prepare_for_mi355x(base.cuda())
    ps = ColocatedPS(net, MomentumUpdater(0.05, 0.9, 0.0))
    opt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(32, 3, 112, 112, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,), device="cuda", generator=g)
    la, lr_ = [], []
    for _ in range(8):
        loss = F.cross_entropy(net(x.bfloat16()).float(), y)
        loss.backward()
        ps.finish_step()
        la.append(loss.item())
        opt.zero_grad()
        lref = F.cross_entropy(ref(x), y)
        lref.backward()
        opt.step()
        lr_.append(lref.item())
    for a, b in zip(la, lr_):
        assert abs(a - b) < 0.05 * max(1.0, abs(b)), (la, lr_)
    assert la[-1] < la[0] - 0.5 and lr_[-1] < lr_[0] - 0.5, (la, lr_)
