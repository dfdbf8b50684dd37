"""Fused FC layer (K2, layer/FcLayer.java:74-110) on MFMA vs fp32 torch autograd: forward with
bias + activation epilogue, backward with act' in the GEMM prologue and db from the staged tile,
fp32 (v_mfma_f32_16x16x4_f32) and bf16 operands, the reference-scale shapes incl. the 275-wide
CTR concat (TestJcublas) and MNIST 784 / CNN 1568 widths, and the fp32 reference models routed
through it on the GPU."""
import pytest
import torch
import torch.nn.functional as F

from ps_amd.ops import dense as D

pytestmark = pytest.mark.gpu
DEV = "cuda"
SHAPES = [(1000, 275, 150), (1000, 784, 150), (100, 1568, 150), (1000, 150, 50), (1000, 50, 10), (1000, 10, 1),
          (37, 275, 275)]


def _ref(x, w, b, act):
    from ps_amd.models.activations import _ClippedSigmoid  # reference backward dy * y * (1 - y)

    z = F.linear(x, w, b)
    if act == 3:
        return _ClippedSigmoid.apply(z)
    return {0: z, 1: torch.relu(z), 2: F.leaky_relu(z, 0.01)}[act]


@pytest.mark.parametrize("m,k,n", SHAPES)
@pytest.mark.parametrize("act", [0, 1, 2, 3])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fused_linear_fwd_bwd(m, k, n, act, dtype):
    g = torch.Generator().manual_seed(m + k + n + act)
    x = torch.randn(m, k, generator=g)
    w = torch.randn(n, k, generator=g) * (1.0 / k ** 0.5)
    b = torch.randn(n, generator=g) * 0.1
    dy = torch.randn(m, n, generator=g)
    # fp32 oracle on the same (rounded) inputs
    xr, wr, br = (t.to(dtype).float().clone().requires_grad_() for t in (x, w, b))
    yr = _ref(xr, wr, br, act)
    yr.backward(dy.to(dtype).float())
    xg, wg = x.detach().to(DEV, dtype).requires_grad_(), w.detach().to(DEV, dtype).requires_grad_()
    bg = b.detach().to(DEV, dtype).requires_grad_()
    y = D.linear_act(xg, wg, bg, act)
    y.backward(dy.to(DEV, dtype))
    tol = dict(rtol=2e-4, atol=2e-4) if dtype == torch.float32 else dict(rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(y.float().cpu(), yr.detach(), **tol)
    scale = max(1.0, float(xr.grad.abs().max()))
    torch.testing.assert_close(xg.grad.float().cpu() / scale, xr.grad / scale, **tol)
    scale = max(1.0, float(wr.grad.abs().max()))
    torch.testing.assert_close(wg.grad.float().cpu() / scale, wr.grad / scale, **tol)
    scale = max(1.0, float(br.grad.abs().max()))
    torch.testing.assert_close(bg.grad.float().cpu() / scale, br.grad / scale, **tol)


def test_fp32_reference_mlp_on_gpu_matches_cpu():
    from ps_amd.context import ctx
    from ps_amd.models.reference import FullConnectedNN
    from ps_amd.train.trainer import CollectiveEngine, Trainer

    g = torch.Generator().manual_seed(0)
    x = torch.rand(200, 784, generator=g) * 255
    y = torch.randint(0, 10, (200,), generator=g)
    out = []
    for dev in ("cpu", DEV):
        ctx.init()
        m = FullConnectedNN.build_model(784, [150, 50, 10], gen=torch.Generator().manual_seed(1)).to(dev)
        tr = Trainer(m, CollectiveEngine(m), device=dev)
        for i in range(5):
            tr.train([{"X": x[i * 40:(i + 1) * 40], "Y": y[i * 40:(i + 1) * 40]}])
        tr.engine.synchronize()
        out.append({k: v.detach().cpu() for k, v in m.named_parameters()})
    for k in out[0]:
        torch.testing.assert_close(out[1][k], out[0][k], rtol=1e-3, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("c,k_out,hw,act", [(1, 16, 28, "relu"), (16, 32, 14, "relu"), (3, 8, 9, "none")])
def test_reference_conv_on_inhouse_kernels_vs_fp32_conv2d(c, k_out, hw, act):
    """CnnMnist convs (CNN.java:37-49) on the GPU default path: HIP im2col -> fp32 MFMA fused
    linear (bias + ReLU epilogue) -> K2 backward -> HIP col2im, vs fp32 F.conv2d autograd."""
    from ps_amd.models import activations as A
    from ps_amd.models.layers import Conv2DLayer

    torch.manual_seed(0)
    layer = Conv2DLayer("conv", hw, hw, c, 3, 1, k_out, padding=1,
                        activation=A.Relu() if act == "relu" else None).cuda()
    x = torch.randn(32, c * hw * hw, device="cuda", requires_grad=True)
    y = layer(x)
    w, b = layer.weights.detach().clone().requires_grad_(), layer.bias.detach().clone().requires_grad_()
    xr = x.detach().clone().requires_grad_()
    yr = torch.nn.functional.conv2d(xr.view(32, c, hw, hw), w, b, 1, 1)
    if act == "relu":
        yr = torch.relu(yr)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(layer.weights.grad, w.grad, rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(layer.bias.grad, b.grad, rtol=1e-4, atol=2e-3)
