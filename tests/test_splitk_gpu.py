"""Split-K weight gradient of the BERT Linears (ops/dense.py linear_wgrad / SplitKLinear, on the
wide-tile kernel of csrc/kernels/convgemm.hip) vs an fp32 torch reference."""
import pytest
import torch

from ps_amd.ops.dense import SplitKLinear, _wgrad_ok, linear_wgrad

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("T,K,N", [(8192, 768, 2304), (4100, 768, 768), (6000, 3072, 768), (5000, 768, 3072)])
def test_linear_wgrad_split_k(T, K, N):
    g = torch.Generator().manual_seed(T + K + N)
    x = torch.randn(T, K, generator=g).bfloat16().to(DEV)
    dy = torch.randn(T, N, generator=g).bfloat16().to(DEV)
    assert _wgrad_ok(x, dy)
    dw = linear_wgrad(dy, x)
    assert dw.shape == (N, K) and dw.dtype == torch.bfloat16
    assert _rel(dw, dy.float().t() @ x.float()) < 5e-3


@pytest.mark.parametrize("T,K,N", [(8192, 768, 2304), (4100, 768, 768), (5000, 3072, 768)])
def test_linear_wgrad_with_fused_bias_grad(T, K, N):
    from ps_amd.ops import native

    g = torch.Generator().manual_seed(T + 3 * K + N)
    x = torch.randn(T, K, generator=g).bfloat16().to(DEV)
    dy = torch.randn(T, N, generator=g).bfloat16().to(DEV)
    dw, db = native().linear_wgrad_db(dy, x)
    assert _rel(dw, dy.float().t() @ x.float()) < 5e-3
    torch.testing.assert_close(db, dy.float().sum(0), rtol=1e-4, atol=1e-2)


def test_splitk_linear_module_matches_linear():
    torch.manual_seed(0)
    a = SplitKLinear(768, 2304).to(DEV).bfloat16()
    b = torch.nn.Linear(768, 2304).to(DEV).bfloat16()
    b.load_state_dict(a.state_dict())
    x = torch.randn(2, 4096, 768, device=DEV).bfloat16()
    dy = torch.randn(2, 4096, 2304, device=DEV).bfloat16()
    xa, xb = x.clone().requires_grad_(), x.clone().requires_grad_()
    ya, yb = a(xa), b(xb)
    assert torch.equal(ya, yb)
    ya.backward(dy)
    yb.backward(dy)
    assert _rel(xa.grad, xb.grad) < 1e-2
    assert _rel(a.weight.grad, b.weight.grad) < 1e-2
    assert _rel(a.bias.grad, b.bias.grad) < 1e-2


@pytest.mark.parametrize("T,K,N", [(65536, 512, 256), (8192, 256, 1024), (1000, 64, 32)])
def test_splitk_linear_fused_relu_matches_linear_relu(T, K, N):
    """SplitKLinear(fuse_relu): bias + ReLU in the GEMM epilogue, ReLU' before the split-K weight
    gradient -- vs nn.Linear + ReLU in fp32 (forward, dx, dW, db)."""
    from ps_amd.ops.dense import SplitKLinear

    torch.manual_seed(T + K)
    lin = SplitKLinear(K, N).cuda().bfloat16()
    lin.fuse_relu = True
    ref = torch.nn.Linear(K, N).cuda()
    ref.weight.data.copy_(lin.weight.data.float())
    ref.bias.data.copy_(lin.bias.data.float())
    x = torch.randn(T, K, device="cuda").bfloat16().requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    y = lin(x)
    yr = torch.relu(ref(xr))
    g = torch.randn(T, N, device="cuda").bfloat16()
    y.backward(g)
    yr.backward(g.float())

    def rel(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()

    assert rel(y, yr) < 1e-2
    assert rel(x.grad, xr.grad) < 2e-2
    assert rel(lin.weight.grad, ref.weight.grad) < 2e-2
    assert rel(lin.bias.grad, ref.bias.grad) < 2e-2


def test_splitk_linear_fork_folds_residual_grad():
    """SplitKLinear.fork: (x W^T + b, x) with the residual gradient added inside the data-gradient
    GEMM -- vs nn.Linear + a residual use of x in fp32."""
    from ps_amd.ops.dense import SplitKLinear

    torch.manual_seed(7)
    T, K, N = 8192, 768, 2304
    lin = SplitKLinear(K, N).cuda().bfloat16()
    ref = torch.nn.Linear(K, N).cuda()
    ref.weight.data.copy_(lin.weight.data.float())
    ref.bias.data.copy_(lin.bias.data.float())
    x = torch.randn(T, K, device="cuda").bfloat16().requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    y, xp = lin.fork(x)
    yr = ref(xr)
    gy, gx = torch.randn(T, N, device="cuda").bfloat16(), torch.randn(T, K, device="cuda").bfloat16()
    (y.float() * gy.float()).sum().add_((xp.float() * gx.float()).sum()).backward()
    ((yr * gy.float()).sum() + (xr * gx.float()).sum()).backward()
    assert _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(lin.weight.grad, ref.weight.grad) < 2e-2
    assert _rel(lin.bias.grad, ref.bias.grad) < 2e-2
