"""PsLinear (ops/linear.py): the weight gradient written into a bound destination view is
adopted by autograd as ``p.grad`` (same storage, no copy) and equals nn.Linear's gradient; a
second use of the weight in one graph and a second backward still give nn.Linear's gradients."""
import torch
import torch.nn as nn

from ps_amd.ops.linear import GradDst, PsLinear


def _pair(seed=0):
    torch.manual_seed(seed)
    ref = nn.Linear(16, 8, bias=False)
    lin = PsLinear(16, 8, bias=False)
    lin.weight.data.copy_(ref.weight.data)
    return ref, lin


def test_weight_grad_lands_in_bound_view():
    ref, lin = _pair()
    buf = torch.zeros(300)
    lin.weight._ps_gdst = GradDst(buf, 100, 128, (8, 16))
    x = torch.randn(3, 5, 16, requires_grad=True)
    x2 = x.detach().clone().requires_grad_()
    ref(x2).square().sum().backward()
    lin(x).square().sum().backward()
    assert lin.weight.grad.data_ptr() == buf[100:].data_ptr()  # adopted, not cloned
    torch.testing.assert_close(lin.weight.grad, ref.weight.grad)
    torch.testing.assert_close(buf[100:228].view(8, 16), ref.weight.grad)
    torch.testing.assert_close(x.grad, x2.grad)
    assert buf[:100].abs().sum() == 0 and buf[228:].abs().sum() == 0


def test_second_use_and_accumulation_fall_back_and_add():
    ref, lin = _pair(1)
    buf = torch.zeros(128)
    lin.weight._ps_gdst = GradDst(buf, 0, 128, (8, 16))
    x = torch.randn(4, 16)
    (lin(x) + lin(2 * x)).sum().backward()  # two uses of the weight in one graph
    (ref(x) + ref(2 * x)).sum().backward()
    torch.testing.assert_close(lin.weight.grad, ref.weight.grad)
    lin(x).sum().backward()  # gradient accumulation: adds into the landed view
    ref(x).sum().backward()
    torch.testing.assert_close(lin.weight.grad, ref.weight.grad)
    # (two uses in one graph: autograd sums the two contributions before adopting, so p.grad may
    # be a fresh tensor -- the bucket landing then copies it, exactly as without PsLinear)


def test_unbound_is_plain_linear():
    ref, lin = _pair(2)
    x = torch.randn(6, 16)
    torch.testing.assert_close(lin(x), ref(x))
    lin(x).sum().backward()
    ref(x).sum().backward()
    torch.testing.assert_close(lin.weight.grad, ref.weight.grad)
