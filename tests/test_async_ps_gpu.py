"""Asynchronous parameter server on the MI355X: native GPU progress thread (fused HIP
optimizer into published slots), completion notifier, and -- between two real processes on
cuda:0 -- CUDA-IPC-mapped mailboxes / slots (the one-node xGMI data plane of async_ps.py)."""
import pytest
import torch
import torch.nn.functional as F

from ps_amd.parallel.transport import run_loopback

from . import dist_util

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _model(dtype=torch.float32):
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.Tanh(), torch.nn.Linear(64, 4)).to(DEV, dtype)


def _data(n=64):
    g = torch.Generator().manual_seed(3)
    return torch.randn(n, 32, generator=g).to(DEV), torch.randint(0, 4, (n,), generator=g).to(DEV)


def _body(tp, staleness, steps, lr, models=None, adam=False):
    from ps_amd.parallel.async_ps import AsyncPS
    from ps_amd.parallel.updaters import AdamUpdater, SimpleUpdater

    torch.cuda.set_device(0)
    m = models[tp.rank] if models is not None else _model()
    upd = AdamUpdater(1e-2, bias_correction="step") if adam else SimpleUpdater(lr)
    ps = AsyncPS(m, upd, tp, staleness=staleness, timeout_s=60)
    x, y = _data()
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    losses = []
    for _ in range(steps):
        loss = F.cross_entropy(m(xs.to(m[0].weight.dtype)).float(), ys)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    ps.synchronize()
    tp.barrier()
    ps.refresh()
    out = {n: p.detach().float().cpu().clone() for n, p in m.named_parameters()}
    ps.close()
    return out, losses


def _oracle(world, steps, lr):
    ref = _model()
    opt = torch.optim.SGD(ref.parameters(), lr=lr)
    x, y = _data()
    for _ in range(steps):
        opt.zero_grad()
        (sum(F.cross_entropy(ref(x[r::world]), y[r::world]) for r in range(world)) / world).backward()
        opt.step()
    return {n: p.detach().cpu() for n, p in ref.named_parameters()}


def test_single_worker_gpu_server_is_plain_sgd():
    res = run_loopback(_body, 1, 0, 6, 0.2, [_model()])
    for k, v in _oracle(1, 6, 0.2).items():
        torch.testing.assert_close(res[0][0][k], v, rtol=1e-5, atol=1e-6)


def test_ssp0_thread_ranks_gpu_track_sync_sgd():
    res = run_loopback(_body, 2, 0, 6, 0.2, [_model(), _model()])
    ref = _oracle(2, 6, 0.2)
    for r in range(2):
        for k, v in ref.items():
            assert torch.equal(res[r][0][k], res[0][0][k])
            torch.testing.assert_close(res[r][0][k], v, rtol=0, atol=5e-3)


def test_asp_bf16_adam_thread_ranks_gpu_converge():
    res = run_loopback(_body, 2, None, 30, 0.0, [_model(torch.bfloat16), _model(torch.bfloat16)], True)
    assert res[0][1][-1] < 0.8 * res[0][1][0]


def _proc_body(tp, steps):
    return _body(tp, 1, steps, 0.2)


def test_two_processes_ipc_mailboxes_on_one_gpu():
    res = dist_util.run(_proc_body, 2, (8,))
    for k in res[0][0]:
        assert torch.equal(res[0][0][k], res[1][0][k])
    assert res[0][1][-1] < res[0][1][0]


def _exact_body(tp, steps, models):
    from ps_amd.parallel.async_ps import AsyncPS
    from ps_amd.parallel.updaters import SimpleUpdater

    torch.cuda.set_device(0)
    m = models[tp.rank]
    ps = AsyncPS(m, SimpleUpdater(0.25), tp, staleness=None, timeout_s=60)  # ASP
    c = torch.full((16, 64), float(tp.rank + 1), device=DEV)
    for _ in range(steps):
        (m.weight * c).sum().backward()  # gradient == c: independent of the weights read
        ps.finish_step()
    ps.synchronize()
    tp.barrier()
    ps.refresh()
    out = m.weight.detach().cpu().clone()
    ps.close()
    return out


def test_asp_slow_server_applies_every_push_exactly_once(monkeypatch):
    """ADVICE r2 (mailbox race): with a slow owner the worker's host runs far ahead; every push
    must still be applied exactly once and never read while being overwritten.  SGD with a
    weight-independent gradient makes the final weights an exact sum:
    w = w0 - lr / W * steps * (c_0 + c_1), exactly representable in fp32."""
    monkeypatch.setenv("PS_AMD_ASYNC_SERVE_DELAY_US", "3000")
    steps = 12
    models = [torch.nn.Linear(64, 16, bias=False).to(DEV) for _ in range(2)]
    with torch.no_grad():
        for mm in models:
            mm.weight.fill_(1.0)
    res = run_loopback(_exact_body, 2, steps, models)
    want = 1.0 - 0.25 / 2 * steps * (1.0 + 2.0)
    for r in range(2):
        assert torch.equal(res[r], torch.full((16, 64), want)), res[r].unique()
