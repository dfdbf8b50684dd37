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


def _wide_gpu_body(tp, consistency, staleness, steps, delay_rank=-1, delay_s=0.0):
    import time

    from ps_amd.context import ctx
    from ps_amd.parallel.async_rows import async_table_factory
    from ps_amd.train.trainer import CollectiveEngine, Trainer
    from tests.test_sparse_ps_cpu import _batches, _build

    torch.cuda.set_device(0)
    ctx.init()
    s = None if consistency == "asp" else staleness
    m = _build(True, async_table_factory(tp, DEV, seed=7, staleness=s)).to(DEV)
    eng = CollectiveEngine(m, tp, consistency=consistency, staleness=staleness or 0)
    eng.ps.gate_log = []
    m.tables()["emF"].gate_log = []
    tr = Trainer(m, eng, device=DEV)
    n = 64
    lo, hi = tp.rank * n // tp.world, (tp.rank + 1) * n // tp.world
    fixed = _batches(1, n, True)[0]
    losses, dlead, rlead, skew = [], [], [], []
    for _ in range(steps):
        if tp.rank == delay_rank:
            time.sleep(delay_s)
        losses.append(tr.train([{k: v[lo:hi] for k, v in fixed.items()}]))
        c = eng.ps.snapshot()["clock"]
        dlead.append(c[tp.rank] - min(c))
        rc = m.tables()["emF"].clocks()
        rlead.append(rc[tp.rank] - min(rc))
        skew.append(min(c) - min(rc))  # dense vs row window seen by this worker's next forward
    eng.ps.synchronize()
    for t in m.tables().values():
        t.synchronize()
    tp.barrier()
    eng.ps.refresh()
    dense = {k: v.detach().float().cpu().clone() for k, v in m.named_parameters()}
    probe = m.tables()["emF"].pull(torch.arange(40).repeat(4, 1).t().contiguous()).cpu()
    dgates, rgates = list(eng.ps.gate_log), list(m.tables()["emF"].gate_log)
    eng.ps.close()
    for t in m.tables().values():
        t.close()
    return {"losses": losses, "dlead": dlead, "rlead": rlead, "skew": skew, "dense": dense, "probe": probe,
            "dgates": dgates, "rgates": rgates}


@pytest.mark.parametrize("consistency,staleness", [("asp", None), ("ssp", 1)])
def test_widedeep_async_two_processes_gpu(consistency, staleness):
    """WideDeepNN (FTRL wide.bias + Adam segments on the owners' HIP fused
    optimizer, embedding and wide ROWS on the owners' row services) under ASP / SSP(1) with 2
    processes on cuda:0 -- no collective anywhere in the step."""
    res = dist_util.run(_wide_gpu_body, 2, (consistency, staleness, 25))
    for r in res:
        assert sum(r["losses"][-5:]) / 5 < 0.8 * sum(r["losses"][:5]) / 5, r["losses"]
    for k in res[0]["dense"]:
        assert torch.equal(res[0]["dense"][k], res[1]["dense"][k])
    assert torch.equal(res[0]["probe"], res[1]["probe"])


def test_ssp1_straggler_bound_dense_and_rows_gpu():
    res = dist_util.run(_wide_gpu_body, 2, ("ssp", 1, 10, 1, 0.15))
    assert max(res[0]["dlead"]) <= 2 and max(res[0]["rlead"]) <= 2, (res[0]["dlead"], res[0]["rlead"])
    # the dense and the row gates are separate clocks, but both count this worker's steps: the
    # slowest worker's dense and row clocks seen together never drift more than the bound apart
    for r in res:
        assert max(abs(k) for k in r["skew"]) <= 2, r["skew"]  # staleness 1 + one push in flight
        # one forward's dense pull and row pull: the same gate target c - 1 and both views inside
        # [c - 1, c] (tests/test_async_rows_cpu.py, the CPU twin)
        dense = {c: (t, seen) for c, t, seen in r["dgates"]}
        rows = {c: (t, seen) for c, t, seen in r["rgates"]}
        common = sorted(set(dense) & set(rows))
        assert len(common) >= 8, (r["dgates"], r["rgates"])
        for c in common:
            assert dense[c][0] == rows[c][0] == c - 1
            assert c - 1 <= dense[c][1] <= c and c - 1 <= rows[c][1] <= c, (c, dense[c], rows[c])
