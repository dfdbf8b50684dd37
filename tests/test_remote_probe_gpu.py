"""Start-up probes of the one-sided remote-write paths on the GPU (parallel/remote_probe.py), W
real processes on cuda:0: the push copy kernel into IPC-mapped owner mailboxes read back by the
serve's acquire kernel (AsyncPS), the owners' row-send kernel into the workers' arenas read after
the inter-process events (row plane).  An injected probe failure on one rank makes EVERY rank take
the fallback, which trains and matches the oracle."""
import types

import pytest
import torch
import torch.nn.functional as F

from tests import dist_util

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.Tanh(), torch.nn.Linear(64, 4)).to(DEV)


def _data(n=64):
    g = torch.Generator().manual_seed(3)
    return torch.randn(n, 32, generator=g).to(DEV), torch.randint(0, 4, (n,), generator=g).to(DEV)


def _engine_body(tp, fail, steps):
    import os

    if fail:
        os.environ["PS_AMD_PROBE_FAIL"] = fail
    from ps_amd.bench_configs import async_or_pipelined
    from ps_amd.parallel.updaters import SimpleUpdater

    torch.cuda.set_device(0)
    m = _model()
    args = types.SimpleNamespace(bucket_mb=0.01, last_bucket_mb=0.005)
    # staleness 0: the async engine is the BSP trajectory too (SSP(0) gate), so both the
    # probe-passed and the fallback engine must reproduce synchronous SGD
    ps, is_async, probe = async_or_pipelined(m, SimpleUpdater(0.2), tp, 0, args)
    x, y = _data()
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    for _ in range(steps):
        F.cross_entropy(m(xs), ys).backward()
        ps.finish_step()
    ps.synchronize()
    tp.barrier()
    if is_async:
        ps.refresh()
    out = {n: p.detach().float().cpu().clone() for n, p in m.named_parameters()}
    ps.close()
    return out, type(ps).__name__, probe


def _oracle(world, steps, lr):
    ref = _model()
    opt = torch.optim.SGD(ref.parameters(), lr=lr)
    x, y = _data()
    for _ in range(steps):
        opt.zero_grad()
        (sum(F.cross_entropy(ref(x[r::world]), y[r::world]) for r in range(world)) / world).backward()
        opt.step()
    return {n: p.detach().cpu() for n, p in ref.named_parameters()}


@pytest.mark.parametrize("fail", [None, "asyncps@1"])
def test_asyncps_probe_and_fallback_two_processes(fail):
    res = dist_util.run(_engine_body, 2, (fail, 6))
    want = _oracle(2, 6, 0.2)
    for out, name, probe in res:
        if fail is None:
            assert name == "AsyncPS" and probe["remote_write_probe"].startswith("ok"), probe
        else:  # rank 1's injected failure: both ranks run the pipelined collective engine
            assert name == "ColocatedPS" and "ranks [1]" in probe["engine_fallback"], probe
        for k, v in want.items():
            torch.testing.assert_close(out[k], v, rtol=0, atol=5e-3)
    for k in res[0][0]:
        assert torch.equal(res[0][0][k], res[1][0][k])


def _rows_body(tp, fail):
    import os

    if fail:
        os.environ["PS_AMD_PROBE_FAIL"] = fail
    from ps_amd.parallel.sparse_table import ShardedSparseTable

    torch.cuda.set_device(0)
    t = ShardedSparseTable("emb", 16, [500], tp, None, device=DEV)
    info = (t.exchange, dict(t.exchange_info))
    t.close()
    return info


@pytest.mark.parametrize("fail", [None, "rowplane@0"])
def test_row_plane_probe_two_processes(fail):
    res = dist_util.run(_rows_body, 2, (fail,))
    for ex, info in res:
        if fail is None:
            assert ex == "plane" and info["remote_write_probe"].startswith("ok"), info
        else:
            assert ex == "collective" and "ranks [0]" in info["fallback"], info


def _async_rows_body(tp, fail):
    import os

    if fail:
        os.environ["PS_AMD_PROBE_FAIL"] = fail
    from ps_amd.parallel import remote_probe as RP
    from ps_amd.parallel.async_rows import AsyncRowTable
    from ps_amd.parallel.updaters import AdagradUpdater

    torch.cuda.set_device(0)
    try:
        t = AsyncRowTable("emb", 8, 1000, tp, AdagradUpdater(0.1, 1e-8), init=(-0.1, 0.1), staleness=1,
                          capacity=256, device=DEV, timeout_s=60)
    except RP.RemoteWriteUnavailable as e:
        return "raised", str(e), None
    ids = torch.arange(0, 40, device=DEV)
    before = t.pull(ids)
    t.push(ids, torch.ones(40, 8, device=DEV))
    t.synchronize()
    after = t.pull(ids)
    torch.cuda.synchronize()
    info = dict(t.info)
    ok = bool((after < before).all())
    t.close()
    return "ok", info, ok


@pytest.mark.parametrize("fail", [None, "asyncrows@1"])
def test_async_rows_probe_two_processes(fail):
    """The asynchronous row tables' mailbox writes (rows.to_peers into IPC-mapped owner mailboxes,
    read back through an acquiring kernel): the probe passes and the rows train; an injected
    failure on one rank raises on both."""
    res = dist_util.run(_async_rows_body, 2, (fail,))
    for kind, info, dec in res:
        if fail:
            assert kind == "raised" and "ranks [1]" in info
        else:
            assert kind == "ok" and info["remote_write_probe"].startswith("ok") and dec
