"""Start-up probes of the one-sided remote-write paths and their uniform fallbacks (VERDICT r5
Next #2; parallel/remote_probe.py).  CPU ranks are gloo processes over shared memory: the same
probe protocol, agreement and fallback code the GPU processes run (tests/test_remote_probe_gpu.py
covers the HIP write / read kernels)."""
import types

import pytest
import torch

from ps_amd.parallel import remote_probe as RP
from ps_amd.parallel.transport import Transport

from . import dist_util


def test_run_probe_detects_a_stale_read():
    """A reader that keeps serving the previous round's lines must fail the probe."""
    mem = {"cur": torch.zeros(4), "seen": torch.zeros(4)}

    def write(k):
        mem["cur"] = RP.pattern(k, 1, 4)

    def read(k):
        out = mem["seen"].clone()  # a stale cache: what the reader saw the round before
        mem["seen"] = mem["cur"].clone()
        return out.view(1, 4)

    with pytest.raises(RP.RemoteWriteUnavailable, match="round 0"):
        RP.run_probe(Transport(), "asyncps", 3, write, lambda k: None, read, lambda k: RP.pattern(k, 1, 4).view(1, 4),
                     lambda: None)
    # a coherent reader passes, and the record says what ran
    ok = RP.run_probe(Transport(), "asyncps", 3, write, lambda k: None, lambda k: mem["cur"].view(1, 4),
                      lambda k: RP.pattern(k, 1, 4).view(1, 4), lambda: None)
    assert ok.startswith("ok (3 rounds")


def test_injection_parsing(monkeypatch):
    monkeypatch.setenv("PS_AMD_PROBE_FAIL", "rowplane@1, asyncps")
    assert RP.injected("rowplane", 1) and not RP.injected("rowplane", 0)
    assert RP.injected("asyncps", 0) and RP.injected("asyncps", 3)
    monkeypatch.setenv("PS_AMD_PROBE_FAIL", "all@2")
    assert RP.injected("asyncrows", 2) and not RP.injected("asyncps", 0)


def _tiny():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 4))


def _asyncps_body(tp, fail):
    import os

    if fail:
        os.environ["PS_AMD_PROBE_FAIL"] = fail
    from ps_amd.parallel.async_ps import AsyncPS
    from ps_amd.parallel.updaters import SimpleUpdater

    try:
        ps = AsyncPS(_tiny(), SimpleUpdater(0.1), tp, staleness=1, timeout_s=60)
    except RP.RemoteWriteUnavailable as e:
        return "raised", str(e)
    info = dict(ps.info)
    ps.close()
    return "ok", info


def test_asyncps_probe_passes_on_shared_memory_ranks():
    res = dist_util.run(_asyncps_body, 2, (None,))
    for kind, info in res:
        assert kind == "ok" and info["remote_write_probe"].startswith("ok")


def test_asyncps_probe_failure_is_agreed_by_every_rank():
    res = dist_util.run(_asyncps_body, 2, ("asyncps@1",))
    for kind, msg in res:  # rank 0 passed its own probe, but rank 1 failed: both raise
        assert kind == "raised" and "ranks [1]" in msg and "injected" in msg


def _fallback_body(tp, steps):
    import os

    os.environ["PS_AMD_PROBE_FAIL"] = "asyncps@0"
    from ps_amd.bench_configs import async_or_pipelined
    from ps_amd.parallel.updaters import SimpleUpdater

    model = _tiny()
    args = types.SimpleNamespace(bucket_mb=0.001, last_bucket_mb=0.0005)
    ps, is_async, probe = async_or_pipelined(model, SimpleUpdater(0.1), tp, 1, args)
    g = torch.Generator().manual_seed(3)
    x, y = torch.randn(16, 8, generator=g), torch.randint(0, 4, (16,), generator=g)
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    for _ in range(steps):
        torch.nn.functional.cross_entropy(model(xs), ys).backward()
        ps.finish_step()
    ps.synchronize() if hasattr(ps, "synchronize") else None
    w = [p.detach().clone() for p in model.parameters()]
    return type(ps).__name__, is_async, probe, w


def test_bert_engine_falls_back_to_pipelined_collective_ssp():
    res = dist_util.run(_fallback_body, 2, (3,))
    for name, is_async, probe, _ in res:
        assert name == "ColocatedPS" and not is_async
        assert probe["remote_write_probe"] == "failed" and "pipelined-collective" in probe["engine_fallback"]
    for a, b in zip(res[0][3], res[1][3]):  # the fallback engine trains in lockstep
        assert torch.equal(a, b)


def _rows_body(tp, fail):
    import os

    if fail:
        os.environ["PS_AMD_PROBE_FAIL"] = fail
    from tests.test_row_plane_cpu import _train

    return _train(tp, None, 2, 40, 1)


def test_row_plane_probe_failure_falls_back_to_collective_all_to_alls():
    from tests.test_row_plane_cpu import _single
    from tests.test_sparse_ps_cpu import _assert_same

    res = dist_util.run(_rows_body, 2, ("rowplane@0",))
    single = _single(2, 40)
    for r in range(2):
        assert all(ex == "collective" for ex, _, _ in res[r][2].values())
        _assert_same(res[r][:2], single)
    ok = dist_util.run(_rows_body, 2, (None,))
    assert all(ex == "plane" for ex, _, _ in ok[0][2].values())


def _async_rows_body(tp, fail):
    import os

    if fail:
        os.environ["PS_AMD_PROBE_FAIL"] = fail
    from ps_amd.parallel.async_rows import AsyncRowTable
    from ps_amd.parallel.updaters import AdagradUpdater

    try:
        t = AsyncRowTable("emb", 8, 1000, tp, AdagradUpdater(0.1, 1e-8), init=(-0.1, 0.1), staleness=1,
                          capacity=256, timeout_s=60)
    except RP.RemoteWriteUnavailable as e:
        return "raised", str(e), None
    ids = torch.arange(0, 40)
    before = t.pull(ids)
    t.push(ids, torch.ones(40, 8))
    t.synchronize()
    after = t.pull(ids)
    info = dict(t.info)
    t.close()
    return "ok", info, bool((after < before).all())


def test_async_rows_probe_passes_and_rows_train():
    res = dist_util.run(_async_rows_body, 2, (None,))
    for kind, info, dec in res:
        assert kind == "ok" and info["remote_write_probe"].startswith("ok") and dec
    # the probe's lines were zeroed: a push after it is applied as pushed (rows decrease, above)


def test_async_rows_probe_failure_is_agreed_by_every_rank():
    res = dist_util.run(_async_rows_body, 2, ("asyncrows@0",))
    for kind, msg, _ in res:
        assert kind == "raised" and "ranks [0]" in msg and "asyncrows" in msg
