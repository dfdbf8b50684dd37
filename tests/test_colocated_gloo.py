"""Co-located PS over multi-process gloo (world 2): BSP equivalence with a single process on
the global batch, SSP(1) semantics, 1-bit compressed push, sharded sparse tables."""
import pytest
import torch

from tests import dist_util


def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(12, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))


def _data(n=64):
    g = torch.Generator().manual_seed(7)
    return torch.randn(n, 12, generator=g), torch.randint(0, 4, (n,), generator=g)


def _bsp_body(tp, staleness, compress, steps):
    import torch.nn.functional as F

    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import MomentumUpdater

    m = _model(seed=tp.rank)  # different init per rank: rank 0's broadcast must win
    ps = ColocatedPS(m, MomentumUpdater(0.1, 0.9, 1e-4), tp, bucket_mb=0.001, last_bucket_mb=0.0005,
                     staleness=staleness, compress=compress)
    x, y = _data()
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    losses = []
    for _ in range(steps):
        loss = F.cross_entropy(m(xs), ys)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    ps.synchronize()
    return {n: p.detach().clone() for n, p in m.named_parameters()}, losses, ps.t.n_ops


def test_bsp_world2_equals_single_process():
    res = dist_util.run(_bsp_body, 2, (0, None, 4))
    w0, w1 = res[0][0], res[1][0]
    for k in w0:
        torch.testing.assert_close(w0[k], w1[k])  # replicas identical after every pull
    # oracle: one process, full batch == average of the two half-batch gradients
    import torch.nn.functional as F

    ref = _model(seed=0)
    opt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x, y = _data()
    for _ in range(4):
        opt.zero_grad()
        loss = (F.cross_entropy(ref(x[0::2]), y[0::2]) + F.cross_entropy(ref(x[1::2]), y[1::2])) / 2
        loss.backward()
        opt.step()
    for n, p in ref.named_parameters():
        torch.testing.assert_close(w0[n], p.detach(), rtol=1e-5, atol=1e-6)


def test_ssp1_world2_consistent_and_learns():
    res = dist_util.run(_bsp_body, 2, (1, None, 12))
    w0, w1 = res[0][0], res[1][0]
    for k in w0:
        torch.testing.assert_close(w0[k], w1[k])
    losses = res[0][1]
    assert losses[-1] < losses[0]


def test_onebit_compressed_push_learns():
    res = dist_util.run(_bsp_body, 2, (0, "onebit", 25))
    losses = res[0][1]
    assert losses[-1] < losses[0] * 0.9
    for k in res[0][0]:
        torch.testing.assert_close(res[0][0][k], res[1][0][k])


def _sparse_body(tp, id_mode):
    from ps_amd.parallel.sparse_table import ShardedSparseTable
    from ps_amd.parallel.updaters import AdagradUpdater

    t = ShardedSparseTable("emb", 8, 1000, tp, AdagradUpdater(0.1, 1e-8), init=(-0.1, 0.1), id_mode=id_mode,
                           seed=3)
    g = torch.Generator().manual_seed(tp.rank)
    ids = torch.unique(torch.randint(0, 1000, (100,), generator=g))
    before = t.pull(ids)
    again = t.pull(ids)
    assert torch.equal(before, again)  # lazy init is stable
    grads = torch.ones(ids.numel(), 8)
    t.push(ids, grads)
    after = t.pull(ids)
    common = torch.tensor([1, 2, 3, 500, 999])
    return ids, before, after, t.pull(common)


def test_sharded_sparse_table_world2():
    for mode in ("direct", "hash"):
        res = dist_util.run(_sparse_body, 2, (mode,))
        # every rank sees the same row values for the same ids
        torch.testing.assert_close(res[0][3], res[1][3])
        for ids, before, after, _ in res:
            assert (after < before).all()  # positive grads -> every touched row decreased


def _warm_body(tp, warm):
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import SimpleUpdater

    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(12, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    ps = ColocatedPS(m, SimpleUpdater(0.1), tp, bucket_mb=0.002, compress="onebit" if warm >= 0 else None,
                     compress_warmup=max(0, warm))
    g = torch.Generator().manual_seed(tp.rank)
    x, y = torch.randn(32, 12, generator=g), torch.randint(0, 4, (32,), generator=g)
    out = []
    for _ in range(4):
        torch.nn.functional.cross_entropy(m(x), y).backward()
        ps.finish_step()
        out.append({k: v.detach().clone() for k, v in m.named_parameters()})
    return out


def test_onebit_warmup_rounds_are_full_precision():
    """compress_warmup=k: the first k rounds push full precision (identical to no
    compression), later rounds are 1-bit (different)."""
    full = dist_util.run(_warm_body, 2, (-1,))
    warm = dist_util.run(_warm_body, 2, (2,))
    for step in (0, 1):
        for k in full[0][step]:
            torch.testing.assert_close(warm[0][step][k], full[0][step][k], rtol=0, atol=0)
    assert any(not torch.equal(warm[0][3][k], full[0][3][k]) for k in full[0][3])


def _split_model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(12, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))


def _split_body(tp, split, clip, models=None):
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import MomentumUpdater

    m = models[tp.rank] if models is not None else _split_model()  # thread-ranks: built outside
    ps = ColocatedPS(m, MomentumUpdater(0.1, 0.9), tp, bucket_mb=0.001, split_comm=split, clip_norm=clip)
    assert (ps.tpull is not ps.t) == (split and tp.world > 1)
    g = torch.Generator().manual_seed(tp.rank)
    for _ in range(4):
        x, y = torch.randn(16, 12, generator=g), torch.randint(0, 4, (16,), generator=g)
        torch.nn.functional.cross_entropy(m(x), y).backward()
        ps.finish_step()
    return {k: v.detach().clone() for k, v in m.named_parameters()}


@pytest.mark.parametrize("clip", [None, 0.5])
def test_split_push_pull_communicators_same_result(clip):
    """pulls on their own communicator give bitwise the same training (gloo world 2)."""
    a = dist_util.run(_split_body, 2, (False, clip))
    b = dist_util.run(_split_body, 2, (True, clip))
    for k in a[0]:
        assert torch.equal(a[0][k], b[0][k]) and torch.equal(b[0][k], b[1][k])


def test_split_communicators_loopback_world3():
    from ps_amd.parallel.transport import run_loopback

    a = run_loopback(_split_body, 3, False, None, [_split_model() for _ in range(3)])
    b = run_loopback(_split_body, 3, True, None, [_split_model() for _ in range(3)])
    for k in a[0]:
        assert torch.equal(a[0][k], b[0][k])


def _probe_body(tp):
    from ps_amd.parallel.comm_probe import probe

    return probe(torch.device("cpu"), sizes_mb=(0.25, 1), iters=2, dtype=torch.float32)


def test_comm_probe_world2():
    """bench.py's after-the-timed-region collective probe: same result structure on every rank,
    MAX-over-ranks times (identical), busbw = algbw * (n-1)/n for RS / AG, 2(n-1)/n for AR."""
    res = dist_util.run(_probe_body, 2, ())
    assert res[0] == res[1]
    for name in ("reduce_scatter", "all_gather", "all_reduce", "reduce_scatter_direct", "all_gather_direct"):
        for size in ("0.25MB", "1MB"):
            r = res[0][name][size]
            assert r["us"] > 0 and r["algbw_GBps"] >= 0
            fac = 1.0 if name == "all_reduce" else 0.5
            assert abs(r["busbw_GBps"] - r["algbw_GBps"] * fac) <= 0.11
