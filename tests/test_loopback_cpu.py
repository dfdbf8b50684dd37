"""In-process fake backend: the co-located PS over LoopbackTransport threads --
deterministic, single process.  BSP equivalence with a single large-batch process at world 4,
the exact SSP(s) semantics (forward t reads weight version max(0, t - s)) against a delayed-SGD
oracle, sharded sparse tables vs one local table, and the collective-order checker."""
import copy

import pytest
import torch
import torch.nn.functional as F

from ps_amd.parallel.transport import run_loopback


def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(10, 24), torch.nn.Tanh(), torch.nn.Linear(24, 3))


def _data(n=48):
    g = torch.Generator().manual_seed(3)
    return torch.randn(n, 10, generator=g), torch.randint(0, 3, (n,), generator=g)


def _train(tp, models, staleness, steps, upd_factory):
    from ps_amd.parallel.colocated import ColocatedPS

    m = models[tp.rank]
    ps = ColocatedPS(m, upd_factory(), tp, bucket_mb=0.0005, last_bucket_mb=0.0002, staleness=staleness)
    x, y = _data()
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    for _ in range(steps):
        F.cross_entropy(m(xs), ys).backward()
        ps.finish_step()
    ps.synchronize()
    return {n: p.detach().clone() for n, p in m.named_parameters()}


def test_loopback_bsp_world4_equals_single_process():
    from ps_amd.parallel.updaters import MomentumUpdater

    world, steps = 4, 5
    models = [_model(seed=r) for r in range(world)]  # rank 0's init is broadcast
    res = run_loopback(_train, world, models, 0, steps, lambda: MomentumUpdater(0.1, 0.9, 1e-4))
    for r in range(1, world):
        for k in res[0]:
            assert torch.equal(res[0][k], res[r][k])  # bitwise-identical replicas
    ref = _model(seed=0)
    opt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x, y = _data()
    for _ in range(steps):
        opt.zero_grad()
        sum(F.cross_entropy(ref(x[r::world]), y[r::world]) for r in range(world)).div(world).backward()
        opt.step()
    for n, p in ref.named_parameters():
        torch.testing.assert_close(res[0][n], p.detach(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("staleness", [1, 2])
def test_loopback_ssp_matches_delayed_sgd_oracle(staleness):
    """SSP(s): the gradient of step t is taken at weight version max(0, t - s) and applied to
    the newest weights -- checked exactly against a single-process delayed-SGD oracle."""
    from ps_amd.parallel.updaters import SimpleUpdater

    world, steps, lr = 2, 7, 0.2
    models = [_model(seed=0) for _ in range(world)]
    res = run_loopback(_train, world, models, staleness, steps, lambda: SimpleUpdater(lr))
    x, y = _data()
    ref = _model(seed=0)
    versions = [{n: p.detach().clone() for n, p in ref.named_parameters()}]  # versions[k] = W_k
    for t in range(steps):
        src = versions[max(0, t - staleness)]
        probe = copy.deepcopy(ref)
        with torch.no_grad():
            for n, p in probe.named_parameters():
                p.copy_(src[n])
        loss = sum(F.cross_entropy(probe(x[r::world]), y[r::world]) for r in range(world)) / world
        grads = torch.autograd.grad(loss, list(probe.parameters()))
        new = {n: versions[-1][n] - lr * g for (n, _), g in zip(probe.named_parameters(), grads)}
        versions.append(new)
    # after finish_step the replica holds the version the NEXT forward reads: max(0, steps - s)
    for n in res[0]:
        torch.testing.assert_close(res[0][n], versions[max(0, steps - staleness)][n], rtol=1e-5, atol=1e-6)


def _sparse(tp, ids_per_rank, grads_per_rank):
    from ps_amd.parallel.sparse_table import ShardedSparseTable
    from ps_amd.parallel.updaters import AdagradUpdater

    tab = ShardedSparseTable("t", 4, 64, tp, AdagradUpdater(0.1, rowwise=True), init=(-0.5, 0.5), seed=5)
    ids = ids_per_rank[tp.rank]
    before = tab.pull(ids).clone()
    tab.push(ids, grads_per_rank[tp.rank])
    after = tab.pull(torch.arange(64))
    return before, after


def test_loopback_sharded_sparse_table_matches_local_table():
    from ps_amd.parallel.sparse_table import SparseTable
    from ps_amd.parallel.updaters import AdagradUpdater

    world = 3
    g = torch.Generator().manual_seed(0)
    ids = [torch.randperm(64, generator=g)[:20] for _ in range(world)]  # unique per worker
    grads = [torch.randn(20, 4, generator=g) for _ in range(world)]
    res = run_loopback(_sparse, world, ids, grads)
    local = SparseTable("t", 4, 64, AdagradUpdater(0.1, rowwise=True), init=(-0.5, 0.5), seed=5)
    for r in range(world):
        torch.testing.assert_close(res[r][0], local.pull(ids[r]))  # same lazy init per (seed, row)
    # one server round = each row's gradients summed over the W workers, scaled by 1/W
    # (push(average=True)), one optimizer step per distinct row
    from ps_amd.ops.sparse import dedup_rows

    u, red = dedup_rows(torch.cat(ids), torch.cat(grads))
    local.push(u, red, 1.0 / world)
    for r in range(world):
        torch.testing.assert_close(res[r][1], local.pull(torch.arange(64)), rtol=1e-5, atol=1e-6)


def _order(tp, diverge):
    from ps_amd.parallel.transport import LoopbackTransport

    assert isinstance(tp, LoopbackTransport)
    tp.check_order = True
    tp.all_reduce(torch.ones(3))
    if diverge and tp.rank == 1:
        tp._note("ag", torch.ones(2))
    try:
        return tp.verify_order()
    except RuntimeError:
        return False


def test_loopback_order_checker():
    assert run_loopback(_order, 3, False) == [True, True, True]
    assert run_loopback(_order, 3, True) == [False, False, False]
