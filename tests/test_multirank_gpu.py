"""World > 1 parameter-server paths through the HIP kernels on ONE MI355X.

The co-located PS, the sharded sparse tables and the reference models run as W thread-ranks
on cuda:0 joined by the in-process LoopbackTransport (collectives are exchanges of GPU
tensors; each rank drains its stream before sharing), so every world > 1 code path -- owner
range shards, reduce-scatter / all-gather landing, SSP slot rings, the clip all-reduce, the
1-bit all-to-all + owner unpack-reduce kernel, the sparse id/row all-to-alls with the HIP hash
map and the sorted-run row optimizer -- executes with GPU tensors and is compared with a
single-process fp32 oracle.  ``overlap=False`` everywhere: with thread-ranks, collectives must
be issued from the rank threads, not from autograd's device thread.
"""
import copy

import pytest
import torch
import torch.nn.functional as F

from ps_amd.parallel.transport import run_loopback

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(40, 64), torch.nn.Tanh(), torch.nn.Linear(64, 5))


def _data(n=64, dev=DEV):
    g = torch.Generator().manual_seed(3)
    return torch.randn(n, 40, generator=g).to(dev), torch.randint(0, 5, (n,), generator=g).to(dev)


def _train(tp, models, kw, steps, upd_factory, dev):
    from ps_amd.parallel.colocated import ColocatedPS

    m = models[tp.rank]
    ps = ColocatedPS(m, upd_factory(), tp, bucket_mb=0.004, last_bucket_mb=0.002, overlap=False, **kw)
    x, y = _data(dev=dev)
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    losses = []
    for _ in range(steps):
        loss = F.cross_entropy(m(xs), ys)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    ps.synchronize()
    return {n: p.detach().float().cpu().clone() for n, p in m.named_parameters()}, losses


def _oracle(world, steps, opt_factory, clip=None):
    ref = _model(0).to(DEV)
    opt = opt_factory(ref.parameters())
    x, y = _data()
    for _ in range(steps):
        opt.zero_grad()
        (sum(F.cross_entropy(ref(x[r::world]), y[r::world]) for r in range(world)) / world).backward()
        if clip is not None:
            torch.nn.utils.clip_grad_norm_(ref.parameters(), clip)
        opt.step()
    return {n: p.detach().cpu() for n, p in ref.named_parameters()}


@pytest.mark.parametrize("world", [2, 4])
def test_bsp_multirank_gpu_equals_single_process(world):
    from ps_amd.parallel.updaters import MomentumUpdater

    models = [_model(seed=r).to(DEV) for r in range(world)]
    res = run_loopback(_train, world, models, {}, 5, lambda: MomentumUpdater(0.1, 0.9, 1e-4), DEV)
    for r in range(1, world):
        for k in res[0][0]:
            assert torch.equal(res[0][0][k], res[r][0][k])
    ref = _oracle(world, 5, lambda p: torch.optim.SGD(p, lr=0.1, momentum=0.9, weight_decay=1e-4))
    for k, v in ref.items():
        torch.testing.assert_close(res[0][0][k], v, rtol=1e-5, atol=1e-5)


def test_clip_norm_multirank_gpu():
    from ps_amd.parallel.updaters import SimpleUpdater

    world = 2
    models = [_model(0).to(DEV) for _ in range(world)]
    res = run_loopback(_train, world, models, {"clip_norm": 0.05}, 4, lambda: SimpleUpdater(0.5), DEV)
    ref = _oracle(world, 4, lambda p: torch.optim.SGD(p, lr=0.5), clip=0.05)
    for k, v in ref.items():
        torch.testing.assert_close(res[0][0][k], v, rtol=1e-5, atol=1e-5)


def test_ssp1_multirank_gpu_matches_delayed_sgd():
    from ps_amd.parallel.updaters import SimpleUpdater

    world, steps, lr, s = 2, 6, 0.2, 1
    models = [_model(0).to(DEV) for _ in range(world)]
    res = run_loopback(_train, world, models, {"staleness": s}, steps, lambda: SimpleUpdater(lr), DEV)
    ref = _model(0).to(DEV)
    x, y = _data()
    versions = [{n: p.detach().clone() for n, p in ref.named_parameters()}]
    for t in range(steps):
        probe = copy.deepcopy(ref)
        with torch.no_grad():
            for n, p in probe.named_parameters():
                p.copy_(versions[max(0, t - s)][n])
        loss = sum(F.cross_entropy(probe(x[r::world]), y[r::world]) for r in range(world)) / world
        grads = torch.autograd.grad(loss, list(probe.parameters()))
        versions.append({n: versions[-1][n] - lr * g for (n, _), g in zip(probe.named_parameters(), grads)})
    want = versions[max(0, steps - s)]
    for k in want:
        torch.testing.assert_close(res[0][0][k], want[k].cpu(), rtol=1e-5, atol=1e-5)


def test_onebit_multirank_gpu_matches_cpu_oracle():
    from ps_amd.parallel.updaters import SimpleUpdater

    world = 2
    upd = lambda: SimpleUpdater(0.3)  # noqa: E731
    gpu = run_loopback(_train, world, [_model(0).to(DEV) for _ in range(world)], {"compress": "onebit"}, 12, upd,
                       DEV)
    cpu = run_loopback(_train, world, [_model(0) for _ in range(world)], {"compress": "onebit"}, 12, upd,
                       torch.device("cpu"))
    for k in gpu[0][0]:
        assert torch.equal(gpu[0][0][k], gpu[1][0][k])
        torch.testing.assert_close(gpu[0][0][k], cpu[0][0][k], rtol=1e-3, atol=1e-3)
    assert gpu[0][1][-1] < gpu[0][1][0]


def _sparse_body(tp, mode, dev):
    from ps_amd.parallel.sparse_table import ShardedSparseTable
    from ps_amd.parallel.updaters import AdagradUpdater

    t = ShardedSparseTable("emb", 16, [3000, 2000], tp, AdagradUpdater(0.1, 1e-8, rowwise=True), init=(-0.1, 0.1),
                           id_mode=mode, seed=3, device=dev, fields=2)
    g = torch.Generator().manual_seed(100 + tp.rank)
    for _ in range(3):
        ids = torch.randint(0, 1500, (128, 2), generator=g)
        rows = t.lookup(ids.to(dev))
        (rows.float() * torch.linspace(-1, 1, 16, device=dev)).sum().backward()
        t.push_pending()
    probe = torch.arange(1500).repeat(2, 1).t().contiguous()
    out = t.pull(probe.to(dev)).cpu()
    t.synchronize()
    return out


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("mode", ["direct", "map"])
def test_sharded_sparse_table_multirank_gpu(world, mode):
    res = run_loopback(_sparse_body, world, mode, DEV)
    ref = run_loopback(_sparse_body, world, mode, torch.device("cpu"))
    for r in range(world):
        torch.testing.assert_close(res[r], res[0], rtol=0, atol=0)
        torch.testing.assert_close(res[r], ref[0], rtol=1e-5, atol=1e-6)


def _dnn_body(tp, wide, dev, n):
    from ps_amd.context import ctx
    from ps_amd.data.dataset import synthetic_ctr
    from ps_amd.models.reference import DNN, WideDeepNN, sharded_table_factory
    from ps_amd.train.trainer import CollectiveEngine, Trainer

    ctx.init()
    tf = sharded_table_factory(tp, dev, seed=7, overlap=False)
    gen = torch.Generator().manual_seed(0)
    if wide:
        m = WideDeepNN.build_model(4, 8, 6, [32, 8, 1], 500, gen=gen, emb_rows=256, table_factory=tf, init_scale=0.2)
    else:
        m = DNN.build_model(4, 8, 6, [32, 8, 1], gen=gen, emb_rows=256, table_factory=tf, init_scale=0.2)
    m = m.to(dev)
    tr = Trainer(m, CollectiveEngine(m, tp, bucket_mb=0.002, overlap=False), device=dev)
    lo, hi = tp.rank * n // tp.world, (tp.rank + 1) * n // tp.world
    for i in range(3):
        b = synthetic_ctr(n, fields=4, numeric=6, ids_per_field=40, wide_k=3 if wide else 0, wide_size=500, seed=i)
        tr.train([{k: v[lo:hi] for k, v in b.items()}])
    tr.engine.synchronize()
    ids = torch.arange(40).repeat(4, 1).t().contiguous().to(dev)
    return ({k: v.detach().cpu() for k, v in m.named_parameters()}, m.tables()["emF"].pull(ids).cpu())


@pytest.mark.parametrize("wide", [False, True])
def test_reference_models_sharded_rows_multirank_gpu(wide):
    gpu = run_loopback(_dnn_body, 2, wide, DEV, 64)
    single = run_loopback(_dnn_body, 1, wide, torch.device("cpu"), 64)[0]
    for r in range(2):
        for k, v in single[0].items():
            torch.testing.assert_close(gpu[r][0][k], v, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(gpu[r][1], single[1], rtol=1e-4, atol=1e-4)


def _dlrm_body(tp, n, inits):
    from ps_amd.models.dlrm import DLRM, dlrm_batch
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import AdagradUpdater

    rows = [700] * 4
    m = DLRM(dense_in=13, table_rows=rows, dim=16, bottom=(32,), top=(32, 16), transport=tp, device=DEV,
             overlap=False)
    m.load_state_dict(inits, strict=False)  # dense init drawn outside the threads (shared global RNG)
    m = m.to(DEV)
    ps = ColocatedPS(m, AdagradUpdater(0.05, 1e-8), tp, bucket_mb=0.05, overlap=False)
    dense, sparse, y = dlrm_batch(n, rows, seed=11, device=DEV)
    lo, hi = tp.rank * n // tp.world, (tp.rank + 1) * n // tp.world
    for _ in range(4):
        F.binary_cross_entropy_with_logits(m(dense[lo:hi], sparse[lo:hi]), y[lo:hi]).backward()
        m.push_sparse()
        ps.finish_step()
    ps.synchronize()
    return ({k: v.detach().cpu() for k, v in m.named_parameters()},
            m.emb.table.pull_keys(torch.arange(2800, device=DEV)).cpu())


def test_dlrm_multirank_gpu_equals_single_rank():
    from ps_amd.models.dlrm import DLRM

    torch.manual_seed(0)
    inits = DLRM(dense_in=13, table_rows=[700] * 4, dim=16, bottom=(32,), top=(32, 16)).state_dict()
    w2 = run_loopback(_dlrm_body, 2, 256, inits)
    w1 = run_loopback(_dlrm_body, 1, 256, inits)[0]
    for r in range(2):
        for k, v in w1[0].items():
            torch.testing.assert_close(w2[r][0][k], v, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(w2[r][1], w1[1], rtol=1e-4, atol=1e-5)


def test_split_push_pull_streams_multirank_gpu():
    """Pull (all-gather) on its own communicator + HIP stream: same result as one communicator."""
    from ps_amd.parallel.updaters import MomentumUpdater

    upd = lambda: MomentumUpdater(0.1, 0.9, 1e-4)  # noqa: E731
    one = run_loopback(_train, 2, [_model(0).to(DEV) for _ in range(2)], {}, 4, upd, DEV)
    two = run_loopback(_train, 2, [_model(0).to(DEV) for _ in range(2)], {"split_comm": True}, 4, upd, DEV)
    for k in one[0][0]:
        torch.testing.assert_close(two[0][0][k], one[0][0][k], rtol=0, atol=0)
