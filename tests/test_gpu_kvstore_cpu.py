"""GpuKVStore (parallel/gpu_kvstore.py): the reference's key-level KVStore API
(store/KVStore.java:109-159, 192-200, 240-277) on the parameter-server engines, driven by a
hand-written loop over raw tensors -- no nn.Module, no autograd hooks.  CPU ranks are gloo
processes; the engines are the same classes the GPU runs (ColocatedPS on the collective and on
the xGMI-protocol plane, AsyncPS for SSP/ASP).  Compared with a single-process fp32 oracle."""
import pytest
import torch

from tests import dist_util

KEYS = {"fc0.weights": (16, 12), "fc0.bias": (16,), "fc1.weights": (4, 16), "fc1.bias": (4,)}


def _init(seed=0):
    g = torch.Generator().manual_seed(seed)
    return {k: torch.randn(*s, generator=g) * 0.3 for k, s in KEYS.items()}


def _data(n=48):
    g = torch.Generator().manual_seed(11)
    return torch.randn(n, 12, generator=g), torch.randint(0, 4, (n,), generator=g)


def _loss(w, x, y):
    h = torch.tanh(x @ w["fc0.weights"].t() + w["fc0.bias"])
    return torch.nn.functional.cross_entropy(h @ w["fc1.weights"].t() + w["fc1.bias"], y)


def _grads(ws, x, y):
    w = {k: v.detach().clone().requires_grad_() for k, v in ws.items()}
    _loss(w, x, y).backward()
    return {k: v.grad for k, v in w.items()}


def _oracle(world, steps, lr=0.1, mom=0.9, staleness=0):
    x, y = _data()
    w = _init(0)
    buf = {k: torch.zeros_like(v) for k, v in w.items()}
    versions = [{k: v.clone() for k, v in w.items()}]
    for t in range(steps):
        seen = versions[max(0, t - staleness)]
        gs = [_grads(seen, x[r::world], y[r::world]) for r in range(world)]
        for k in w:
            g = sum(gr[k] for gr in gs) / world
            buf[k] = mom * buf[k] + g
            w[k] = w[k] - lr * buf[k]
        versions.append({k: v.clone() for k, v in w.items()})
    return versions[max(0, steps - staleness)] if staleness else w


def _lockstep(tp):
    """The SSP gate is a LOWER bound: a pull waits for every worker's earlier pushes but may also
    see a fast worker's NEXT push, applied in the meantime.  A collective barrier after each round
    (the pull inside ``kv.barrier()`` comes first, behind the gate) keeps the workers in lockstep,
    which with apply-on-arrival and plain SGD makes SSP(0) the BSP trajectory exactly."""
    tp.barrier()


def _kv_body(tp, consistency, plane, steps, staleness=0, style="pushpull", mom=0.9):
    from ps_amd.parallel.gpu_kvstore import GpuKVStore
    from ps_amd.parallel.updaters import MomentumUpdater, SimpleUpdater

    u = MomentumUpdater(0.1, mom) if mom else SimpleUpdater(0.1)
    kv = GpuKVStore(tp, u, consistency=consistency, staleness=staleness, device="cpu",
                    bucket_mb=0.0005, last_bucket_mb=0.0002, plane=plane, timeout_s=60)
    kv.init(_init(tp.rank))  # every rank declares; rank 0's values win (broadcast at seal)
    x, y = _data()
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    names = list(KEYS)
    for _ in range(steps):
        if style == "async":  # reference prefetch idiom: queue every key, then wait for the views
            for k in names:
                kv.async_get(k)
            ws = kv.async_wait()
        else:
            ws = dict(zip(names, kv.pull(names)))
        g = _grads(ws, xs, ys)
        if style in ("pushpull", "async"):
            kv.push(names, [g[k] for k in names])
            kv.barrier()
            if consistency == "ssp":
                _lockstep(tp)
        else:  # reference style: two half-contributions summed then averaged by update()
            for k in names:
                kv.sum(k, g[k] * 0.5)
                kv.sum(k, g[k] * 1.5)
            kv.update()
            kv.clear()
    kv.synchronize(collective=True)  # the final weights hold every worker's pushes
    out = {k: kv.get(k).detach().clone() for k in names}
    st = kv.stats()
    kv.close()
    return out, st


@pytest.mark.parametrize("plane", ["collective", "xgmi"])
def test_bsp_push_pull_barrier_matches_oracle(plane):
    res = dist_util.run(_kv_body, 2, ("bsp", plane, 4))
    want = _oracle(2, 4)
    for k in want:
        torch.testing.assert_close(res[0][0][k], want[k], rtol=1e-5, atol=1e-6)
        assert torch.equal(res[0][0][k], res[1][0][k])
    assert res[0][1]["plane_kind"] == plane


def test_reference_sum_update_clear_style_matches_oracle():
    res = dist_util.run(_kv_body, 2, ("bsp", "collective", 3, 0, "sum"))
    want = _oracle(2, 3)
    for k in want:
        torch.testing.assert_close(res[0][0][k], want[k], rtol=1e-5, atol=1e-6)


def test_ssp0_async_engine_is_bsp_exact():
    # the async owners apply every worker's push on arrival (one update per push, gradient / W):
    # with plain SGD and the SSP(0) gate that is the BSP trajectory
    res = dist_util.run(_kv_body, 2, ("ssp", None, 4, 0, "pushpull", 0.0))
    want = _oracle(2, 4, mom=0.0)
    for k in want:
        torch.testing.assert_close(res[0][0][k], want[k], rtol=1e-5, atol=1e-6)
    assert res[0][1]["engine"] == "AsyncPS"


def test_bsp_staleness1_matches_delayed_oracle():
    res = dist_util.run(_kv_body, 2, ("bsp", "collective", 5, 1))
    want = _oracle(2, 5, staleness=1)
    for k in want:
        torch.testing.assert_close(res[0][0][k], want[k], rtol=1e-5, atol=1e-6)


def test_async_get_wait_views_are_post_barrier_under_ssp1():
    """async_get / async_wait (store/KVStore.java:109-111) under SSP(1): the views they return
    must be the version the staleness gate allows after each barrier -- the delayed oracle."""
    res = dist_util.run(_kv_body, 2, ("bsp", "collective", 5, 1, "async"))
    want = _oracle(2, 5, staleness=1)
    for k in want:
        torch.testing.assert_close(res[0][0][k], want[k], rtol=1e-5, atol=1e-6)


def test_single_rank_api_semantics():
    from ps_amd.context import Stat, ctx
    from ps_amd.parallel.gpu_kvstore import GpuKVStore
    from ps_amd.parallel.updaters import SimpleUpdater

    kv = GpuKVStore(None, SimpleUpdater(0.5), device="cpu", last_bucket_mb=0)  # one bucket: w + b
    assert kv.get("w") is None  # unknown key, store open: nothing declared
    kv.init({"w": torch.ones(3), "b": ((2,), torch.float32)})
    kv.init({"w": torch.zeros(3)})  # re-declaration: first writer wins
    with pytest.raises(ValueError):
        kv.init({"w": torch.zeros(4)})
    torch.testing.assert_close(kv.get("w"), torch.ones(3))  # seals
    assert kv.get("nope") is None
    # keys may appear after the seal (reference: create on the first get(key, init)): a second
    # key group with an engine of its own
    torch.testing.assert_close(kv.get("nope", lambda: torch.zeros(1)), torch.zeros(1))
    kv.init({"late": torch.full((1,), 3.0)})
    assert "late" in kv and kv.stats()["groups"] == 2
    torch.testing.assert_close(kv.pull("late"), torch.full((1,), 3.0))
    assert kv.stats()["groups"] == 3
    # a key pushed twice in a round is summed while its bucket waits for its other key
    kv.push("w", torch.ones(3))
    kv.push("w", torch.ones(3))
    kv.push("b", torch.full((2,), 2.0))  # last key: the bucket leaves
    with pytest.raises(RuntimeError):
        kv.push("w", torch.ones(3))  # too late for this round
    kv.barrier()
    torch.testing.assert_close(kv.pull("w"), torch.zeros(3))  # 1 - 0.5 * 2
    torch.testing.assert_close(kv.pull("b"), torch.full((2,), -1.0))
    kv.barrier()  # nothing pushed: zero gradients, SGD leaves the weights
    torch.testing.assert_close(kv.pull("b"), torch.full((2,), -1.0))
    # async_get / async_wait return the current views
    kv.async_get("w")
    got = kv.async_wait()
    assert set(got) == {"w"}
    # async_get(new_key, init) after barriers creates the key (store/KVStore.java:109): async_wait
    # returns its initial value, not None
    kv.async_get("late_async", lambda: torch.full((2,), 7.0))
    kv.async_get("w")
    got = kv.async_wait()
    torch.testing.assert_close(got["late_async"], torch.full((2,), 7.0))
    assert "late_async" in kv
    # loss surface: s * w_init + (1 - s) * w
    prev = ctx.status
    ctx.status, ctx.weights_scale = Stat.LOSS_SURFACE_EVAL, 0.25
    try:
        torch.testing.assert_close(kv.get("w"), torch.full((3,), 0.25))
    finally:
        ctx.status = prev
    with pytest.raises(ValueError):
        kv.set_updaters(SimpleUpdater(0.1))
    kv.close()


def _rows_body(tp, steps):
    from ps_amd.parallel.gpu_kvstore import GpuKVStore
    from ps_amd.parallel.updaters import AdagradUpdater

    kv = GpuKVStore(tp, AdagradUpdater(0.1), device="cpu")
    kv.add_table("emb", 4, 1000, AdagradUpdater(0.1), init=(-0.1, 0.1))
    g = torch.Generator().manual_seed(tp.rank + 5)
    for _ in range(steps):
        ids = torch.randint(0, 50, (32,), generator=g)
        rows = kv.pull_rows("emb", ids)
        kv.push_rows("emb", ids, rows * 0.5 + 1.0)
    allids = torch.arange(50)
    return kv.pull_rows("emb", allids)


def _rows_oracle(world, steps):
    from ps_amd.parallel.gpu_kvstore import GpuKVStore
    from ps_amd.parallel.updaters import AdagradUpdater

    kv = GpuKVStore(None, AdagradUpdater(0.1), device="cpu")
    kv.add_table("emb", 4, 1000, AdagradUpdater(0.1), init=(-0.1, 0.1))
    gens = [torch.Generator().manual_seed(r + 5) for r in range(world)]
    for _ in range(steps):
        ids = [torch.randint(0, 50, (32,), generator=gens[r]) for r in range(world)]
        rows = [kv.pull_rows("emb", i) for i in ids]
        grads = [r * 0.5 + 1.0 for r in rows]
        kv.tables["emb"].push(torch.cat(ids), torch.cat(grads), gscale=1.0 / world)
    return kv.pull_rows("emb", torch.arange(50))


def test_rows_pull_push_two_ranks_match_single_rank():
    res = dist_util.run(_rows_body, 2, (3,))
    want = _rows_oracle(2, 3)
    torch.testing.assert_close(res[0], want, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(res[1], want, rtol=1e-5, atol=1e-6)


def _app_body(tp, steps):
    """A reference model (FullConnectedNN, fc0/fc1/fc2 keys) trained by the reference Trainer
    protocol (KVEngine: pull_into -> train -> sum_from -> update -> clear) over GpuKVStore."""
    from ps_amd.context import ctx
    from ps_amd.models.reference import FullConnectedNN
    from ps_amd.parallel.gpu_kvstore import GpuKVStore
    from ps_amd.train.trainer import CollectiveEngine, KVEngine, Trainer

    ctx.init()
    x, y = torch.randn(64, 10, generator=torch.Generator().manual_seed(1)), torch.arange(64) % 3
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    outs = []
    for kind in ("kv", "collective"):
        m = FullConnectedNN.build_model(10, [8, 3], gen=torch.Generator().manual_seed(3), softmax_temp=1.0,
                                        reference_backward=False)
        eng = KVEngine(m, GpuKVStore(tp, device="cpu", bucket_mb=0.001)) if kind == "kv" else \
            CollectiveEngine(m, tp, bucket_mb=0.001)
        tr = Trainer(m, eng)
        for _ in range(steps):
            tr.train([{"X": xs, "Y": ys}])
        tr.engine.synchronize()
        if kind == "kv":
            tr.engine.pull()
        outs.append({n: p.detach().clone() for n, p in m.named_parameters()})
        (eng.kv if kind == "kv" else eng.ps).close()
    return outs


def test_reference_model_trains_through_kvengine_on_gpu_kvstore():
    res = dist_util.run(_app_body, 2, (4,))
    kv, coll = res[0]
    for k in coll:
        torch.testing.assert_close(kv[k], coll[k], rtol=1e-5, atol=1e-6)


LATE = "late.w"


def _late_oracle(world, steps, t_new, lr=0.1, mom=0.9):
    """_oracle's model plus a key created at round t_new (rank 0's initial value 2.0) whose loss
    term is 0.1 * sum((L - 1)^2) per rank -- momentum state starting at its creation."""
    x, y = _data()
    w = _init(0)
    buf = {k: torch.zeros_like(v) for k, v in w.items()}
    for t in range(steps):
        if t == t_new:
            w[LATE] = torch.full((5,), 2.0)
            buf[LATE] = torch.zeros(5)
        gs = [_grads({k: v for k, v in w.items() if k != LATE}, x[r::world], y[r::world]) for r in range(world)]
        for k in list(w):
            g = (0.2 * (w[k] - 1.0)) if k == LATE else sum(gr[k] for gr in gs) / world
            buf[k] = mom * buf[k] + g
            w[k] = w[k] - lr * buf[k]
    return w


def _late_body(tp, consistency, plane, steps, t_new, mom=0.9):
    from ps_amd.parallel.gpu_kvstore import GpuKVStore
    from ps_amd.parallel.updaters import MomentumUpdater, SimpleUpdater

    dev = "cuda" if plane == "gpu" else "cpu"
    if dev == "cuda":
        torch.cuda.set_device(0)
    kv = GpuKVStore(tp, MomentumUpdater(0.1, mom) if mom else SimpleUpdater(0.1), consistency=consistency,
                    device=dev, bucket_mb=0.0005,
                    last_bucket_mb=0.0002, plane="xgmi" if plane == "gpu" else plane, timeout_s=60)
    kv.init({k: v.to(dev) for k, v in _init(tp.rank).items()})
    x, y = _data()
    xs, ys = x[tp.rank::tp.world].to(dev), y[tp.rank::tp.world].to(dev)
    names = list(KEYS)
    for t in range(steps):
        if t == t_new:  # a key first appears in round t_new (collective; rank 0's value wins)
            assert kv.get(LATE, lambda: torch.full((5,), 2.0 + tp.rank, device=dev)) is not None
        ws = dict(zip(names, kv.pull(names)))
        g = _grads(ws, xs, ys)
        kv.push(names, [g[k] for k in names])
        if t >= t_new:
            lw = kv.pull(LATE)
            kv.push(LATE, 0.2 * (lw - 1.0))
        kv.barrier()
        if consistency == "ssp":
            _lockstep(tp)
    kv.synchronize(collective=True)
    out = {k: kv.get(k).detach().float().cpu().clone() for k in names + [LATE]}
    st = kv.stats()
    kv.close()
    return out, st


@pytest.mark.parametrize("consistency,plane", [("bsp", "collective"), ("bsp", "xgmi"), ("ssp", None)])
def test_key_created_after_seal_matches_oracle(consistency, plane):
    """VERDICT r4 Next #6: a dense key first appears in round 3, after the store sealed -- it
    becomes a second key group (its own engine on the same ranks) and trains like the others."""
    steps, t_new = 6, 3
    # the async owners apply each worker's push on arrival (gradient / W): with plain SGD, the
    # SSP(0) gate and lockstep rounds that is the BSP trajectory (test_ssp0_async_engine_is_bsp_exact)
    mom = 0.9 if consistency == "bsp" else 0.0
    res = dist_util.run(_late_body, 2, (consistency, plane, steps, t_new, mom))
    want = _late_oracle(2, steps, t_new, mom=mom)
    for k in want:
        torch.testing.assert_close(res[0][0][k], want[k], rtol=1e-5, atol=1e-6)
        assert torch.equal(res[0][0][k], res[1][0][k])
    assert res[0][1]["groups"] == 2
