"""The xGMI plane's protocol on CPU: the native engine (csrc/plane.cpp) drives the one-sided
push / serve / pull state machine over a /dev/shm control block between real gloo processes
(and between loopback thread-ranks), with Python callbacks standing in for the kernels.
Compared with single-process oracles: BSP, SSP(1), global-norm clipping, 1-bit pushes (vs the
collective 1-bit path), a straggler, and checkpoint restore."""
import copy

import pytest
import torch
import torch.nn.functional as F

from ps_amd.parallel.transport import run_loopback
from tests import dist_util


def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(12, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))


def _data(n=60):
    g = torch.Generator().manual_seed(7)
    return torch.randn(n, 12, generator=g), torch.randint(0, 4, (n,), generator=g)


def _body(tp, kw, steps, upd="momentum", plane="xgmi", seed_per_rank=True, fault=None, models=None):
    import os

    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import AdamUpdater, MomentumUpdater, SimpleUpdater

    if fault is not None and tp.rank == fault[0]:
        os.environ["PS_AMD_FAULT"] = fault[1]
    # thread-ranks share the global RNG: they get models built beforehand
    m = models[tp.rank] if models is not None else _model(seed=tp.rank if seed_per_rank else 0)
    u = {"momentum": lambda: MomentumUpdater(0.1, 0.9, 1e-4), "sgd": lambda: SimpleUpdater(0.2),
         "mixed": lambda: {"0.": AdamUpdater(0.01), "default": MomentumUpdater(0.1, 0.9)}}[upd]()
    ps = ColocatedPS(m, u, tp, bucket_mb=0.001, last_bucket_mb=0.0005, plane=plane, timeout_s=60, **kw)
    x, y = _data()
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    losses = []
    for _ in range(steps):
        loss = F.cross_entropy(m(xs), ys)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    ps.synchronize()
    out = {n: p.detach().clone() for n, p in m.named_parameters()}
    kind = ps.plane_kind
    st = ps.plane_stats()
    ps.close()
    return out, losses, kind, st


def _oracle(world, steps, opt_factory, clip=None):
    ref = _model(0)
    opt = opt_factory(ref.parameters())
    x, y = _data()
    for _ in range(steps):
        opt.zero_grad()
        (sum(F.cross_entropy(ref(x[r::world]), y[r::world]) for r in range(world)) / world).backward()
        if clip is not None:
            torch.nn.utils.clip_grad_norm_(ref.parameters(), clip)
        opt.step()
    return {n: p.detach() for n, p in ref.named_parameters()}


@pytest.mark.parametrize("world", [2, 3])
def test_plane_bsp_processes_equal_single_process(world):
    res = dist_util.run(_body, world, ({}, 4))
    assert res[0][2] == "xgmi"
    for r in range(1, world):
        for k in res[0][0]:
            assert torch.equal(res[0][0][k], res[r][0][k])
    ref = _oracle(world, 4, lambda p: torch.optim.SGD(p, lr=0.1, momentum=0.9, weight_decay=1e-4))
    for k, v in ref.items():
        torch.testing.assert_close(res[0][0][k], v, rtol=1e-5, atol=1e-6)
    assert res[0][3]["rounds"] >= 1


def test_plane_mixed_updaters_loopback_world4():
    # per-key-prefix updaters: Adam on the first Linear, momentum elsewhere (segments per bucket)
    res = run_loopback(_body, 4, {}, 5, "mixed", "xgmi", False, None, [_model(r) for r in range(4)])
    ref = _model(0)
    opts = [torch.optim.Adam(ref[0].parameters(), lr=0.01, eps=1e-8),
            torch.optim.SGD(ref[2].parameters(), lr=0.1, momentum=0.9)]
    x, y = _data()
    for _ in range(5):
        for o in opts:
            o.zero_grad()
        (sum(F.cross_entropy(ref(x[r::4]), y[r::4]) for r in range(4)) / 4).backward()
        for o in opts:
            o.step()
    for n, p in ref.named_parameters():
        torch.testing.assert_close(res[0][0][n], p.detach(), rtol=1e-5, atol=1e-5)
        assert torch.equal(res[0][0][n], res[3][0][n])


def test_plane_ssp1_matches_delayed_sgd():
    world, steps, lr, s = 2, 6, 0.2, 1
    res = dist_util.run(_body, world, ({"staleness": s}, steps, "sgd", "xgmi", False))
    ref = _model(0)
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
        torch.testing.assert_close(res[0][0][k], want[k], rtol=1e-5, atol=1e-6)


def test_plane_clip_norm_processes():
    world = 2
    res = dist_util.run(_body, world, ({"clip_norm": 0.05}, 4, "sgd", "xgmi", False))
    ref = _oracle(world, 4, lambda p: torch.optim.SGD(p, lr=0.2), clip=0.05)
    for k, v in ref.items():
        torch.testing.assert_close(res[0][0][k], v, rtol=1e-5, atol=1e-6)


def test_plane_onebit_equals_collective_onebit():
    kw = {"compress": "onebit", "compress_warmup": 1}
    a = run_loopback(_body, 2, kw, 6, "momentum", "xgmi", False, None, [_model(0), _model(1)])
    b = run_loopback(_body, 2, kw, 6, "momentum", "collective", False, None, [_model(0), _model(1)])
    assert a[0][2] == "xgmi" and b[0][2] == "collective"
    for k in a[0][0]:
        torch.testing.assert_close(a[0][0][k], b[0][0][k], rtol=1e-6, atol=1e-6)
        assert torch.equal(a[0][0][k], a[1][0][k])


def test_plane_straggler_still_bsp_exact():
    # rank 1 sleeps before every push: the fast rank must wait in the plane, not race ahead
    res = dist_util.run(_body, 2, ({}, 3, "momentum", "xgmi", True, (1, "delay_push:ms=150")))
    ref = _oracle(2, 3, lambda p: torch.optim.SGD(p, lr=0.1, momentum=0.9, weight_decay=1e-4))
    for k, v in ref.items():
        torch.testing.assert_close(res[0][0][k], v, rtol=1e-5, atol=1e-6)


def _ckpt_body(tp, steps, kw=None):
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import MomentumUpdater

    def make():
        m = _model(0)
        return m, ColocatedPS(m, MomentumUpdater(0.1, 0.9), tp, bucket_mb=0.001, last_bucket_mb=0.0005, plane="xgmi",
                              timeout_s=20, **(kw or {}))

    x, y = _data()
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]

    def run(m, ps, n):
        for _ in range(n):
            F.cross_entropy(m(xs), ys).backward()
            ps.finish_step()
        ps.synchronize()

    m1, ps1 = make()
    run(m1, ps1, steps)
    st = ps1.shard_state()
    run(m1, ps1, steps)
    want = {n: p.detach().clone() for n, p in m1.named_parameters()}
    ps1.close()
    m2, ps2 = make()
    ps2.load_shard_state(st)
    run(m2, ps2, steps)
    got = {n: p.detach().clone() for n, p in m2.named_parameters()}
    ps2.close()
    return want, got


def test_plane_checkpoint_restore_processes():
    res = dist_util.run(_ckpt_body, 2, (3,))
    for want, got in res:
        for k in want:
            assert torch.equal(want[k], got[k])


def test_plane_checkpoint_restore_with_clipping_processes():
    """a restore at round R >= 2 with global-norm clipping used to hang in the
    first clip phase (fdone >= R - 1 on a fresh control block) and abort after timeout_s.  The
    engine now marks its control words as of round R (plane.cpp restore_round)."""
    res = dist_util.run(_ckpt_body, 2, (3, {"clip_norm": 0.05}))
    for want, got in res:
        for k in want:
            assert torch.equal(want[k], got[k])


def test_plane_clip_ssp1_straggler_matches_delayed_clipped_sgd():
    """clipping + staleness 1 with a straggler.  Round r+1 must not reduce
    into the bucket's one fp32 gradient buffer while round r still waits for its clip factor;
    the result equals delayed SGD on the clipped averaged gradient."""
    world, steps, lr, s, clip = 2, 6, 0.2, 1, 0.05
    res = dist_util.run(_body, world, ({"staleness": s, "clip_norm": clip}, steps, "sgd", "xgmi", False,
                                       (1, "delay_push:ms=60")))
    ref = _model(0)
    x, y = _data()
    versions = [{n: p.detach().clone() for n, p in ref.named_parameters()}]
    for t in range(steps):
        probe = copy.deepcopy(ref)
        with torch.no_grad():
            for n, p in probe.named_parameters():
                p.copy_(versions[max(0, t - s)][n])
        loss = sum(F.cross_entropy(probe(x[r::world]), y[r::world]) for r in range(world)) / world
        grads = torch.autograd.grad(loss, list(probe.parameters()))
        tot = torch.sqrt(sum((g.double() ** 2).sum() for g in grads)).float()
        f = min(1.0, clip / (float(tot) + 1e-6))
        versions.append({n: versions[-1][n] - lr * f * g for (n, _), g in zip(probe.named_parameters(), grads)})
    want = versions[max(0, steps - s)]
    for k in want:
        torch.testing.assert_close(res[0][0][k], want[k], rtol=1e-5, atol=1e-6)
        assert torch.equal(res[0][0][k], res[1][0][k])
