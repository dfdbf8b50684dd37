"""1-bit Adam (parallel/updaters.py OneBitAdamUpdater + ColocatedPS onebit_momentum): full-precision
Adam for the warm-up rounds, then every worker pushes its error-compensated 1-bit MOMENTUM and the
owners run Adam with beta1 = 0 and a frozen variance.  Checked on gloo world 2, over the collective
plane and the xGMI-protocol plane, against a single-process fp32 oracle of the same algorithm
(the oracle lays the parameters out at the registry's flat offsets, so its 1024-element chunk
scales are the engine's)."""
import pytest
import torch

from tests import dist_util

LR, B1, B2, EPS = 0.01, 0.9, 0.99, 1e-8


def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(12, 24), torch.nn.Tanh(), torch.nn.Linear(24, 4))  # 412 params


def _data(n=64):
    g = torch.Generator().manual_seed(5)
    return torch.randn(n, 12, generator=g), torch.randint(0, 4, (n,), generator=g)


def _body(tp, plane, steps, warm, refresh=0):
    import torch.nn.functional as F

    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import OneBitAdamUpdater

    m = _model(seed=tp.rank)  # rank 0's broadcast wins
    u = OneBitAdamUpdater(LR, B1, B2, EPS, warmup=warm, refresh=refresh)
    ps = ColocatedPS(m, u, tp, bucket_mb=0.01, last_bucket_mb=0.01, compress="onebit", compress_warmup=warm,
                     onebit_momentum=B1, plane=plane)
    assert len({b.group for b in ps.reg.buckets}) == 1 and all(b.start % 1024 == 0 for b in ps.reg.buckets)
    layout = ({n: ps.reg.keys[n].offset for n in ps.params}, max(b.start + b.size for b in ps.reg.buckets))
    x, y = _data()
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    losses = []
    for _ in range(steps):
        loss = F.cross_entropy(m(xs), ys)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    ps.synchronize()
    return {n: p.detach().clone() for n, p in m.named_parameters()}, losses, ps.plane_kind, layout


def _oracle(steps, warm, layout, world=2, refresh=0):
    import torch.nn.functional as F

    offs, n = layout
    ref = _model(seed=0)
    named = list(ref.named_parameters())
    x, y = _data()

    def flat_grad(xb, yb):
        ref.zero_grad()
        F.cross_entropy(ref(xb), yb).backward()
        g = torch.zeros(n)
        for nm, p in named:
            g[offs[nm]:offs[nm] + p.numel()] = p.grad.reshape(-1)
        return g

    mw = [torch.zeros(n) for _ in range(world)]
    ew = [torch.zeros(n) for _ in range(world)]
    s0, s1 = torch.zeros(n), torch.zeros(n)
    for t in range(steps):
        gs = [flat_grad(x[w::world], y[w::world]) for w in range(world)]
        for w in range(world):
            mw[w] = B1 * mw[w] + (1 - B1) * gs[w]
        step = t + 1
        full = step <= warm or (refresh and (step - warm) % refresh == 0)
        nfull = step if step <= warm else warm + ((step - warm) // refresh if refresh else 0)
        if full:
            g = sum(gs) / world
            s0 = B1 * s0 + (1 - B1) * g
            s1 = B2 * s1 + (1 - B2) * g * g
            bc1 = 1 / (1 - B1 ** step) if step <= warm else 1.0
            bc2 = 1 / (1 - B2 ** nfull)
            upd = (s0 * bc1) / ((s1 * bc2).sqrt() + EPS)
        else:
            dec = []
            for w in range(world):
                c = mw[w] + ew[w]
                scale = c.abs().view(-1, 1024).mean(1).repeat_interleave(1024)  # per 1024-element chunk
                d = torch.where(c >= 0, scale, -scale)
                ew[w] = c - d
                dec.append(d)
            s0 = sum(dec) / world  # beta1 = 0: m := the decoded average of the worker momenta
            bc2 = 1 / (1 - B2 ** nfull)  # variance frozen since the last full-precision round
            upd = s0 / ((s1 * bc2).sqrt() + EPS)
        with torch.no_grad():
            for nm, p in named:
                p -= LR * upd[offs[nm]:offs[nm] + p.numel()].view_as(p)
    return {nm: p.detach() for nm, p in named}


def test_momentum_pack_op_matches_reference():
    from ps_amd.ops.compress import onebit_momentum, onebit_pack, packed_sizes

    g = torch.randn(3000)
    mom = torch.randn(3000)
    err = torch.randn(3000) * 0.1
    nw, ns = packed_sizes(3000)
    w1, s1 = torch.zeros(nw, dtype=torch.int64), torch.zeros(ns)
    m_want = 0.9 * mom + 0.1 * g
    e_ref = err.clone()
    w2, s2 = torch.zeros(nw, dtype=torch.int64), torch.zeros(ns)
    onebit_pack(m_want, e_ref, w2, s2)  # plain pack of the updated momentum
    onebit_pack(g, err, w1, s1, mom, 0.9)
    torch.testing.assert_close(mom, m_want)
    assert torch.equal(w1, w2)
    torch.testing.assert_close(s1, s2)
    torch.testing.assert_close(err, e_ref)
    m2 = mom.clone()
    onebit_momentum(g, m2, 0.5)
    torch.testing.assert_close(m2, 0.5 * mom + 0.5 * g)


def test_updater_freezes_variance_after_warmup():
    from ps_amd.parallel.updaters import AdamUpdater, OneBitAdamUpdater

    u, a = OneBitAdamUpdater(1e-3, 0.9, 0.999, warmup=5), AdamUpdater(1e-3, 0.9, 0.999)
    for s in (1, 3, 5):
        assert u.hyper(s) == a.hyper(s)
    h = u.hyper(6)
    assert h["beta1"] == 0.0 and h["beta2"] == 1.0 and h["bc1"] == 1.0 and h["bc2"] == a.hyper(5)["bc2"]
    r = OneBitAdamUpdater(1e-3, 0.9, 0.999, warmup=5, refresh=3)
    assert [r.full_round(s) for s in range(1, 13)] == [True] * 5 + [False, False, True] * 2 + [False]
    h8, h9 = r.hyper(8), r.hyper(9)  # step 8: a refresh round (live betas, v's 6th update)
    assert h8["beta1"] == 0.9 and h8["beta2"] == 0.999 and h8["bc1"] == 1.0 and h8["bc2"] == a.hyper(6)["bc2"]
    assert h9["beta1"] == 0.0 and h9["bc2"] == h8["bc2"]
    with pytest.raises(ValueError):
        OneBitAdamUpdater(warmup=0)


@pytest.mark.parametrize("plane,refresh", [("collective", 0), ("xgmi", 0), ("collective", 2), ("xgmi", 3)])
def test_onebit_adam_world2_matches_oracle(plane, refresh):
    steps, warm = 9, 3
    res = dist_util.run(_body, 2, (plane, steps, warm, refresh))
    assert res[0][2] == plane
    want = _oracle(steps, warm, res[0][3], refresh=refresh)
    for k in want:
        torch.testing.assert_close(res[0][0][k], res[1][0][k], rtol=0, atol=0)  # replicas identical
        torch.testing.assert_close(res[0][0][k], want[k], rtol=1e-4, atol=1e-5)


def test_onebit_adam_rejects_a_plain_updater():
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import AdamUpdater

    with pytest.raises(ValueError):
        ColocatedPS(_model(), AdamUpdater(), compress="onebit", compress_warmup=2, onebit_momentum=0.9)
