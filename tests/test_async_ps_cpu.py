"""Asynchronous parameter server (ASP / SSP without lockstep collectives) on CPU.

Reference: async pushes are applied on arrival and the barrier returns at once
(net/PServer.java:176-184, 242-248).  Checked: SSP(0) with SGD equals synchronous data
parallelism exactly (W sequential updates of g_w / W == one averaged step); with a straggler the
fast worker's clock leads by at most s + 1 under SSP(s) and runs away under ASP; ASP still
converges.  Thread-ranks (loopback) and real processes (gloo + POSIX shared memory, native
progress threads) both run."""
import time

import pytest
import torch
import torch.nn.functional as F

from ps_amd.parallel.transport import run_loopback

from . import dist_util


def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(10, 24), torch.nn.Tanh(), torch.nn.Linear(24, 3))


def _data(n=48):
    g = torch.Generator().manual_seed(3)
    return torch.randn(n, 10, generator=g), torch.randint(0, 3, (n,), generator=g)


def _body(tp, staleness, steps, lr, delay_rank=-1, delay_s=0.0, models=None):
    from ps_amd.parallel.async_ps import AsyncPS
    from ps_amd.parallel.updaters import SimpleUpdater

    m = models[tp.rank] if models is not None else _model(0)  # thread-ranks: built outside (global RNG)
    ps = AsyncPS(m, SimpleUpdater(lr), tp, staleness=staleness)
    x, y = _data()
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    leads, losses = [], []
    for _ in range(steps):
        if tp.rank == delay_rank:
            time.sleep(delay_s)
        loss = F.cross_entropy(m(xs), ys)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
        c = ps.snapshot()["clock"]
        leads.append(c[tp.rank] - min(c))
    ps.synchronize()
    tp.barrier()
    ps.refresh()  # every rank's pushes are applied: all replicas read the same final version
    out = {n: p.detach().clone() for n, p in m.named_parameters()}
    ps.close()
    return out, leads, losses


def _oracle(world, steps, lr):
    ref = _model(0)
    opt = torch.optim.SGD(ref.parameters(), lr=lr)
    x, y = _data()
    for _ in range(steps):
        opt.zero_grad()
        (sum(F.cross_entropy(ref(x[r::world]), y[r::world]) for r in range(world)) / world).backward()
        opt.step()
    return {n: p.detach() for n, p in ref.named_parameters()}


def test_single_worker_is_plain_sgd():
    res = run_loopback(_body, 1, 0, 5, 0.2, -1, 0.0, [_model(0)])
    for k, v in _oracle(1, 5, 0.2).items():
        torch.testing.assert_close(res[0][0][k], v, rtol=1e-6, atol=1e-7)


def _close_to_sync(res, world, steps, lr):
    # SSP(0) reads AT LEAST every update of the previous clock (it may also see a faster
    # worker's newer push), so it tracks synchronous SGD closely but not bitwise
    ref = _oracle(world, steps, lr)
    for r in range(world):
        for k, v in ref.items():
            assert torch.equal(res[r][0][k], res[0][0][k])  # identical replicas at the end
            torch.testing.assert_close(res[r][0][k], v, rtol=0, atol=5e-3)


def test_ssp0_threads_tracks_sync_sgd():
    _close_to_sync(run_loopback(_body, 3, 0, 5, 0.2, -1, 0.0, [_model(0) for _ in range(3)]), 3, 5, 0.2)


def test_ssp0_processes_tracks_sync_sgd():
    _close_to_sync(dist_util.run(_body, 2, (0, 6, 0.2)), 2, 6, 0.2)


@pytest.mark.parametrize("s", [1, 2])
def test_ssp_bound_with_straggler(s):
    res = dist_util.run(_body, 2, (s, 12, 0.1, 1, 0.05))
    assert max(res[0][1]) <= s + 1, res[0][1]  # the fast rank never runs further ahead
    assert max(res[0][1]) >= s  # ... but it does use the slack


def test_asp_runs_ahead_and_converges():
    res = dist_util.run(_body, 2, (None, 20, 0.1, 1, 0.05))
    assert max(res[0][1]) > 3, res[0][1]  # no bound: the fast worker runs away
    assert res[0][2][-1] < res[0][2][0]


def _bert_body(tp, staleness, steps):
    from ps_amd.models.transformer import BertConfig, BertForMLM
    from ps_amd.parallel.async_ps import AsyncPS
    from ps_amd.parallel.updaters import AdamUpdater

    torch.manual_seed(0)
    c = BertConfig(vocab=128, hidden=64, layers=2, heads=4, ffn=128, max_pos=64, dropout=0.0)
    m = BertForMLM(c)
    ps = AsyncPS(m, AdamUpdater(1e-2, 0.9, 0.999, 1e-6, bias_correction="step", weight_decay=0.01), tp,
                 staleness=staleness)
    # a learnable language: a random first-order Markov chain over a Zipf-skewed vocabulary
    tg = torch.Generator().manual_seed(7)
    prior = -1.5 * torch.log(torch.arange(1, c.vocab + 1).float())
    trans = torch.softmax(torch.randn(c.vocab, c.vocab, generator=tg) * 2.0 + prior, dim=1)
    g = torch.Generator().manual_seed(100 + tp.rank)
    losses = []
    for _ in range(steps):
        ids = torch.empty(16, 32, dtype=torch.long)
        ids[:, 0] = torch.randint(0, c.vocab, (16,), generator=g)
        for t in range(1, 32):
            ids[:, t] = torch.multinomial(trans[ids[:, t - 1]], 1, generator=g).squeeze(1)
        pos = torch.stack([torch.randperm(31, generator=g)[:5] + 1 for _ in range(16)])  # 5 masked per sequence
        labels = torch.full_like(ids, -100)
        labels.scatter_(1, pos, ids.gather(1, pos))
        inp = ids.scatter(1, pos, 0)  # token 0 = [MASK]
        loss = m(inp, labels, pos)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    ps.synchronize()
    ps.close()
    return losses


def test_tiny_bert_converges_on_async_ssp1():
    """the BERT config's semantics (SSP s=1 on the asynchronous PS) train a
    tiny BERT MLM on a learnable synthetic language (gloo world 2).  Calibration: plain
    single-process torch AdamW on the same model / data goes 3.64 -> 3.25 (first vs last 10
    steps) in 80 steps."""
    res = dist_util.run(_bert_body, 2, (1, 80))
    for losses in res:
        first, last = sum(losses[:10]) / 10, sum(losses[-10:]) / 10
        assert last < first - 0.25, (first, last)


def _ckpt_body(tp, path, phase):
    from ps_amd.parallel.async_ps import AsyncPS
    from ps_amd.parallel.updaters import AdamUpdater

    m = _model(0)
    ps = AsyncPS(m, AdamUpdater(0.05, bias_correction="reference"), tp, staleness=0)
    x, y = _data()
    xs, ys = x[tp.rank::tp.world], y[tp.rank::tp.world]
    if phase == 1:
        ps.load_shard_state(torch.load(f"{path}.{tp.rank}", weights_only=True))
    for _ in range(3):
        F.cross_entropy(m(xs), ys).backward()
        ps.finish_step()
    st = ps.shard_state()
    if phase == 0:
        torch.save(st, f"{path}.{tp.rank}")
    ps.synchronize()
    tp.barrier()
    ps.refresh()
    out = {n: p.detach().clone() for n, p in m.named_parameters()}
    ps.close()
    return out, st["master"], st["states"]


def test_async_ps_checkpoint_resume(tmp_path):
    """Save the owners' shards (master + Adam state) after 3 steps, resume fresh processes from
    them: shard state after the resumed steps equals a second save of an uninterrupted run."""
    p = str(tmp_path / "ck")
    a = dist_util.run(_ckpt_body, 2, (p, 0))
    b = dist_util.run(_ckpt_body, 2, (p, 1))
    for r in range(2):
        for s0, s1 in zip(a[r][2], b[r][2]):
            assert s0.shape == s1.shape
        # the resumed run continued from the saved state: its moments moved on from there
        assert not torch.equal(a[r][1], b[r][1])
        assert torch.isfinite(b[r][1]).all()


def _resume_parity_body(tp, split):
    """6 Adam(bias_correction="step") steps, either straight through or 3 + checkpoint + a
    FRESH AsyncPS (new control block) restored from it + 3."""
    from ps_amd.parallel.async_ps import AsyncPS
    from ps_amd.parallel.updaters import AdamUpdater

    x, y = _data()

    def run(ps, m, n):
        for _ in range(n):
            F.cross_entropy(m(x), y).backward()
            ps.finish_step()

    m = _MODELS[0]
    ps = AsyncPS(m, AdamUpdater(0.05, bias_correction="step"), tp, staleness=0)
    run(ps, m, 3 if split else 6)
    st = ps.shard_state()
    ps.close()
    if split:
        ps = AsyncPS(m, AdamUpdater(0.05, bias_correction="step"), tp, staleness=0)
        ps.load_shard_state(st)
        run(ps, m, 3)
        st = ps.shard_state()
        ps.close()
    return st


_MODELS = None


def test_async_resume_restores_adam_step_count():
    """the owner's update count (Adam's t) is part of the shard state; a resumed
    owner must continue at t = 4, not restart bias correction at t = 1 on warm moments."""
    global _MODELS
    _MODELS = [_model(0)]
    a = run_loopback(_resume_parity_body, 1, False)[0]
    _MODELS = [_model(0)]
    b = run_loopback(_resume_parity_body, 1, True)[0]
    assert a["version"] == b["version"] == 6
    torch.testing.assert_close(a["master"], b["master"], rtol=0, atol=0)
