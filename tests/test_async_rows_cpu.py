"""Asynchronous sparse rows + per-key updaters under ASP / SSP (CPU, gloo processes).

Reference: the async server applies every push -- dense keys and every embedding / wide row --
on arrival (net/PServer.java:164-184; rows fetched with getList, store/KVStore.java:74-127), and
WideDeepNN mixes FTRL on the wide part with Adam elsewhere (model/WideDeepNN.java:109-113).
Checked: the row protocol applies every push exactly once (SGD on weight-independent
gradients: an exact sum); WideDeepNN trains under ASP and SSP(1) with FTRL + Adam per-key
segments on the owners and rows on the owners' row services; a straggler leads by at most
s + 1 rounds on the dense keys AND the rows under SSP(s), and runs away under ASP."""
import time

import pytest
import torch

from tests import dist_util
from tests.test_sparse_ps_cpu import _batches, _build


def _exact_body(tp, steps):
    from ps_amd.parallel.async_rows import AsyncRowTable
    from ps_amd.parallel.updaters import SimpleUpdater

    t = AsyncRowTable("emb", 4, 1000, tp, SimpleUpdater(0.5), init=(0.0, 0.0), staleness=None)
    keys = torch.arange(0, 40, dtype=torch.int64)
    for _ in range(steps):
        # worker r pushes gradient (r + 1) for every key: weight-independent
        t.push(keys, torch.full((40, 4), float(tp.rank + 1)))
    t.synchronize()
    tp.barrier()
    rows = t.pull(keys)
    clocks = t.clocks()
    t.close()
    return rows, clocks


def test_async_rows_apply_every_push_exactly_once():
    W, steps = 3, 7
    res = dist_util.run(_exact_body, W, (steps,))
    want = 0.0 - 0.5 / W * steps * sum(r + 1 for r in range(W))
    for rows, clocks in res:
        assert clocks == [steps] * W
        # a missing or doubled push moves a row by >= 0.5 / W; fp32 order effects are ~1e-6
        torch.testing.assert_close(rows, torch.full((40, 4), want), rtol=0, atol=1e-4)


def _wide_body(tp, consistency, staleness, steps, delay_rank=-1, delay_s=0.0):
    from ps_amd.context import ctx
    from ps_amd.parallel.async_rows import async_table_factory
    from ps_amd.train.trainer import CollectiveEngine, Trainer

    ctx.init()
    s = None if consistency == "asp" else staleness
    m = _build(True, async_table_factory(tp, None, seed=7, staleness=s))
    eng = CollectiveEngine(m, tp, consistency=consistency, staleness=staleness or 0)
    eng.ps.gate_log = []
    m.tables()["emF"].gate_log = []
    tr = Trainer(m, eng)
    n = 64
    lo, hi = tp.rank * n // tp.world, (tp.rank + 1) * n // tp.world
    losses, dlead, rlead = [], [], []
    fixed = _batches(1, n, True)[0]  # one batch, repeated: the loss must fall
    for b in [fixed] * steps:
        if tp.rank == delay_rank:
            time.sleep(delay_s)
        losses.append(tr.train([{k: v[lo:hi] for k, v in b.items()}]))
        c = eng.ps.snapshot()["clock"]
        dlead.append(c[tp.rank] - min(c))
        rc = m.tables()["emF"].clocks()
        rlead.append(rc[tp.rank] - min(rc))
    eng.ps.synchronize()
    for t in m.tables().values():
        t.synchronize()
    tp.barrier()
    eng.ps.refresh()
    dense = {k: v.detach().clone() for k, v in m.named_parameters()}
    probe = m.tables()["emF"].pull(torch.arange(40).repeat(4, 1).t().contiguous())
    segs = [u.name.split("@")[0] for u, _, _ in eng.ps.segs]
    dgates, rgates = list(eng.ps.gate_log), list(m.tables()["emF"].gate_log)
    eng.ps.close()
    for t in m.tables().values():
        t.close()
    return {"losses": losses, "dlead": dlead, "rlead": rlead, "dense": dense, "probe": probe, "segs": segs,
            "dgates": dgates, "rgates": rgates}


@pytest.mark.parametrize("consistency,staleness", [("asp", None), ("ssp", 1)])
def test_widedeep_trains_async_with_ftrl_and_adam_segments(consistency, staleness):
    res = dist_util.run(_wide_body, 2, (consistency, staleness, 12))
    for r in res:
        first, last = sum(r["losses"][:3]) / 3, sum(r["losses"][-3:]) / 3
        assert last < first, r["losses"]
    # after the final barrier + refresh every replica holds the same dense weights and rows
    for k in res[0]["dense"]:
        assert torch.equal(res[0]["dense"][k], res[1]["dense"][k])
    assert torch.equal(res[0]["probe"], res[1]["probe"])
    # the owners' dense shards carry more than one updater (FTRL wide.bias + Adam)
    assert any("ftrl" in s for r in res for s in r["segs"]) and any("adam" in s for r in res for s in r["segs"])


def test_ssp_straggler_bound_holds_on_dense_and_rows():
    s = 1
    res = dist_util.run(_wide_body, 2, ("ssp", s, 10, 1, 0.15))
    fast = res[0]
    assert max(fast["dlead"]) <= s + 1, fast["dlead"]
    assert max(fast["rlead"]) <= s + 1, fast["rlead"]


def test_ssp_dense_and_row_gates_share_one_round_window():
    """The dense weights (AsyncPS pull at the end of step k) and the rows (AsyncRowTable pull in
    step k + 1's forward) that one forward sees are gated on the SAME clock target c - s and
    both include every worker's first c - s pushes and at most this worker's c (c = rounds this
    worker pushed): one round window [c - s, c] for both views."""
    s = 1
    res = dist_util.run(_wide_body, 2, ("ssp", s, 10, 1, 0.15))
    for r in res:
        dense = {c: (t, seen) for c, t, seen in r["dgates"]}
        rows = {c: (t, seen) for c, t, seen in r["rgates"]}
        common = sorted(set(dense) & set(rows))
        assert len(common) >= 8, (r["dgates"], r["rgates"])
        for c in common:
            (td, sd), (tr, sr) = dense[c], rows[c]
            assert td == tr == c - s
            assert c - s <= sd <= c and c - s <= sr <= c, (c, sd, sr)
    # the straggler holds the fast worker at the window's lower edge: the gate was binding
    fast = res[0]
    assert any(seen == c - s for c, _, seen in fast["dgates"] if c > s)
    assert any(seen == c - s for c, _, seen in fast["rgates"] if c > s)


def test_asp_straggler_runs_ahead_on_dense_and_rows():
    res = dist_util.run(_wide_body, 2, ("asp", None, 10, 1, 0.15))
    fast = res[0]
    assert max(fast["dlead"]) >= 3, fast["dlead"]
    assert max(fast["rlead"]) >= 3, fast["rlead"]
