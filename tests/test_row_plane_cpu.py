"""One-node sparse row exchange over the shared-memory row plane (row_plane.py), CPU / gloo.

Reference semantics: each batch's rows are pulled from their owner servers and the row
gradients pushed back (layer/EmbeddingField.java:57-104, store/KVStore.java:74-127,
net/PServer.java:143-162).  The plane replaces the count + key + row all-to-alls with owner
reads of the workers' key segments; checked here:

* ``exchange == "plane"`` is the auto default on one host, with zero host syncs on the plane;
* plane and collective exchanges give the same dense weights and rows, both equal to ONE
  process on the concatenated batch (W = 2 and the non-power-of-two W = 3);
* micro-batch accumulation (n_threads = 2) through the plane accumulator == one big batch.
"""
import pytest
import torch

from ps_amd.context import ctx
from ps_amd.models.reference import WideDeepNN, local_table_factory, sharded_table_factory
from ps_amd.train.trainer import CollectiveEngine, Trainer

from . import dist_util
from .test_sparse_ps_cpu import FIELDS, DIM, NUM, _assert_same, _batches, _build, _probe


def _train(tp, exchange, steps, n, threads):
    ctx.init()
    m = _build(True, sharded_table_factory(tp, None, seed=7, exchange=exchange))
    tabs = m.tables()
    tr = Trainer(m, CollectiveEngine(m, tp, bucket_mb=0.001), n_threads=threads)
    lo, hi = tp.rank * n // tp.world, (tp.rank + 1) * n // tp.world
    for b in _batches(steps, n, True):
        mine = {k: v[lo:hi] for k, v in b.items()}
        if threads == 1:
            tr.train([mine])
        else:
            h = (hi - lo) // 2
            tr.train([{k: v[:h] for k, v in mine.items()}, {k: v[h:] for k, v in mine.items()}])
    info = {k: (t.exchange, t.plane.stats["host_syncs"] if t.plane is not None else -1, t.round)
            for k, t in tabs.items()}
    dense = {k: v.detach().clone() for k, v in m.named_parameters()}
    return dense, _probe(m, True), info


def _single(steps, n):
    ctx.init()
    m = _build(True, local_table_factory(seed=7))
    tr = Trainer(m, CollectiveEngine(m, bucket_mb=0.001))
    for b in _batches(steps, n, True):
        tr.train([b])
    return {k: v.detach().clone() for k, v in m.named_parameters()}, _probe(m, True)


@pytest.mark.parametrize("world", [2, 3])
def test_plane_and_collective_exchange_equal_single_process(world):
    steps, n = 3, 60
    plane = dist_util.run(_train, world, (None, steps, n, 1))
    coll = dist_util.run(_train, world, ("collective", steps, n, 1))
    single = _single(steps, n)
    for r in range(world):
        for name, (ex, syncs, rnd) in plane[r][2].items():
            assert ex == "plane", name
            assert syncs == 0, name
            assert rnd == steps, name
        assert all(ex == "collective" for ex, _, _ in coll[r][2].values())
        _assert_same(plane[r][:2], coll[r][:2], 1e-6)
        _assert_same(plane[r][:2], single)


def test_plane_microbatch_accumulation_equals_big_batch():
    steps, n = 3, 64
    res = dist_util.run(_train, 2, ("plane", steps, n, 2))
    single = _single(steps, n)
    for r in range(2):
        assert all(rnd == steps for _, _, rnd in res[r][2].values())  # one owner step per round
        _assert_same(res[r][:2], single)


def _timed(tp, steps, n):
    import os

    os.environ["PS_AMD_ROWPLANE_TIMING"] = "1"
    ctx.init()
    m = _build(True, sharded_table_factory(tp, None, seed=7))
    tabs = m.tables()
    tr = Trainer(m, CollectiveEngine(m, tp, bucket_mb=0.001))
    lo, hi = tp.rank * n // tp.world, (tp.rank + 1) * n // tp.world
    for b in _batches(steps, n, True):
        tr.train([{k: v[lo:hi] for k, v in b.items()}])
    return {k: t.plane.timing_summary() for k, t in tabs.items()}


def test_plane_stage_timing_table():
    """Per-stage table of the row plane (VERDICT r4 Next #3): every stage timed, host waits at
    each cross-rank point, bytes per pull / push."""
    res = dist_util.run(_timed, 2, (3, 40))
    for r in range(2):
        for name, tm in res[r].items():
            assert tm["pulls"] >= 3 and tm["pushes"] >= 3 and tm["applies"] >= 3, (name, tm)
            for k in ("pub_ms", "serve_ms", "out_ms", "grd_ms", "wait_pub_ms", "wait_rows_ms", "wait_grd_ms",
                      "pull_bytes", "push_bytes"):
                assert k in tm and tm[k] >= 0, (name, k, tm)
