"""Sparse embedding / wide rows on the parameter server for the reference models (CPU).

Reference: every embedding row and every wide weight is a PS key pulled per batch and pushed
back after backward (layer/EmbeddingField.java:57-104, layer/LRLayer.java:62-120,
store/KVStore.java:74-127, net/PServer.java:143-162).  Checked here:

* co-located PS (gloo world 2, loopback world 4): DNN / WideDeepNN with rows sharded over the
  ranks train exactly like ONE process on the concatenated batch (dense AND sparse state);
* dedicated TCP servers (1 server, 2 worker processes, BSP): both workers read identical rows,
  equal to the single-process run on the concatenated batch; server-created rows equal the
  GPU/CPU lazy-init values (same Philox);
* micro-batch accumulation: n_threads=2 == one big batch, sparse tables included (one owner
  step per row per round);
* table seeds do not depend on PYTHONHASHSEED; map-mode tables resume from a checkpoint.
"""
import os
import subprocess
import sys

import pytest
import torch

from ps_amd.context import ctx
from ps_amd.data.dataset import synthetic_ctr
from ps_amd.models.reference import DNN, WideDeepNN, local_table_factory, sharded_table_factory
from ps_amd.parallel.transport import run_loopback
from ps_amd.train.trainer import CollectiveEngine, Trainer

from . import dist_util

FIELDS, DIM, NUM = 4, 4, 6


def _build(wide, tf):
    gen = torch.Generator().manual_seed(0)
    if wide:
        return WideDeepNN.build_model(FIELDS, DIM, NUM, [12, 6, 1], 500, gen=gen, emb_rows=256, table_factory=tf,
                                      init_scale=0.2)
    return DNN.build_model(FIELDS, DIM, NUM, [12, 6, 1], gen=gen, emb_rows=256, table_factory=tf, init_scale=0.2)


def _batches(steps, n, wide):
    return [synthetic_ctr(n, fields=FIELDS, numeric=NUM, ids_per_field=40, wide_k=3 if wide else 0, wide_size=500,
                          seed=77 + i) for i in range(steps)]


def _probe(m, wide):
    ids = torch.arange(40).repeat(FIELDS, 1).t().contiguous()  # every id of every field
    out = {"emF": m.tables()["emF"].pull(ids)}
    if wide:
        out["wide"] = m.tables()["wide.weights"].pull(torch.arange(500))
    return out


def _train_sharded(tp, wide, steps, n):
    ctx.init()
    m = _build(wide, sharded_table_factory(tp, None, seed=7))
    tr = Trainer(m, CollectiveEngine(m, tp, bucket_mb=0.001))
    lo, hi = tp.rank * n // tp.world, (tp.rank + 1) * n // tp.world
    for b in _batches(steps, n, wide):
        tr.train([{k: v[lo:hi] for k, v in b.items()}])
    dense = {k: v.detach().clone() for k, v in m.named_parameters()}
    return dense, _probe(m, wide)


def _train_single(wide, steps, n):
    ctx.init()
    m = _build(wide, local_table_factory(seed=7))
    tr = Trainer(m, CollectiveEngine(m, bucket_mb=0.001))
    for b in _batches(steps, n, wide):
        tr.train([b])
    return {k: v.detach().clone() for k, v in m.named_parameters()}, _probe(m, wide)


def _assert_same(a, b, tol=2e-5):
    (da, pa), (db, pb) = a, b
    for k in da:
        torch.testing.assert_close(da[k], db[k], rtol=tol, atol=tol)
    for k in pa:
        torch.testing.assert_close(pa[k], pb[k], rtol=tol, atol=tol)


@pytest.mark.parametrize("wide", [False, True])
def test_sharded_rows_gloo_world2_equal_single_process(wide):
    res = dist_util.run(_train_sharded, 2, (wide, 4, 64))
    single = _train_single(wide, 4, 64)
    _assert_same(res[0], res[1], 1e-6)  # both ranks see the same dense weights and rows
    _assert_same(res[0], single)


def test_sharded_rows_loopback_world4_equal_single_process():
    res = run_loopback(_train_sharded, 4, True, 3, 64)
    single = _train_single(True, 3, 64)
    for r in range(4):
        _assert_same(res[r], single)


def test_sharded_rows_nonpow2_world3():
    res = dist_util.run(_train_sharded, 3, (False, 3, 60))
    _assert_same(res[0], res[2], 1e-6)
    _assert_same(res[0], _train_single(False, 3, 60))


def test_microbatch_accumulation_equals_big_batch_with_sparse_rows():
    ctx.init()
    batches = _batches(3, 64, True)
    m1 = _build(True, local_table_factory(seed=7))
    tr1 = Trainer(m1, CollectiveEngine(m1, bucket_mb=0.001), n_threads=2)
    for b in batches:
        tr1.train([{k: v[:32] for k, v in b.items()}, {k: v[32:] for k, v in b.items()}])
    a = ({k: v.detach().clone() for k, v in m1.named_parameters()}, _probe(m1, True))
    assert m1.tables()["emF"].round == 3  # ONE owner step per round, not one per micro-batch
    _assert_same(a, _train_single(True, 3, 64))


# ----------------------------------------------------------------------------- TCP servers
def _tcp_worker(wid, port, steps, n, q):
    os.environ["PS_AMD_WORKER_ID"] = str(wid)
    torch.set_num_threads(1)
    from ps_amd.context import ctx as c
    from ps_amd.models.reference import tcp_table_factory
    from ps_amd.parallel.kvstore import KVStore
    from ps_amd.parallel.tcp import PSRouterClient
    from ps_amd.train.trainer import KVEngine, Trainer as T

    c.init()
    client = PSRouterClient([f"127.0.0.1:{port}"])
    m = _build(True, tcp_table_factory(client, seed=7))
    tr = T(m, KVEngine(m, KVStore(client, worker_id=wid, consistency="bsp")))
    lo, hi = wid * n // 2, (wid + 1) * n // 2
    for b in _batches(steps, n, True):
        tr.train([{k: v[lo:hi] for k, v in b.items()}])
    tr.engine.pull()  # final weights from the servers
    dense = {k: v.detach().clone().numpy() for k, v in m.named_parameters()}
    probe = {k: v.numpy() for k, v in _probe(m, True).items()}
    q.put((wid, dense, probe))


def test_tcp_rows_two_workers_identical_and_equal_single_process():
    import multiprocessing as mp

    from ps_amd.parallel.tcp import PServer

    srv = PServer(0, workers=2, mode="bsp").start()
    try:
        mpc = mp.get_context("spawn")
        q = mpc.Queue()
        ps = [mpc.Process(target=_tcp_worker, args=(w, srv.port, 3, 64, q)) for w in range(2)]
        for p in ps:
            p.start()
        got = sorted(q.get(timeout=300) for _ in ps)
        for p in ps:
            p.join(60)
    finally:
        srv.stop()
    res = [({k: torch.from_numpy(v) for k, v in d.items()}, {k: torch.from_numpy(v) for k, v in pr.items()})
           for _, d, pr in got]
    _assert_same(res[0], res[1], 1e-6)
    _assert_same(res[0], _train_single(True, 3, 64), 1e-4)


def test_tcp_server_rows_use_the_gpu_init_values():
    from ps_amd.ops.sparse import init_values
    from ps_amd.parallel.tcp import PSClient, PServer

    srv = PServer(0, workers=1).start()
    try:
        c = PSClient("127.0.0.1", srv.port)
        keys = torch.tensor([0, 5, 1 << 40, 123456789])
        rows = c.row_pull("t", 6, keys, -0.3, 0.3, seed=99)
        torch.testing.assert_close(rows, init_values(99, keys, 6, -0.3, 0.3), rtol=0, atol=0)
        again = c.row_pull("t", 6, keys, -0.3, 0.3, seed=99)
        assert torch.equal(rows, again)
        c.row_push("t", 6, keys[:2], torch.ones(2, 6), "simple@eta:0.5@", apply_now=True)
        after = c.row_pull("t", 6, keys, -0.3, 0.3, seed=99)
        torch.testing.assert_close(after[:2], rows[:2] - 0.5)
        torch.testing.assert_close(after[2:], rows[2:])
    finally:
        srv.stop()


# ----------------------------------------------------------------------------- seeds / ckpt
_SEED_CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from ps_amd.models.reference import DNN, local_table_factory
m = DNN.build_model(3, 4, 2, [4, 1], emb_rows=64, table_factory=local_table_factory(seed=5))
print(m.tables()["emF"].pull(torch.tensor([[1, 2, 3], [4, 5, 6]])).sum().item())
"""


def test_table_init_independent_of_python_hash_seed():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for hs in ("1", "2"):
        env = dict(os.environ, PYTHONHASHSEED=hs)
        r = subprocess.run([sys.executable, "-c", _SEED_CHILD, root], env=env, capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        outs.append(r.stdout.strip().splitlines()[-1])
    assert outs[0] == outs[1]


def test_map_mode_checkpoint_resume(tmp_path):
    from ps_amd.parallel.sparse_table import SparseTable
    from ps_amd.parallel.updaters import AdamUpdater
    from ps_amd.utils.checkpoint import CheckpointManager

    def make():
        return SparseTable("t", 3, 100, AdamUpdater(0.1), init=(-0.1, 0.1), id_mode="map", seed=1)

    a = make()
    a.push(torch.tensor([900, 7, 123456]), torch.ones(3, 3))
    ck = CheckpointManager(str(tmp_path))
    ck.save(1, None, {"t": a}, blocking=True)
    b = make()
    CheckpointManager(str(tmp_path)).load(None, None, {"t": b})
    for t in (a, b):  # new ids after the resume must not alias trained rows
        t.push(torch.tensor([55, 7]), torch.full((2, 3), 2.0))
    probe = torch.tensor([900, 7, 123456, 55, 4242])
    assert torch.equal(a.pull(probe), b.pull(probe))
    assert not torch.equal(b.pull(torch.tensor([55])), b.pull(torch.tensor([900])))


def test_lazy_init_fields_with_same_id_get_independent_rows():
    # map-mode keys are field << 44 | id: the Philox counter carries the whole key (128-bit
    # counter), so the same raw id in two fields must not start from the same vector
    from ps_amd.ops.sparse import init_values

    keys = torch.tensor([(0 << 44) | 5, (1 << 44) | 5, (2 << 44) | 5, 5 + (1 << 20)], dtype=torch.int64)
    rows = init_values(7, keys, 8, -0.5, 0.5)
    for i in range(len(keys)):
        for j in range(i + 1, len(keys)):
            assert not torch.allclose(rows[i], rows[j])


def _prefetch_body(tp, use_prefetch):
    from ps_amd.parallel.sparse_table import ShardedSparseTable
    from ps_amd.parallel.updaters import AdagradUpdater

    t = ShardedSparseTable("emb", 8, [500] * 3, tp, AdagradUpdater(0.05, 1e-8, rowwise=True), init=(-0.1, 0.1),
                           seed=4, fields=3)
    g = torch.Generator().manual_seed(10 + tp.rank)
    batches = [torch.randint(0, 500, (32, 3), generator=g) for _ in range(5)]
    outs = []
    if use_prefetch:
        t.prefetch(batches[0])
    for i, ids in enumerate(batches):
        if use_prefetch and i + 1 < len(batches):
            t.prefetch(batches[i + 1])  # routed a step ahead (counts exchanged now)
        rows = t.lookup(ids)
        (rows.pow(2).sum() * 0.01).backward()
        t.push_pending()
        outs.append(rows.detach().clone())
    t.synchronize()
    left = len(t._pf)
    return outs, t.pull(torch.arange(500).repeat(3, 1).t().contiguous()), left


def test_prefetched_routing_matches_inline_routing_gloo_world2():
    a = dist_util.run(_prefetch_body, 2, (False,))
    b = dist_util.run(_prefetch_body, 2, (True,))
    for (oa, ta, _), (ob, tb, left) in zip(a, b):
        assert left == 0  # every prefetched route was consumed by its lookup
        for x, y in zip(oa, ob):
            assert torch.equal(x, y)
        assert torch.equal(ta, tb)
