"""HIP sparse-path kernels vs their CPU oracles, and the sparse tables on cuda:0.

* hash_slots: device open-addressing id -> slot map (insert, lookup, duplicates inside one
  launch, misses) vs the set semantics of a dict;
* lazy_init_rows keyed by global keys == the torch Philox oracle (ops/sparse.py) bit for bit;
* sparse_opt over sorted runs (several pushes of one row merged in the kernel) == CPU oracle,
  plus the Nesterov / AdamW hyper-parameters the row path now forwards;
* SparseTable on the GPU (map / direct / hash) trains exactly like the CPU table.
"""
import pytest
import torch

from ps_amd import ops
from ps_amd.ops import sparse as S

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_hash_slots_insert_lookup_duplicates():
    cap = 1024
    hk = torch.full((cap,), -1, dtype=torch.int64, device=DEV)
    st = torch.zeros(1, dtype=torch.int32, device=DEV)
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, 1 << 40, (300,), generator=g)
    ids = torch.cat([ids, ids[:50]])  # duplicates inside one launch share a slot
    s1 = S.hash_slots(hk, ids.to(DEV), True, st).cpu()
    assert int(st.item()) == 0 and (s1 >= 0).all()
    by_id = {}
    for i, s in zip(ids.tolist(), s1.tolist()):
        assert by_id.setdefault(i, s) == s
    assert len(set(by_id.values())) == len(by_id)  # distinct ids -> distinct slots
    s2 = S.hash_slots(hk, ids.to(DEV), False, st).cpu()  # lookup-only finds every one again
    assert torch.equal(s1, s2)
    miss = S.hash_slots(hk, torch.tensor([(1 << 41) + 3], device=DEV), False, st).cpu()
    assert miss.item() == -1
    assert int((hk >= 0).sum().item()) == len(by_id)


def test_hash_slots_overflow_sets_status():
    hk = torch.full((64,), -1, dtype=torch.int64, device=DEV)
    st = torch.zeros(1, dtype=torch.int32, device=DEV)
    s = S.hash_slots(hk, torch.arange(100, device=DEV), True, st).cpu()
    assert int(st.item()) == 1 and int((s >= 0).sum()) == 64


def test_lazy_init_keys_match_cpu_philox():
    keys = torch.tensor([0, 1, 1007, (3 << 44) | 12345, (1 << 57) + 9])
    rows = torch.tensor([4, 0, 9, 2, 7])
    t = torch.zeros(10, 6, device=DEV)
    f = torch.zeros(10, dtype=torch.uint8, device=DEV)
    S.lazy_init_rows(t, rows.to(DEV), f, 1234, 0, -0.25, 0.25, keys=keys.to(DEV))
    ref = S.init_values(1234, keys, 6, -0.25, 0.25)
    assert torch.equal(t.cpu()[rows], ref)
    # range-partitioned form (key = row + row_base) agrees with the keyed form
    t2 = torch.zeros(10, 6, device=DEV)
    f2 = torch.zeros(10, dtype=torch.uint8, device=DEV)
    S.lazy_init_rows(t2, torch.tensor([7], device=DEV), f2, 1234, 1000, -0.25, 0.25)
    assert torch.equal(t2.cpu()[7], ref[2])


@pytest.mark.parametrize("kind,rowwise,extra", [(ops.ADAGRAD, True, {}), (ops.ADAM, False, {}),
                                                (ops.ADAM, False, dict(wd=0.1, adamw=True)),
                                                (ops.SGD, False, dict(momentum=0.9, nesterov=True, wd=0.01)),
                                                (ops.FTRL, False, dict(l1=0.01, l2=0.01, ftrl_mode=0))])
def test_sparse_opt_sorted_runs(kind, rowwise, extra):
    torch.manual_seed(5)
    rows_total, dim, n = 300, 12, 500
    table = torch.randn(rows_total, dim)
    slots = torch.randint(0, rows_total, (n,))
    slots[:7] = -1  # unresolved keys are skipped
    grad = torch.randn(n, dim)
    srt, perm = torch.sort(slots)
    st0 = torch.rand(rows_total) if rowwise else torch.rand(rows_total, dim)
    st1 = torch.rand(rows_total, dim) if kind in (ops.ADAM, ops.FTRL) else None
    hp = dict(lr=0.05, eps=1e-6, bc1=1.0, bc2=1.0, gscale=0.5, **extra)
    c = [x.clone() if x is not None else None for x in (table, st0, st1)]
    ops.sparse_opt(kind, c[0], c[1], c[2], srt, grad, rowwise=rowwise, perm=perm, **hp)
    g = [x.to(DEV) if x is not None else None for x in (table, st0, st1)]
    ops.sparse_opt(kind, g[0], g[1], g[2], srt.to(DEV), grad.to(DEV), rowwise=rowwise, perm=perm.to(DEV), **hp)
    torch.testing.assert_close(g[0].cpu(), c[0], rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(g[1].cpu(), c[1], rtol=2e-5, atol=2e-5)
    # rows never pushed are untouched
    untouched = torch.ones(rows_total, dtype=torch.bool)
    untouched[slots[slots >= 0]] = False
    assert torch.equal(g[0].cpu()[untouched], table[untouched])


@pytest.mark.parametrize("mode", ["map", "direct", "hash"])
def test_sparse_table_gpu_matches_cpu(mode):
    from ps_amd.parallel.sparse_table import SparseTable
    from ps_amd.parallel.updaters import AdamUpdater

    def run(dev):
        t = SparseTable("t", 8, [1000, 500], AdamUpdater(0.05), init=(-0.2, 0.2), id_mode=mode, seed=3, device=dev,
                        fields=2)
        g = torch.Generator().manual_seed(1)
        outs = []
        for step in range(4):
            ids = torch.randint(0, 400, (64, 2), generator=g)
            if mode == "map":
                ids = ids * 7919 + (1 << 35)
            rows = t.lookup(ids.to(dev))
            (rows.float().pow(2).sum() * 0.01).backward()
            t.push_pending()
            outs.append(rows.detach().cpu())
        t.synchronize()
        return outs

    for a, b in zip(run("cpu"), run(DEV)):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("mode", ["map", "direct"])
def test_sparse_table_gpu_world1_is_host_sync_free(mode):
    """W = 1 on the GPU: lookups / pushes never read a count back to the host (buffers sized by
    the host-known n, pad keys -> slot -1), and the deferred id check still fires."""
    from ps_amd.parallel.sparse_table import SparseTable
    from ps_amd.parallel.updaters import AdagradUpdater

    t = SparseTable("t", 16, [3000] * 4, AdagradUpdater(0.05, 1e-8, rowwise=True), init=(-0.1, 0.1),
                    id_mode=mode, seed=5, device=DEV, fields=4)
    g = torch.Generator().manual_seed(2)
    for _ in range(5):
        ids = torch.randint(0, 200, (128, 4), generator=g).to(DEV)  # heavy duplication
        rows = t.lookup(ids)
        (rows.float().pow(2).sum() * 0.01).backward()
        t.push_pending()
    assert t.stats["host_syncs"] == 0
    t.synchronize()
    st = t.row_stats()
    assert 0 < st["rows_pulled"] <= 5 * 4 * 200
    assert int(t.shard.status.item()) == 0  # pad keys never flag the hash map
    if mode == "direct":
        t.lookup(torch.full((4, 4), 5000, device=DEV))  # out of range: deferred, raised at the check
        with pytest.raises(IndexError):
            t.synchronize()


def test_hash_slots_pad_keys_are_silent():
    hk = torch.full((256,), -1, dtype=torch.int64, device=DEV)
    st = torch.zeros(1, dtype=torch.int32, device=DEV)
    s = S.hash_slots(hk, torch.tensor([-1, 5, -1, 7], device=DEV), True, st).cpu()
    assert s[0].item() == -1 and s[2].item() == -1 and (s[[1, 3]] >= 0).all()
    assert int(st.item()) == 0
