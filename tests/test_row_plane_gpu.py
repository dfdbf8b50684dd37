"""The one-node sparse-row exchange (parallel/row_plane.py) with W real PROCESSES on cuda:0:
IPC-mapped arenas, inter-process events, owner kernels that read the peers' key segments and
write rows straight into the peers' arenas (csrc/kernels/sparse.hip row_plane_*), the rank-order
accumulate + one row-optimizer update per touched row.  No RCCL (it refuses two ranks on one
GPU), no host copy of a count.  A DLRM (4 tables, row-wise Adagrad) trained by 2 and 4 processes
matches the single-rank run; the table reports the plane path and zero host syncs."""
import pytest
import torch
import torch.nn.functional as F

from tests import dist_util

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _dlrm_body(tp, n, overlap, steps=4, grow=()):
    from ps_amd.models.dlrm import DLRM, dlrm_batch
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import AdagradUpdater

    torch.cuda.set_device(0)
    rows = [700] * 4
    torch.manual_seed(0)
    inits = DLRM(dense_in=13, table_rows=rows, dim=16, bottom=(32,), top=(32, 16)).state_dict()
    m = DLRM(dense_in=13, table_rows=rows, dim=16, bottom=(32,), top=(32, 16), transport=tp, device=DEV,
             overlap=overlap)
    m.load_state_dict(inits, strict=False)
    m = m.to(DEV)
    ps = ColocatedPS(m, AdagradUpdater(0.05, 1e-8), tp, bucket_mb=0.05, overlap=False,
                     plane="collective" if tp.world == 1 else "xgmi")
    # ``grow``: batch sizes of later steps -- a larger batch after the first pushes makes every
    # rank's unique-key count outgrow the arena, i.e. a collective re-map while the peers' last
    # accumulate may still be reading the old arenas (drain + barrier before release)
    sizes = [n] * steps + list(grow)
    for i, nb in enumerate(sizes):
        dense, sparse, y = dlrm_batch(nb, rows, seed=11 + (i if grow else 0), device=DEV)
        lo, hi = tp.rank * nb // tp.world, (tp.rank + 1) * nb // tp.world
        F.binary_cross_entropy_with_logits(m(dense[lo:hi], sparse[lo:hi]), y[lo:hi]).backward()
        m.push_sparse()
        ps.finish_step()
    ps.synchronize()
    m.emb.table.synchronize()
    table_rows = m.emb.table.pull_keys(torch.arange(2800, device=DEV)).cpu()
    torch.cuda.synchronize()
    info = {"exchange": m.emb.table.exchange, "cap": m.emb.table.plane.cap if m.emb.table.plane is not None else 0,
            "plane": dict(m.emb.table.plane.stats) if m.emb.table.plane is not None else {}}
    out = ({k: v.detach().cpu() for k, v in m.named_parameters()}, table_rows, info)
    m.emb.table.close()
    ps.close()
    return out


@pytest.mark.parametrize("world,overlap", [(2, False), (2, True), (4, True)])
def test_dlrm_processes_row_plane_equals_single_rank(world, overlap):
    wn = dist_util.run(_dlrm_body, world, (256, overlap))
    w1 = dist_util.run(_dlrm_body, 1, (256, overlap))[0]
    for r in range(world):
        info = wn[r][2]
        assert info["exchange"] == "plane", info
        assert info["plane"]["host_syncs"] == 0 and info["plane"]["pushes"] >= 4, info
        for k, v in w1[0].items():
            torch.testing.assert_close(wn[r][0][k], v, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(wn[r][1], w1[1], rtol=1e-4, atol=1e-5)
        if r:
            torch.testing.assert_close(wn[r][1], wn[0][1], rtol=0, atol=0)


def test_dlrm_processes_row_plane_arena_grows_after_pushes():
    """Unique keys per rank: <= 256 for the first two steps (arena cap 1024), then up to 2800
    (4 x 700 rows, batch 4096): the arenas grow after pushes went out -- same result as one rank."""
    wn = dist_util.run(_dlrm_body, 2, (128, True, 2, (4096, 4096)))
    w1 = dist_util.run(_dlrm_body, 1, (128, True, 2, (4096, 4096)))[0]
    for r in range(2):
        info = wn[r][2]
        assert info["exchange"] == "plane" and info["plane"]["grows"] >= 2 and info["cap"] > 1024, info
        for k, v in w1[0].items():
            torch.testing.assert_close(wn[r][0][k], v, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(wn[r][1], w1[1], rtol=1e-4, atol=1e-5)
