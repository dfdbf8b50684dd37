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


def _dlrm_body(tp, n, overlap, steps=4):
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
    dense, sparse, y = dlrm_batch(n, rows, seed=11, device=DEV)
    lo, hi = tp.rank * n // tp.world, (tp.rank + 1) * n // tp.world
    for _ in range(steps):
        F.binary_cross_entropy_with_logits(m(dense[lo:hi], sparse[lo:hi]), y[lo:hi]).backward()
        m.push_sparse()
        ps.finish_step()
    ps.synchronize()
    m.emb.table.synchronize()
    table_rows = m.emb.table.pull_keys(torch.arange(2800, device=DEV)).cpu()
    torch.cuda.synchronize()
    info = {"exchange": m.emb.table.exchange,
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
