"""Arenas the processes of a node map from each other (parallel/ipc_arena.py): hipMalloc + IPC handle
up to 1 GiB, VMM chunks exported as dma-buf fds above (hipIpcOpenMemHandle hangs above 2 GiB on this
stack: profiles/r6_plane_ipc_2gib.txt).  Two processes on cuda:0 write a pattern at offsets below
and above 2 GiB and read each other's through the plane's production copy kernel."""
import pytest
import torch

from tests import dist_util

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _body(tp, gb, vmm):
    from ps_amd import _C
    from ps_amd.parallel.ipc_arena import IpcArena

    torch.cuda.set_device(0)
    n = int(gb * 2**30)
    a = IpcArena(n, 0, vmm=vmm)
    t = a.tensor()
    assert t.numel() == n and bool((t[:4096] == 0).all()) and bool((t[-4096:] == 0).all())
    offs = sorted({0, n // 2, max(0, n - 4096), min(n - 4096, (2 << 30) + 8192)})
    for o in offs:
        t[o:o + 4096].fill_(17 + tp.rank * 10 + offs.index(o))
    torch.cuda.synchronize()
    hs = tp.all_gather_object((a.handle(), 0))
    bases = [a.base if r == tp.rank else a.open(h, d) for r, (h, d) in enumerate(hs)]
    tp.barrier()
    out = {}
    buf = torch.empty(4096, dtype=torch.uint8, device=DEV)
    st = torch.cuda.current_stream()
    for r in range(tp.world):
        for o in offs:
            _C.plane.copy_many([(bases[r] + o, buf.data_ptr(), 4096)], st.cuda_stream, 0)
            torch.cuda.synchronize()
            out[(r, o)] = int(buf[0]), bool((buf == buf[0]).all())
    tp.barrier()
    a.close()
    return a.vmm, offs, out


@pytest.mark.parametrize("gb,vmm", [(0.25, False), (0.25, True), (3.0, None)])
def test_ipc_arena_peer_reads(gb, vmm):
    res = dist_util.run(_body, 2, (gb, vmm))
    for rank, (is_vmm, offs, out) in enumerate(res):
        assert is_vmm == (vmm if vmm is not None else gb > 1.0)
        for (r, o), (v, uniform) in out.items():
            assert uniform and v == 17 + r * 10 + offs.index(o), (rank, r, o, v)
