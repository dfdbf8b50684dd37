"""Cross-process device-side ordering through IPC events (csrc/plane.cpp IpcEvent) on cuda:0:
rank 0 enqueues a long kernel, then writes a value into its IPC-mapped arena and records an
interprocess event; rank 1 (another process) makes its stream wait on that event and then
reads rank 0's arena over the peer mapping.  The host of rank 1 only waits until rank 0 has
ENQUEUED the record (a gloo barrier here) -- the dependency itself is on the device queues.
This is the primitive behind the plane's round end and the IPC row exchange."""
import pytest
import torch

from tests import dist_util

pytestmark = pytest.mark.gpu


def _body(tp, rounds):
    from ps_amd import _C

    P = _C.plane
    torch.cuda.set_device(0)
    arena = P.Arena(4096, 0)
    ev = P.IpcEvent(0)
    hs = tp.all_gather_object((arena.handle(), ev.handle()))
    peer_base = arena.open(hs[0][0], 0) if tp.rank == 1 else arena.base
    peer_ev = P.IpcEvent(hs[0][1], 0) if tp.rank == 1 else None
    mine = arena.tensor().view(torch.float32)
    s = torch.cuda.Stream()
    got = []
    for r in range(rounds):
        val = float(100 + r)
        tp.barrier()
        if tp.rank == 0:
            with torch.cuda.stream(s):
                torch.cuda._sleep(200_000_000)  # ~0.1 s of device time before the write
                mine[:256].fill_(val)
            ev.record(s.cuda_stream)
            tp.barrier()  # the record is enqueued (not necessarily executed)
            s.synchronize()
        else:
            tp.barrier()
            peer_ev.wait(s.cuda_stream)
            with torch.cuda.stream(s):
                P.copy_many([(peer_base, mine.data_ptr(), 1024)], s.cuda_stream, 0)
            s.synchronize()
            got.append(mine[:256].clone().cpu())
        tp.barrier()
    arena.close()
    return got


def test_ipc_event_orders_a_peer_read_after_the_owner_write():
    res = dist_util.run(_body, 2, (3,))
    for r, t in enumerate(res[1]):
        assert bool((t == 100 + r).all()), (r, t[:4])
