"""Phase-by-phase probe of the VMM-chunked IPC arena (ps_amd/parallel/ipc_arena.py).
usage: python scripts/probe_vmm_arena.py self GB      (one process: export + import its own chunks)
       python -m torch.distributed.run --nproc-per-node 2 scripts/probe_vmm_arena.py peer GB"""
import faulthandler
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    faulthandler.dump_traceback_later(15, repeat=True)
    from ps_amd import _C

    mode, gb = sys.argv[1], float(sys.argv[2])
    torch.cuda.set_device(0)
    t0 = time.time()
    rank = int(os.environ.get("RANK", "0"))

    def say(m):
        print(f"[{mode} rank {rank} +{time.time() - t0:6.2f}s] {m}", flush=True)

    n = int(gb * 2**30)
    if mode == "self":
        a = _C.plane.VmmArena(n, 0, 1 << 30)
        say(f"created, chunks {a.chunk_sizes()}")
        fds = a.export_fds()
        say(f"exported fds {fds}")
        b = _C.plane.VmmArena(4096, 0, 1 << 30)
        base = b.open(list(fds), list(a.chunk_sizes()), 0)
        say(f"imported at {base:#x} (own base {a.base:#x})")
        a.tensor()[:8].fill_(42)
        buf = torch.zeros(16, dtype=torch.uint8, device="cuda")
        _C.plane.copy_many([(base, buf.data_ptr(), 16)], torch.cuda.current_stream().cuda_stream, 0)
        torch.cuda.synchronize()
        say(f"read through the import: {buf[:8].tolist()}")
        os._exit(0)
    import torch.distributed as dist

    from ps_amd.parallel.ipc_arena import IpcArena

    dist.init_process_group("gloo")
    a = IpcArena(n, 0, vmm=True)
    say("arena + fd server up")
    hs = [None] * dist.get_world_size()
    dist.all_gather_object(hs, a.handle())
    say("handles exchanged")
    for p, h in enumerate(hs):
        if p != rank:
            base = a.open(h, 0)
            say(f"opened peer {p} at {base:#x}")
    dist.barrier()
    say("done")
    os._exit(0)


if __name__ == "__main__":
    main()
