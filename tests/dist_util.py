"""Run a test body in W gloo processes on 127.0.0.1 and collect per-rank results."""
import os
import socket
import sys
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pack(o):
    import torch

    if isinstance(o, torch.Tensor):
        return ("__t__", o.detach().cpu().numpy().copy())
    if isinstance(o, dict):
        return {k: _pack(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return type(o)(_pack(v) for v in o)
    return o


def _unpack(o):
    import torch

    if isinstance(o, tuple) and len(o) == 2 and isinstance(o[0], str) and o[0] == "__t__":
        return torch.from_numpy(o[1])
    if isinstance(o, dict):
        return {k: _unpack(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return type(o)(_unpack(v) for v in o)
    return o


def _entry(rank, world, port, fn, q, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    try:
        import torch
        import torch.distributed as dist

        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from ps_amd.parallel.transport import Transport

        res = fn(Transport(), *args)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok", _pack(res)))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


def run(fn, world: int = 2, args=(), timeout: float = 240.0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, q, args)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, status, res = q.get(timeout=timeout)
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{res}")
            out[rank] = _unpack(res)
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    return [out[r] for r in range(world)]
