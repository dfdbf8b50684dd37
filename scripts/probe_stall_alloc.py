"""Root-cause probe for the once-per-process multi-second stall of the ResNet-50 bench with an
unbounded host run-ahead (PS_AMD_MAX_INFLIGHT=0, VERDICT r5 Next #6).

Hypothesis: with the host many steps ahead of the GPU, blocks freed on the host but still used
by a side stream (record_stream) cannot be reused, the caching allocator keeps asking HIP for
new segments, hits the device limit, and then runs its OOM retry path -- synchronize every
stream, hipFree every cached segment, hipMalloc again -- which takes seconds.

Per step (no device sync between steps) this records the host time between step() returns and
the allocator counters: reserved bytes, segments hipMalloc'ed / hipFree'd, alloc retries.
usage: PS_AMD_MAX_INFLIGHT=0 python scripts/probe_stall_alloc.py [--steps N] [--batch B]"""
import collections
import json
import os
import sys
import threading
import time
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _snap():
    s = torch.cuda.memory_stats()
    return {"reserved_gb": round(s.get("reserved_bytes.all.current", 0) / 2 ** 30, 2),
            "active_gb": round(s.get("active_bytes.all.current", 0) / 2 ** 30, 2),
            "segments": s.get("segment.all.current", 0),
            "device_alloc": s.get("num_device_alloc", 0), "device_free": s.get("num_device_free", 0),
            "alloc_retries": s.get("num_alloc_retries", 0), "ooms": s.get("num_ooms", 0),
            "sync_all_streams": s.get("num_sync_all_streams", 0)}


def _task_state(tid):
    """(wchan, syscall number) of one thread of this process: where the kernel has it blocked."""
    out = []
    for f in ("wchan", "syscall"):
        try:
            with open(f"/proc/self/task/{tid}/{f}") as fh:
                out.append(fh.read().split()[0] if f == "syscall" else fh.read())
        except Exception:
            out.append("?")
    return tuple(out)


class Sampler:
    """Every 25 ms: every thread's kernel wait channel + syscall, and the Python stack of the
    Python threads -- so a step that blocks for seconds reports where each thread sat."""

    def __init__(self):
        self.samples = []
        self.stop = threading.Event()
        self.th = threading.Thread(target=self.run, daemon=True)
        self.me = None

    def run(self):
        self.me = threading.get_native_id()
        while not self.stop.is_set():
            t = time.perf_counter()
            frames = sys._current_frames()
            names = {th.ident: (th.name, th.native_id) for th in threading.enumerate()}
            py = {}
            for ident, fr in frames.items():
                nm, nid = names.get(ident, ("?", None))
                if nid is None or nid == self.me:
                    continue
                st = traceback.extract_stack(fr)[-4:]
                py[nid] = nm + ": " + " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}"
                                                  for f in reversed(st))
            tasks = {}
            for tid in os.listdir("/proc/self/task"):
                if int(tid) != self.me:
                    tasks[int(tid)] = _task_state(tid)
            self.samples.append((t, py, tasks))
            time.sleep(0.025)

    def report(self, t0, t1):
        c = collections.Counter()
        for t, py, tasks in self.samples:
            if t0 <= t <= t1:
                for tid, (wchan, sc) in tasks.items():
                    if wchan not in ("0", "?", "do_epoll_wait", "futex_wait_queue", "hrtimer_nanosleep") or tid in py:
                        c[(tid, wchan, sc, py.get(tid, ""))] += 1
        return [f"{n:4d} x tid {tid} wchan={w} syscall={sc} {p}" for (tid, w, sc, p), n in c.most_common(12)]


def main():
    n, batch = 40, 1024
    if "--steps" in sys.argv:
        n = int(sys.argv[sys.argv.index("--steps") + 1])
    if "--batch" in sys.argv:
        batch = int(sys.argv[sys.argv.index("--batch") + 1])
    sys.argv = [sys.argv[0]]
    import bench as B
    from ps_amd import bench_configs as BC
    from ps_amd.parallel.transport import init_distributed

    args = B.parse()
    args.batch_per_gpu = batch
    torch.cuda.set_device(0)
    tp = init_distributed(backend="gloo")
    torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    bench = BC.SETUPS["resnet50"](args, tp, dev)
    torch.cuda.synchronize()
    print(json.dumps({"inflight": os.environ.get("PS_AMD_MAX_INFLIGHT", "2"), "setup": _snap()}), flush=True)
    smp = Sampler()
    smp.th.start()
    ext = None
    if os.environ.get("PROBE_PROC_OUT"):  # an outside sampler: sees every thread even while the GIL is held
        import subprocess

        ext = subprocess.Popen([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "proc_sampler.py"),
                                str(os.getpid()), os.environ["PROBE_PROC_OUT"]])
    prev = time.perf_counter()
    t_start = prev
    for k in range(n):
        bench.step()
        now = time.perf_counter()
        rec = {"step": k, "host_ms": round((now - prev) * 1e3, 1), "wall": time.time()}
        rec.update(_snap())
        print(json.dumps(rec), flush=True)
        if now - prev > 1.0:  # a stall: where every thread was blocked meanwhile
            for line in smp.report(prev, now):
                print("  [stall] " + line, flush=True)
        prev = now
    smp.stop.set()
    torch.cuda.synchronize()
    total = time.perf_counter() - t_start
    print(json.dumps({"total_s": round(total, 2), "ms_per_step": round(total / n * 1e3, 1), "end": _snap()}),
          flush=True)


if __name__ == "__main__":
    main()
