"""Find a one-off multi-second stall in the first steps of the ResNet-50 bench (seen with --warmup 5:
some runs time 238 ms/step instead of 62): per-step host time of step() with a device sync after
each, and a sampler thread that records the main thread's Python stack every 20 ms, so a step that
takes > 0.5 s reports where the host was.  usage: python scripts/probe_stall.py [--steps N]"""
import collections
import json
import os
import sys
import threading
import time
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n = 40
    if "--steps" in sys.argv:
        n = int(sys.argv[sys.argv.index("--steps") + 1])
    sys.argv = [sys.argv[0]]
    import bench as B
    from ps_amd import bench_configs as BC
    from ps_amd.parallel.transport import init_distributed

    args = B.parse()
    if args.batch_per_gpu == 0:
        args.batch_per_gpu = 1024
    torch.cuda.set_device(0)
    tp = init_distributed(backend="gloo")
    torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    t_setup = time.perf_counter()
    bench = BC.SETUPS["resnet50"](args, tp, dev)
    print(f"setup {time.perf_counter() - t_setup:.2f}s", flush=True)
    main_id = threading.get_ident()
    samples = []  # (t, stack text)
    stop = threading.Event()

    def sampler():
        while not stop.is_set():
            fr = sys._current_frames().get(main_id)
            if fr is not None:
                st = traceback.extract_stack(fr)[-6:]
                samples.append((time.perf_counter(), " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}"
                                                                 for f in reversed(st))))
            time.sleep(0.02)

    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    rec = []
    for k in range(n):
        t0 = time.perf_counter()
        bench.step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rec.append((k, t0, t1, t2))
    stop.set()
    th.join()
    out = {"steps_ms": [round((t2 - t0) * 1e3, 1) for _, t0, _, t2 in rec],
           "issue_ms": [round((t1 - t0) * 1e3, 1) for _, t0, t1, _ in rec]}
    print(json.dumps(out), flush=True)
    for k, t0, t1, t2 in rec:
        if t2 - t0 > 0.5:
            c = collections.Counter(s for t, s in samples if t0 <= t <= t2)
            print(f"step {k}: {(t2 - t0) * 1e3:.0f} ms (issue {(t1 - t0) * 1e3:.0f} ms); top host stacks:")
            for s, cnt in c.most_common(6):
                print(f"   {cnt:4d} x {s}")


if __name__ == "__main__":
    main()
