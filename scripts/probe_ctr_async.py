"""Where a ctr-async step goes (VERDICT r5 Next #8: 326-456K samples/s box to box for one tree).
Runs the bench's ctr-async setup and splits each step on the HOST into forward (row pulls wait for the
owner service), backward, row push, dense finish (push + gated pull), plus the GPU time of the step's
compute-stream work (events), over N steps after a warm-up; also the owner service threads' CPU time
and the process's involuntary context switches (CPU contention on the box).
usage: python scripts/probe_ctr_async.py [--steps N]"""
import json
import os
import resource
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n = 60
    if "--steps" in sys.argv:
        n = int(sys.argv[sys.argv.index("--steps") + 1])
    sys.argv = [sys.argv[0], "--config", "ctr-async"]
    import bench as B
    from ps_amd import bench_configs as BC
    from ps_amd.parallel.transport import Transport

    args = B.parse()
    args.batch_per_gpu = args.batch_per_gpu or BC.DEFAULTS["ctr-async"]["batch"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    torch.manual_seed(1234)
    bench = BC.SETUPS["ctr-async"](args, Transport(), dev)
    for _ in range(10):
        bench.step()
    torch.cuda.synchronize()
    # the step's phases, with the same calls as bench_configs.setup_ctr_async's step (re-made here)
    import ps_amd.bench_configs as bc

    model, ps = None, None
    for c in bench.step.__closure__ or ():
        v = c.cell_contents
        if hasattr(v, "push_sparse"):
            model = v
        elif hasattr(v, "finish_step") and hasattr(v, "peer_mbox"):
            ps = v
    pool_it = [c.cell_contents for c in bench.step.__closure__ if hasattr(c.cell_contents, "__next__")][0]
    cpu0 = os.times()
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    rec = {"fwd": [], "bwd": [], "push_rows": [], "finish": [], "pull_w": [], "host": [], "gpu": [], "wall": []}
    st = torch.cuda.current_stream()
    t_all = time.perf_counter()
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(st)
        b = next(pool_it)
        loss = model.loss(model(b), b["Y"])
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        model.push_sparse()
        t3 = time.perf_counter()
        ps.finish_step()
        t4 = time.perf_counter()
        model.pull_weights()
        t5 = time.perf_counter()
        e1.record(st)
        torch.cuda.synchronize()
        t6 = time.perf_counter()
        for k, v in (("fwd", t1 - t0), ("bwd", t2 - t1), ("push_rows", t3 - t2), ("finish", t4 - t3),
                     ("pull_w", t5 - t4), ("host", t5 - t0), ("wall", t6 - t0)):
            rec[k].append(v * 1e3)
        rec["gpu"].append(e0.elapsed_time(e1))
    total = time.perf_counter() - t_all
    cpu1 = os.times()
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    med = {k: round(sorted(v)[len(v) // 2], 3) for k, v in rec.items()}
    mean = {k: round(sum(v) / len(v), 3) for k, v in rec.items()}
    out = {"steps": n, "batch": args.batch_per_gpu, "samples_per_s": round(args.batch_per_gpu * n / total, 1),
           "ms_median": med, "ms_mean": mean,
           "process_cpu_s_per_step": round(((cpu1.user - cpu0.user) + (cpu1.system - cpu0.system)) / n, 5),
           "invol_ctx_switches_per_step": round((ru1.ru_nivcsw - ru0.ru_nivcsw) / n, 2),
           "vol_ctx_switches_per_step": round((ru1.ru_nvcsw - ru0.ru_nvcsw) / n, 2),
           "cpu_count_visible": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
           "loadavg": os.getloadavg()}
    print(json.dumps(out), flush=True)
    bench.engine.close()


if __name__ == "__main__":
    main()
