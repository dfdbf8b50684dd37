"""Thread states during the stalled step of probe_stall_alloc.py (outside sampler rows of proc_sampler.py).
usage: stall_threads.py probe.jsonl proc.jsonl"""
import collections
import json
import sys

steps = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{"step"')]
rows = [json.loads(l) for l in open(sys.argv[2])]
for r in steps:
    if r["host_ms"] < 1000:
        continue
    t1 = r["wall"]
    t0 = t1 - r["host_ms"] / 1e3
    win = [x for x in rows if t0 + 0.05 <= x["t"] <= t1 - 0.05]
    print(f"step {r['step']}: {r['host_ms']:.0f} ms, {len(win)} samples")
    c = collections.Counter()
    for x in win:
        for tid, comm, state, wchan, sc in x["th"]:
            c[(tid, comm, state, wchan, sc.split()[0] if sc != "?" else sc)] += 1
    for (tid, comm, state, wchan, sc), n in sorted(c.items(), key=lambda kv: -kv[1]):
        if wchan in ("futex_do_wait",) and state == "S" and n == len(win):
            continue  # idle for the whole stall
        print(f"  {n:4d} x tid {tid} {comm:16s} {state} wchan={wchan} syscall={sc}")
    # full syscall text of the non-futex threads
    seen = set()
    for x in win[len(win) // 2:len(win) // 2 + 1]:
        for tid, comm, state, wchan, sc in x["th"]:
            if wchan != "futex_do_wait" and tid not in seen:
                seen.add(tid)
                print(f"  mid-stall tid {tid} {comm} {state} {wchan} syscall: {sc}")
