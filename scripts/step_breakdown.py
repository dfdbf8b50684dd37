"""Per-step kernel-family breakdown of a rocprofv3 kernel trace (one steady-state step,
delimited by a once-per-step marker kernel).  Usage: step_breakdown.py trace.csv [marker]"""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from trace_summary import family  # noqa: E402

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "maxpool_nhwc_fwd"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
seg = rows[idx[-3]:idx[-2]]
wall = (int(rows[idx[-2]]["Start_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
fam = collections.defaultdict(float)
cnt = collections.Counter()
scratch = set()
for r in seg:
    f = family(r["Kernel_Name"])[:60]
    fam[f] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    cnt[f] += 1
    if int(r.get("Scratch_Size", 0) or 0) > 0 and "psamd" in r["Kernel_Name"]:
        scratch.add(r["Kernel_Name"][:80])
tot = sum(fam.values())
print(f"step wall {wall:.3f} ms, kernel sum {tot:.3f} ms, dispatches {len(seg)}")
for k, v in sorted(fam.items(), key=lambda x: -x[1]):
    print(f"{k:62s} {v:7.3f} {100 * v / tot:5.1f}% {cnt[k]}")
if scratch:
    print("ps_amd kernels using scratch:", *sorted(scratch), sep="\n  ")

# per-dispatch timeline of the same step (order, duration, grid) -> <trace>.timeline.txt
with open(sys.argv[1] + ".timeline.txt", "w") as f:
    t0 = int(seg[0]["Start_Timestamp"])
    for r in seg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        st = (int(r["Start_Timestamp"]) - t0) / 1e3
        grid = r.get("Grid_Size_X", r.get("Grid_Size", ""))
        f.write(f"{st:10.1f} {d:9.1f}us grid={grid:>8s} {r['Kernel_Name'][:110]}\n")

# per-queue occupancy of the same step: busy = union of that queue's kernel intervals; overlap =
# time with kernels of two or more queues in flight (the side-stream weight gradients hiding
# under the data-gradient chain)
ev = []
byq = collections.defaultdict(list)
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    byq[r.get("Queue_Id", "0")].append((s, e, r["Kernel_Name"]))
    ev += [(s, 1), (e, -1)]
print("queue occupancy:")
for q, ks in sorted(byq.items(), key=lambda x: -len(x[1])):
    ks.sort()
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in ks:
        if cur_e is None or s > cur_e:
            busy += (cur_e - cur_s) if cur_e is not None else 0
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    ksum = sum(e - s for s, e, _ in ks)
    print(f"  queue {q}: {len(ks)} kernels, busy {busy / 1e6:.3f} ms, kernel sum {ksum / 1e6:.3f} ms")
ev.sort()
depth, last, multi, any_ = 0, None, 0, 0
for t_, d in ev:
    if last is not None:
        if depth >= 1:
            any_ += t_ - last
        if depth >= 2:
            multi += t_ - last
    depth += d
    last = t_
print(f"  GPU busy (any queue) {any_ / 1e6:.3f} ms, 2+ kernels in flight {multi / 1e6:.3f} ms, idle {wall - any_ / 1e6:.3f} ms")
