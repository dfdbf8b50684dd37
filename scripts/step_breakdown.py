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
