"""Longest HIP runtime API calls of a rocprofv3 --hip-runtime-trace CSV (finding a host-side block).
usage: api_trace_top.py run_hip_api_trace.csv [N]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in rows:
    r["dur_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
t0 = min(int(r["Start_Timestamp"]) for r in rows)
print(f"{len(rows)} API calls")
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for r in rows:
    a = agg[r["Function"]]
    a[0] += 1
    a[1] += r["dur_ms"]
    a[2] = max(a[2], r["dur_ms"])
print("per function: calls, total ms, max ms")
for f, (c, tot, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:15]:
    print(f"  {f:40s} {c:7d} {tot:10.1f} {mx:9.2f}")
print(f"longest {n} calls (start ms from the first call):")
for r in sorted(rows, key=lambda r: -r["dur_ms"])[:n]:
    print(f"  {r['Function']:40s} {r['dur_ms']:9.2f} ms  at {(int(r['Start_Timestamp']) - t0) / 1e6:9.1f} ms  tid {r.get('Thread_Id')}")
