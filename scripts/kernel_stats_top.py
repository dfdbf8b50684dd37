"""Top kernels of a rocprofv3 --stats kernel_stats.csv: total ms, calls, share.
Usage: kernel_stats_top.py run_kernel_stats.csv [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.2f} ms over {sum(int(r['Calls']) for r in rows)} calls")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    t = float(r["TotalDurationNs"])
    print(f"{t / 1e6:9.2f} ms {100 * t / tot:5.1f}% {int(r['Calls']):6d} calls  {r['Name'][:120]}")
