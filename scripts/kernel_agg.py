"""Per-kernel-name time aggregate of a rocprofv3 kernel_trace.csv: total ms / N steps, dispatches / step.
usage: python scripts/kernel_agg.py TRACE.csv STEPS [TOP]"""
import collections
import csv
import sys

t, n = collections.Counter(), collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:110]
    t[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    n[k] += 1
steps = float(sys.argv[2])
print("total %.3f ms / step" % (sum(t.values()) / 1e6 / steps))
for k, v in t.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 50):
    print("%9.3f ms %6.1f %s" % (v / 1e6 / steps, n[k] / steps, k))
