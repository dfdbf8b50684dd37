"""Achieved HBM bandwidth per kernel over the last N ResNet-50 steps.

usage: python scripts/pmc_step_summary.py FETCH_DIR WRITE_DIR CLEAN_DB_OR_TRACE_CSV [--steps 2] [--per-step 5]
FETCH_SIZE / WRITE_SIZE (KB, rocprofv3 --pmc, one counter per pass) give the bytes each kernel
moved through HBM; durations come from a clean (counter-free) kernel trace of the same tree,
matched by kernel name.  Prints per kernel: dispatches/step, ms/step, GB/step, TB/s.
"""
import argparse
import collections
import csv
import glob
import os
import sqlite3


def short(n):
    n = n.replace("void ", "")
    return n.split("(")[0][:90] if "psamd::" in n or "at::" in n else n[:60]


def pmc(dirname, counter, steps, per_step):
    f = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)[0]
    rows = []
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    idx = [i for i, r in enumerate(rows) if "fused_opt" in r[1]]
    ends = idx[per_step - 1::per_step]
    lo, hi = ends[-steps - 1] + 1, ends[-1] + 1
    tot = collections.defaultdict(float)
    for _, n, v in rows[lo:hi]:
        tot[short(n)] += v * 1024 / steps
    return tot


def durations(db, steps=5, per_step=5):
    if db.endswith(".csv"):  # a clean rocprofv3 --kernel-trace csv of the same tree
        with open(db) as fh:
            rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                           for r in csv.DictReader(fh)), key=lambda r: r[1])
    else:
        c = sqlite3.connect(db)
        rows = list(c.execute("select name,start,end from kernels order by start"))
    idx = [i for i, r in enumerate(rows) if "fused_opt" in r[0]]
    ends = idx[per_step - 1::per_step]
    lo, hi = ends[-steps - 1] + 1, ends[-1] + 1
    t = collections.defaultdict(float)
    cnt = collections.Counter()
    for n, s, e in rows[lo:hi]:
        t[short(n)] += (e - s) / 1e6 / steps
        cnt[short(n)] += 1
    return t, {k: v // steps for k, v in cnt.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--per-step", type=int, default=5)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rd = pmc(a.fetch, "FETCH_SIZE", a.steps, a.per_step)
    wr = pmc(a.write, "WRITE_SIZE", a.steps, a.per_step)
    ms, cnt = durations(a.db)
    tot_ms = sum(ms.values())
    tot_b = sum(rd.values()) + sum(wr.values())
    print(f"step: {tot_ms:.2f} ms kernel time, {tot_b / 1e9:.2f} GB HBM traffic "
          f"({tot_b / 1e9 / tot_ms:.2f} TB/s averaged over the step)")
    print(f"{'ms/step':>8} {'n':>4} {'GB read':>8} {'GB write':>8} {'TB/s':>6}  kernel")
    for k, t in sorted(ms.items(), key=lambda x: -x[1])[:a.top]:
        r, w = rd.get(k, 0.0), wr.get(k, 0.0)
        print(f"{t:8.3f} {cnt[k]:4d} {r / 1e9:8.3f} {w / 1e9:8.3f} {(r + w) / 1e9 / t if t else 0:6.2f}  {k}")


if __name__ == "__main__":
    main()
