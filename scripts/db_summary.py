"""Per-kernel summary over the last N steps of a rocprofv3 SQLite trace (run_results.db).

Usage: python scripts/db_summary.py <run_results.db> [--steps 5] [--marker fused_opt] [--per-step 5]
Steps are delimited by the LAST dispatch of the marker kernel family in each step.
"""
import argparse
import collections
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--marker", default="fused_opt")
ap.add_argument("--per-step", type=int, default=5, help="marker dispatches per step")
ap.add_argument("--top", type=int, default=45)
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = list(c.execute("select name,start,end,grid_x,grid_y,grid_z,workgroup_x from kernels order by start"))
idx = [i for i, r in enumerate(rows) if a.marker in r[0]]
ends = idx[a.per_step - 1::a.per_step]
lo, hi = ends[-a.steps - 1] + 1, ends[-1] + 1
win = rows[lo:hi]
wall = (win[-1][2] - win[0][1]) / 1e6 / a.steps
tot = collections.defaultdict(float)
cnt = collections.Counter()
for n, s, e, gx, gy, gz, wx in win:
    k = n.replace("void ", "")[:110]
    tot[k] += (e - s) / 1e3
    cnt[k] += 1
ksum = sum(tot.values()) / 1e3 / a.steps
print(f"steps {a.steps}: wall {wall:.3f} ms/step, kernel sum {ksum:.3f} ms/step, dispatches/step {len(win) / a.steps:.0f}")
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:a.top]:
    print(f"{v / a.steps / 1e3:8.3f} ms {cnt[k] // a.steps:4d}x  {k}")
