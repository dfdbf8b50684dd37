"""Stream concurrency of one steady-state step in a rocprofv3 SQLite trace (run_results.db):
per-stream busy time, the time two or more streams had kernels in flight, and the dispatches of
the side stream next to what the compute stream ran meanwhile.

Usage: python scripts/db_streams.py <run_results.db> [--marker maxpool_nhwc_fwd] [--timeline]
A step runs from one marker dispatch to the next (the second-to-last complete step is used)."""
import argparse
import collections
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--marker", default="maxpool_nhwc_fwd")
ap.add_argument("--timeline", action="store_true")
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = list(c.execute("select name, start, end, stream_id, queue_id from kernels order by start"))
idx = [i for i, r in enumerate(rows) if a.marker in r[0]]
lo, hi = idx[-3], idx[-2]
t0, t1 = rows[lo][1], rows[hi][1]
seg = [r for r in rows if t0 <= r[1] < t1]
busy = collections.defaultdict(float)
cnt = collections.Counter()
for n, s, e, st, q in seg:
    busy[st] += (e - s) / 1e6
    cnt[st] += 1
# overlap: sweep over start/end events
ev = sorted([(s, 1) for _, s, _, _, _ in seg] + [(e, -1) for _, _, e, _, _ in seg])
depth, last, multi, any_ = 0, t0, 0.0, 0.0
for t, d in ev:
    if depth >= 2:
        multi += (t - last) / 1e6
    if depth >= 1:
        any_ += (t - last) / 1e6
    depth += d
    last = t
print(f"step wall {(t1 - t0) / 1e6:.3f} ms, GPU busy (any stream) {any_:.3f} ms, >=2 streams in flight {multi:.3f} ms")
for st in sorted(busy, key=lambda k: -busy[k]):
    print(f"  stream {st}: {busy[st]:8.3f} ms kernel time, {cnt[st]} dispatches")
if a.timeline:
    for n, s, e, st, q in seg:
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f}us s{st} {n.replace('void ', '')[:110]}")
