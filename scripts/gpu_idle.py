"""GPU idle time in the steady-state part of a rocprofv3 kernel trace (any config): the union of kernel
intervals over the trace's last ``frac`` of time, its idle total, and the largest idle gaps with the
kernel that ended each (and its queue).
usage: python scripts/gpu_idle.py KERNEL_TRACE.csv [frac=0.5] [top=12]"""
import csv
import sys


def main():
    path = sys.argv[1]
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    ks = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", ""), r["Kernel_Name"][:90]))
    ks.sort()
    t_end = max(e for _, e, _, _ in ks)
    t_lo = ks[0][0] + (1 - frac) * (t_end - ks[0][0])
    ks = [k for k in ks if k[0] >= t_lo]
    busy_end, idle, gaps = ks[0][1], 0, []
    for s, e, q, n in ks[1:]:
        if s > busy_end:
            idle += s - busy_end
            gaps.append((s - busy_end, s, q, n))
        busy_end = max(busy_end, e)
    span = busy_end - ks[0][0]
    print(f"window {span / 1e6:.2f} ms, {len(ks)} kernels, idle {idle / 1e6:.3f} ms ({100 * idle / span:.1f} %)")
    for g, s, q, n in sorted(gaps, reverse=True)[:top]:
        print(f"  gap {g / 1e3:8.1f} us before q{q} {n}")


if __name__ == "__main__":
    main()
