"""Host launch time vs GPU start for every kernel of the last profiled step: joins rocprofv3's kernel
trace with its HIP API trace on the correlation id.  A GPU gap whose next kernel was LAUNCHED by
the host only at the end of the gap is host-bound; one whose kernel was queued long before waits on
a device-side dependency.
usage: python scripts/launch_lag.py KERNEL_TRACE.csv HIP_API_TRACE.csv [gap_us]"""
import csv
import sys


def main():
    kt, at = sys.argv[1], sys.argv[2]
    gap_min = float(sys.argv[3]) if len(sys.argv) > 3 else 50.0
    api = {}
    with open(at) as f:
        for r in csv.DictReader(f):
            api[r["Correlation_Id"]] = (int(r["Start_Timestamp"]), r["Function"])
    ks = []
    with open(kt) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:90], r["Correlation_Id"],
                       r.get("Queue_Id", "")))
    ks.sort()
    # the last step: from the last stem_conv_fwd_kernel but one
    stems = [i for i, k in enumerate(ks) if "stem_conv_fwd_kernel" in k[2]]
    lo = stems[-2] if len(stems) >= 2 else 0
    hi = stems[-1] + 1 if len(stems) >= 1 else len(ks)
    ks = ks[lo:hi]
    t0 = ks[0][0]
    busy_end = ks[0][1]
    print(f"{'gpu_start_us':>12s} {'gap_us':>8s} {'host_launch_us':>14s} {'queued_ahead_us':>15s}  kernel")
    for s, e, name, cid, q in ks:
        gap = (s - busy_end) / 1e3
        h = api.get(cid)
        hl = (h[0] - t0) / 1e3 if h else float("nan")
        ahead = (s - h[0]) / 1e3 if h else float("nan")
        if gap >= gap_min:
            print(f"{(s - t0) / 1e3:12.1f} {gap:8.1f} {hl:14.1f} {ahead:15.1f}  q{q} {name}")
        busy_end = max(busy_end, e)


if __name__ == "__main__":
    main()
