"""List one steady-state step's calls of kernels matching a pattern (duration, grid) from a
rocprofv3 kernel trace: kernel_calls.py trace.csv pattern [marker]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2]
marker = sys.argv[3] if len(sys.argv) > 3 else "maxpool_nhwc_fwd"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
for r in rows[idx[-3]:idx[-2]]:
    n = r["Kernel_Name"]
    if pat in n:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        name = n.split("(")[0].replace("void ", "").replace("psamd::", "")
        print(f"{name[:40]:40s} grid={int(r['Grid_Size_X']) // 256:6d} vgpr={r['VGPR_Count']:>4s} lds={r['LDS_Block_Size']:>6s} {d:8.1f} us")
