"""Per-kernel mean of rocprofv3 --pmc counters (run_counter_collection.csv of one or more passes).

usage: python scripts/pmc_summary.py DIR [DIR ...] [--match SUBSTR ...]
Kernels are keyed by a shortened name (template args kept for psamd kernels, library kernels by
their first 60 characters); prints one block per kernel with the mean value per dispatch and
derived ratios (MFMA busy share, wait shares, LDS conflict share, L2 hit rate)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    if "psamd::" in name:
        return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:120]
    return name[:60]


def main():
    args = sys.argv[1:]
    match = []
    if "--match" in args:
        i = args.index("--match")
        match, args = args[i + 1:], args[:i]
    vals = defaultdict(lambda: defaultdict(list))
    for d in args:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = short(r["Kernel_Name"])
                    if match and not any(m in k for m in match):
                        continue
                    vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"== {k}  (dispatches: {max(len(v) for v in cs.values())})")
        for c in sorted(m):
            print(f"   {c:32s} {m[c]:16.0f}")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    print(f"   {c + ' / WAVE_CYCLES':32s} {m[c] / wc:16.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CYCLES" in m:
            # MFMA busy is summed over SIMDs; busy cycles per SE -> normalise by the ratio of units
            print(f"   {'MFMA_BUSY / BUSY_CYCLES':32s} {m['SQ_VALU_MFMA_BUSY_CYCLES'] / m['SQ_BUSY_CYCLES']:16.3f}")
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            print(f"   {'LDS conflict share':32s} {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:16.3f}")
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            t = m["TCC_HIT_sum"] + m["TCC_MISS_sum"]
            if t:
                print(f"   {'L2 hit rate':32s} {m['TCC_HIT_sum'] / t:16.3f}")


if __name__ == "__main__":
    main()
