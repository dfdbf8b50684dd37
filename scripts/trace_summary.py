"""Summarise a rocprofv3 kernel-trace CSV over the steady-state window.

Usage: python scripts/trace_summary.py <run_kernel_trace.csv> [--last-frac 0.5] [--after KERNEL_SUBSTR]
Prints per-kernel-family time over the window, the busy fraction (union of kernel
intervals / wall) and the number of dispatches.
"""
import argparse
import csv
import re
from collections import defaultdict


def family(name: str) -> str:
    n = name
    if n.startswith("void "):
        n = n[5:]
    rules = [
        (r"naive_conv", "miopen naive conv (find)"),
        (r"psamd::conv_fwd_kernel", "ps_amd implicit-GEMM conv (fwd / dgrad)"),
        (r"psamd::conv_wgrad_kernel", "ps_amd implicit-GEMM conv (wgrad)"),
        (r"igemm_fwd|conv_fwd|grouped_conv_fwd", "conv fwd"),
        (r"igemm_bwd|bwd_data", "conv bwd-data"),
        (r"igemm_wrw|bwd_weight|wrw", "conv bwd-weight"),
        (r"BatchNormFwd", "batchnorm fwd"),
        (r"BatchNormBwd", "batchnorm bwd"),
        (r"batched_gemm|Cijk|gemm", "gemm (fc)"),
        (r"threshold_kernel", "relu bwd (threshold)"),
        (r"clamp_scalar|clamp_min", "relu fwd (clamp)"),
        (r"CUDAFunctor_add<c10::BFloat16>", "add bf16 (residual / grad accumulate)"),
        (r"CUDAFunctor_add<float>", "add fp32"),
        (r"max_pool", "maxpool"),
        (r"fused_opt_kernel", "ps_amd fused optimizer"),
        (r"fillBuffer", "memset"),
        (r"copyBuffer", "memcpy"),
        (r"SubTensorOp", "miopen SubTensorOp"),
        (r"ncclDevKernel|rccl", "rccl"),
        (r"reduce_kernel|reduce", "reduction"),
        (r"softmax|log_softmax|nll_loss|cross_entropy", "loss"),
        (r"elementwise", "other elementwise"),
    ]
    for pat, fam in rules:
        if re.search(pat, n):
            return fam
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last-frac", type=float, default=0.0)
    ap.add_argument("--after", default="naive_conv")
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    start_t = rows[0][0]
    if a.after:
        last = [e for s, e, n in rows if a.after in n]
        if last:
            start_t = max(last)
    if a.last_frac:
        t0, t1 = rows[0][0], rows[-1][1]
        start_t = max(start_t, t1 - int((t1 - t0) * a.last_frac))
    win = [(s, e, n) for s, e, n in rows if s >= start_t]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, n in win:
        fam = family(n)
        tot[fam] += (e - s) / 1e6
        cnt[fam] += 1
    wall = (win[-1][1] - win[0][0]) / 1e6
    # union of intervals
    busy = 0.0
    cs, ce = None, None
    for s, e, _ in win:
        if cs is None:
            cs, ce = s, e
        elif s <= ce:
            ce = max(ce, e)
        else:
            busy += (ce - cs) / 1e6
            cs, ce = s, e
    busy += (ce - cs) / 1e6
    div = a.steps or 1
    ksum = sum(tot.values())
    print(f"window wall {wall:.2f} ms, kernel-busy {busy:.2f} ms ({100 * busy / wall:.1f}%), "
          f"sum kernel time {ksum:.2f} ms, dispatches {len(win)}" + (f", per step /{div}" if div > 1 else ""))
    print(f"{'family':45s} {'ms':>10s} {'%':>6s} {'calls':>7s}")
    for fam, t in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"{fam:45s} {t / div:10.3f} {100 * t / ksum:6.1f} {cnt[fam] // div:7d}")


if __name__ == "__main__":
    main()
