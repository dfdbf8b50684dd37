"""1x1 forward implicit GEMMs of the ResNet-50 bottleneck at the bench batch (conv_gemm with the
bn prologue / statistics epilogue as the fused block runs them): time, TF/s, HBM-side TB/s.
Used to pick the persistent-grid threshold (PS_AMD_PERSIST_NK_PRO).

    python scripts/probe_conv_fwd.py [--batch 1024]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402
from ps_amd.ops.convgemm import geo  # noqa: E402

SHAPES = [  # H, Cin, Cout, bn prologue
    (56, 64, 256, True), (28, 128, 512, True), (14, 256, 1024, True), (7, 512, 2048, True),
    (56, 256, 64, False), (28, 512, 128, False), (14, 1024, 256, False), (7, 2048, 512, False)]


def bench(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--variants", type=int, default=0,
                    help="also time each shape without the statistics epilogue / without the BN prologue")
    a = ap.parse_args()
    nat = native()
    for h, ci, co, pro in SHAPES:
        M = a.batch * h * h
        x = torch.randn(M, ci, device="cuda").bfloat16()
        w = (torch.randn(co, ci, device="cuda") * 0.05).bfloat16()
        coef = torch.cat([torch.rand(ci, device="cuda") + 0.5, torch.randn(ci, device="cuda")]) if pro else None
        ks = torch.zeros(co, device="cuda")
        t = bench(lambda: nat.conv_gemm(x, w, geo(h, h), coef, 1, None, ks))
        tb = bench(lambda: x @ w.t())
        fl = 2.0 * M * ci * co
        by = 2.0 * M * (ci + co)
        rec = {"shape": f"1x1 {h}x{h} {ci}->{co}" + (" +bn" if pro else ""), "us": round(t, 1),
               "tflops": round(fl / t / 1e6, 1), "tbps": round(by / t / 1e6, 2),
               "blas_us": round(tb, 1), "persist_nk_pro": os.environ.get("PS_AMD_PERSIST_NK_PRO", "4")}
        if a.variants:
            rec["no_stats_us"] = round(bench(lambda: nat.conv_gemm(x, w, geo(h, h), coef, 0)), 1)
            if pro:
                rec["no_pro_us"] = round(bench(lambda: nat.conv_gemm(x, w, geo(h, h), None, 1, None, ks)), 1)
                rec["no_pro_no_stats_us"] = round(bench(lambda: nat.conv_gemm(x, w, geo(h, h), None, 0)), 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
