"""1x1 stride-1 weight gradients are plain GEMMs (dW[N, K] = dZ[M, N]^T X[M, K], M = pixels):
in-house split-K MFMA kernel (nat.conv_wgrad) vs the library GEMM (hipBLASLt via torch.mm) on
every ResNet-50 1x1 stride-1 shape at the bench batch.

    python scripts/probe_wgrad_blas.py [--batch 1024]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402
from ps_amd.ops.convgemm import geo  # noqa: E402

SHAPES = [(56, 64, 64, 1), (56, 256, 64, 2), (56, 64, 256, 4), (56, 256, 128, 1), (28, 512, 128, 3),
          (28, 128, 512, 4), (28, 512, 256, 1), (14, 1024, 256, 5), (14, 256, 1024, 6), (14, 1024, 512, 1),
          (7, 2048, 512, 2), (7, 512, 2048, 3)]


def bench(fn, it):
    for _ in range(3):
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
    ap.add_argument("--it", type=int, default=10)
    a = ap.parse_args()
    nat = native()
    tot = {"ours": 0.0, "blas": 0.0, "best": 0.0}
    for h, ci, co, calls in SHAPES:
        M = a.batch * h * h
        x2 = torch.randn(M, ci, device="cuda").bfloat16()
        dz2 = torch.randn(M, co, device="cuda").bfloat16()
        g = geo(h, h, 1, 1, 0)
        flops = 2.0 * M * co * ci
        t0 = bench(lambda: nat.conv_wgrad(dz2, x2, g), a.it)
        t1 = bench(lambda: torch.mm(dz2.t(), x2), a.it)
        ref = torch.mm(dz2.t().float(), x2.float())
        err = ((torch.mm(dz2.t(), x2).float() - ref).abs().max() / ref.abs().max()).item()
        rec = {"shape": f"1x1 {h}x{h} {ci}->{co}", "calls": calls, "ours_us": round(t0, 1),
               "ours_tflops": round(flops / t0 / 1e6, 1), "blas_us": round(t1, 1),
               "blas_tflops": round(flops / t1 / 1e6, 1), "blas_relerr": round(err, 5)}
        tot["ours"] += calls * t0
        tot["blas"] += calls * t1
        tot["best"] += calls * min(t0, t1)
        print(json.dumps(rec), flush=True)
        del x2, dz2
        torch.cuda.empty_cache()
    print(json.dumps({"step_total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
