"""Split-K linear weight gradient (csrc/kernels/convgemm.hip conv_wgrad_wide_kernel as a 1x1
"convolution", ops/dense.py linear_wgrad_db) on the BERT-base bench shapes (1024 x 128 tokens)
vs hipBLASLt (dy^T x): time and TF/s per GEMM.
Usage: python scripts/probe_linear_wgrad.py [--tokens 131072] [--it 10]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops._ext import native  # noqa: E402


def bench(fn, it):
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
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--it", type=int, default=10)
    ap.add_argument("--blas", type=int, default=1)
    a = ap.parse_args()
    T = a.tokens
    for name, n, k in (("qkv", 2304, 768), ("proj", 768, 768), ("fc1", 3072, 768), ("fc2", 768, 3072)):
        dy = torch.randn(T, n, device="cuda").bfloat16()
        x = torch.randn(T, k, device="cuda").bfloat16()
        fl = 2.0 * T * n * k
        t = bench(lambda: native().linear_wgrad_db(dy, x), a.it)
        rec = {"gemm": name, "T": T, "N": n, "K": k, "splitk_us": round(t, 1), "splitk_tf": round(fl / t / 1e6, 1)}
        if a.blas:
            tb = bench(lambda: dy.t() @ x, a.it)
            rec.update(blas_us=round(tb, 1), blas_tf=round(fl / tb / 1e6, 1))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
