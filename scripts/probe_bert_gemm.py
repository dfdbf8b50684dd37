"""BERT-base GEMM shapes (T = 256 x 128 tokens) through torch matmul: forward (x W^T), data grad
(dy W) and weight grad (dy^T x) per Linear, under the current BLAS backend.  Run with
TORCH_BLAS_PREFER_HIPBLASLT=0 to compare rocBLAS."""
import json
import os

import torch


def bench(fn, it=10):
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
    T = 256 * 128
    tot = 0.0
    for name, k, n in [("qkv", 768, 2304), ("proj", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768)]:
        x = torch.randn(T, k, device="cuda").bfloat16()
        w = torch.randn(n, k, device="cuda").bfloat16()
        dy = torch.randn(T, n, device="cuda").bfloat16()
        fl = 2.0 * T * k * n
        r = {"gemm": name, "T": T, "K": k, "N": n}
        for d, fn in (("fwd", lambda: torch.nn.functional.linear(x, w)), ("dgrad", lambda: dy @ w),
                      ("wgrad", lambda: dy.t() @ x)):
            t = bench(fn)
            tot += t
            r[d + "_us"] = round(t, 1)
            r[d + "_tf"] = round(fl / t / 1e6, 1)
        print(json.dumps(r), flush=True)
    print(json.dumps({"layer_total_us": round(tot, 1), "backend": os.environ.get("TORCH_BLAS_PREFER_HIPBLASLT", "default")}))


if __name__ == "__main__":
    main()
