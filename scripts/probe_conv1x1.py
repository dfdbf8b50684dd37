"""Micro-benchmark: ResNet-50 1x1 convolutions (bs 256, NHWC bf16) via MIOpen vs hipBLASLt GEMM.

For each shape prints fwd / bwd-data / bwd-weight times for F.conv2d (MIOpen, find mode)
and for the equivalent GEMMs on the [N*H*W, C] view (torch.matmul -> hipBLASLt).
"""
import json
import time

import torch
import torch.nn.functional as F

SHAPES = [  # (H, Cin, Cout, stride)
    (56, 64, 64, 1), (56, 64, 256, 1), (56, 256, 64, 1), (56, 256, 128, 1),
    (28, 128, 512, 1), (28, 512, 128, 1), (28, 512, 256, 1),
    (14, 256, 1024, 1), (14, 1024, 256, 1), (14, 1024, 512, 1),
    (7, 512, 2048, 1), (7, 2048, 512, 1),
]


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    torch.backends.cudnn.benchmark = True
    N = 256
    dev = "cuda"
    tot = {"miopen": 0.0, "gemm": 0.0}
    for H, ci, co, s in SHAPES:
        x = torch.randn(N, ci, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, 1, 1, device=dev) * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, co, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        xr = x.permute(0, 2, 3, 1).reshape(-1, ci)
        dyr = dy.permute(0, 2, 3, 1).reshape(-1, co)
        w2 = w.view(co, ci)
        r = {}
        r["miopen_fwd"] = bench(lambda: F.conv2d(x, w))
        r["miopen_bwd_data"] = bench(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False]))
        r["miopen_bwd_w"] = bench(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False]))
        r["gemm_fwd"] = bench(lambda: xr @ w2.t())
        r["gemm_bwd_data"] = bench(lambda: dyr @ w2)
        r["gemm_bwd_w"] = bench(lambda: dyr.t() @ xr)
        flops = 2 * N * H * H * ci * co
        rec = {"H": H, "cin": ci, "cout": co, **{k: round(v, 1) for k, v in r.items()},
               "tflops_best_fwd": round(flops / min(r["miopen_fwd"], r["gemm_fwd"]) / 1e6, 1)}
        tot["miopen"] += r["miopen_fwd"] + r["miopen_bwd_data"] + r["miopen_bwd_w"]
        tot["gemm"] += r["gemm_fwd"] + r["gemm_bwd_data"] + r["gemm_bwd_w"]
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_us": tot}))


if __name__ == "__main__":
    main()
