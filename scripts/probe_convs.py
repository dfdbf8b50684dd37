"""Micro-benchmark every distinct ResNet-50 convolution at batch 512 (NHWC bf16): MIOpen
fwd / bwd-data / bwd-weight, and for 1x1 stride-1 convs the equivalent hipBLASLt GEMMs on
the [N*H*W, C] view, against the roofline max(FLOPs / 2.3 PF, bytes / 6 TB/s).

Prints one JSON line per shape (times in us, x multiplicity in the network) and totals.
"""
import json
import sys
import time

import torch
import torch.nn.functional as F

# (H_in, Cin, Cout, k, stride, count in ResNet-50 v1.5)
SHAPES = [
    (224, 3, 64, 7, 2, 1),
    (56, 64, 64, 1, 1, 1), (56, 64, 64, 3, 1, 3), (56, 64, 256, 1, 1, 4), (56, 256, 64, 1, 1, 2),
    (56, 256, 128, 1, 1, 1), (56, 128, 128, 3, 2, 1), (56, 256, 512, 1, 2, 1),
    (28, 128, 512, 1, 1, 4), (28, 512, 128, 1, 1, 3), (28, 128, 128, 3, 1, 3),
    (28, 512, 256, 1, 1, 1), (28, 256, 256, 3, 2, 1), (28, 512, 1024, 1, 2, 1),
    (14, 256, 1024, 1, 1, 6), (14, 1024, 256, 1, 1, 5), (14, 256, 256, 3, 1, 5),
    (14, 1024, 512, 1, 1, 1), (14, 512, 512, 3, 2, 1), (14, 1024, 2048, 1, 2, 1),
    (7, 512, 2048, 1, 1, 3), (7, 2048, 512, 1, 1, 2), (7, 512, 512, 3, 1, 2),
]


def bench(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
    from bench import setup_miopen_db

    setup_miopen_db()
    torch.backends.cudnn.benchmark = True
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    dev = "cuda"
    tot = {"miopen": 0.0, "best": 0.0, "roof": 0.0}
    for H, ci, co, k, s, cnt in SHAPES:
        p = k // 2
        x = torch.randn(N, ci, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, k, k, device=dev) * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
        Ho = (H + 2 * p - k) // s + 1
        dy = torch.randn(N, co, Ho, Ho, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        args = (dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1)
        r = {"fwd": bench(lambda: F.conv2d(x, w, None, s, p)),
             "bwd_data": 0.0 if ci == 3 else bench(  # the stem input needs no gradient
                 lambda: torch.ops.aten.convolution_backward(*args, [True, False, False])),
             "bwd_w": bench(lambda: torch.ops.aten.convolution_backward(*args, [False, True, False]))}
        best = dict(r)
        if k == 1 and s == 1:
            xr = x.permute(0, 2, 3, 1).reshape(-1, ci)
            dyr = dy.permute(0, 2, 3, 1).reshape(-1, co)
            w2 = w.view(co, ci)
            r["gemm_fwd"] = bench(lambda: xr @ w2.t())
            r["gemm_bwd_data"] = bench(lambda: dyr @ w2)
            best["fwd"] = min(best["fwd"], r["gemm_fwd"])
            best["bwd_data"] = min(best["bwd_data"], r["gemm_bwd_data"])
        flops = 2 * N * Ho * Ho * ci * co * k * k
        bx, by, bw = 2 * N * H * H * ci, 2 * N * Ho * Ho * co, 2 * co * ci * k * k
        one = max(flops / 2.3e15, (bx + by + bw) / 6e12) * 1e6
        roof = {"fwd": one, "bwd_data": one if ci != 3 else 0.0, "bwd_w": one}
        rec = {"H": H, "cin": ci, "cout": co, "k": k, "s": s, "count": cnt,
               **{kk: round(v, 1) for kk, v in r.items()},
               "tflops": {kk: round(flops / r[kk] / 1e6, 0) for kk in ("fwd", "bwd_data", "bwd_w") if r[kk] > 0},
               "roof_us": round(sum(roof.values()), 1)}
        tot["miopen"] += cnt * (r["fwd"] + r["bwd_data"] + r["bwd_w"])
        tot["best"] += cnt * sum(best.values())
        tot["roof"] += cnt * sum(roof.values())
        print(json.dumps(rec), flush=True)
        del x, w, dy
    print(json.dumps({"total_ms": {kk: round(v / 1e3, 2) for kk, v in tot.items()}}))


if __name__ == "__main__":
    main()
