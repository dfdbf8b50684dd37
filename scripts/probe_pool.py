"""Stem max-pool kernels at the ResNet-50 bench shape (1024 x 64 x 112 x 112 -> 56 x 56, 3x3/2,
fused BN-apply + ReLU): time and HBM-side bandwidth of forward and backward."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402


def timed(fn, it=20):
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
    nat = native()
    N, C, H = 1024, 64, 112
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    coef = torch.cat([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.5]).contiguous()
    y, idx = nat.maxpool_nhwc_fwd(x, coef, 3, 2, 1)
    dy = torch.randn_like(y)
    tf = timed(lambda: nat.maxpool_nhwc_fwd(x, coef, 3, 2, 1))
    tb = timed(lambda: nat.maxpool_nhwc_bwd(dy, idx, H, H, 3, 2, 1))
    bf = (x.numel() + y.numel()) * 2 + idx.numel()
    bb = (x.numel() + dy.numel()) * 2 + idx.numel()
    print(json.dumps({"fwd_us": round(tf, 1), "fwd_tbps": round(bf / tf / 1e6, 2), "bwd_us": round(tb, 1),
                      "bwd_tbps": round(bb / tb / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
