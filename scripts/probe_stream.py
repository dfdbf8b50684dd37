"""HBM streaming ceilings vs the BN apply pass at the ResNet-50 stage-1 block-output shape
(512 x 56 x 56 x 256 bf16 = 822 MB per tensor): torch copy (1R+1W), torch add (2R+1W), and
bn_apply_coef with residual + ReLU-bit output (2R+1W + bits).  One JSON line per case."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402


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
    R, C = 512 * 56 * 56, 256
    a = torch.randn(R, C, device="cuda").bfloat16()
    b = torch.randn(R, C, device="cuda").bfloat16()
    c = torch.empty_like(a)
    nb = a.numel() * 2
    coef = torch.cat([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")])
    rcoef = torch.cat([torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")])
    nat = native()
    cases = [
        ("copy 1R1W", lambda: c.copy_(a), 2 * nb),
        ("add 2R1W", lambda: torch.add(a, b, out=c), 3 * nb),
        ("bn_apply res+bits", lambda: nat.bn_apply_coef(a, coef, b, None, 1, True), 3 * nb + nb // 16),
        ("bn_apply_dual+bits", lambda: nat.bn_apply_coef(a, coef, b, rcoef, 1, True), 3 * nb + nb // 16),
        ("bn_apply no-res", lambda: nat.bn_apply_coef(a, coef, None, None, 1, False), 2 * nb),
    ]
    for name, fn, byts in cases:
        t = bench(fn)
        print(json.dumps({"case": name, "us": round(t, 1), "tbps": round(byts / t / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
