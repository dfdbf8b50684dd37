"""Standalone bandwidth of the BN-backward apply pass (bn_bwd_partials: finalize + dz = A gy + B z + C)
at the ResNet-50 bs1024 shapes, against torch's 2-read / 1-write elementwise add of the same tensors
(the HBM roofline of the pass).  Prints one JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


def main():
    from ps_amd.ops._ext import native

    nat = native()
    B = int(os.environ.get("B", "1024"))
    for hw, c in [(56, 64), (28, 128), (14, 256), (7, 512), (56, 256), (28, 512)]:
        R = B * hw * hw
        g = torch.randn(R, c, device="cuda").bfloat16()
        z = torch.randn(R, c, device="cuda").bfloat16()
        G = 256
        part = torch.randn(2, G, c, device="cuda")
        gamma = torch.rand(c, device="cuda") + 0.5
        mean = torch.randn(c, device="cuda") * 0.1
        invstd = torch.rand(c, device="cuda") + 0.5
        out = torch.empty_like(g)
        t_apply = timed(lambda: nat.bn_bwd_partials(g, z, part, gamma, mean, invstd))
        t_add = timed(lambda: torch.add(g, z, out=out))
        gb = 3 * R * c * 2 / 1e9
        print(json.dumps({"rows": R, "C": c, "bn_bwd_partials_ms": round(t_apply, 4),
                          "tbps": round(gb / t_apply, 2), "torch_add_ms": round(t_add, 4),
                          "torch_add_tbps": round(gb / t_add, 2)}), flush=True)
        del g, z, out


if __name__ == "__main__":
    main()
