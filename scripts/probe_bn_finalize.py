"""The BN finalize chain (partials fold + per-channel finalize) standalone at the ResNet-50 partial-row
counts: forward statistics (bn_finalize_sums) and backward coefficients (bn_bwd_coef), back to back
200 times per shape.  Run under rocprofv3 --kernel-trace --stats for per-kernel durations; the
event time per call printed here also includes the launch gaps of a dependent chain."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from ps_amd.ops._ext import native

    nat = native()
    it = int(os.environ.get("IT", "200"))
    for G, C in [(25088, 64), (12544, 64), (6272, 128), (3136, 256), (512, 256), (784, 1024), (196, 2048), (256, 512)]:
        part = torch.randn(2, G, C, device="cuda")
        ks = torch.zeros(C, device="cuda")
        gamma, beta = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        mean, invstd = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        R = G * 128
        res = {"G": G, "C": C}
        for name, fn in [("fwd", lambda: nat.bn_finalize_sums(part, ks, R, gamma, beta, rm, rv, 0.1, 1e-5)),
                         ("bwd", lambda: nat.bn_bwd_coef(part, gamma, mean, invstd, R))]:
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(it):
                fn()
            b.record()
            torch.cuda.synchronize()
            res[name + "_us"] = round(a.elapsed_time(b) / it * 1e3, 2)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
