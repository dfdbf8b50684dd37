"""BN finalize per call (statistics and backward coefficients from [2, G, C] partials) at the
ResNet-50 shapes: the one-launch coalesced kernel (default) vs fold + 8-channel finalize
(PS_AMD_BN_FIN2=0, read once per process).  One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402

SHAPES = [(12544, 64), (12544, 256), (3136, 128), (3136, 512), (784, 256), (784, 1024), (196, 512), (196, 2048),
          (3136, 64), (784, 128), (196, 256), (49, 512)]


def timeit(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    nat = native()
    for G, C in SHAPES:
        part = torch.rand(2, G, C, device="cuda") + 0.1
        k = torch.zeros(C, device="cuda")
        gam, mean, inv = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        tf = timeit(lambda: nat.bn_finalize_sums(part, k, G * 256, gam, gam, None, None, 0.1, 1e-5))
        tb = timeit(lambda: nat.bn_bwd_coef(part, gam, mean, inv, G * 256))
        print(json.dumps({"fin2": os.environ.get("PS_AMD_BN_FIN2", "1"), "G": G, "C": C, "stats_us": round(tf, 2),
                          "bwd_coef_us": round(tb, 2)}), flush=True)


if __name__ == "__main__":
    main()
