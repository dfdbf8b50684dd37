"""Fused FC layer kernels (csrc/kernels/fc.hip, the reference FcLayer K2 backward + fp32 forward)
vs the equivalent torch (hipBLASLt) GEMMs on the same tensors: reference shapes (MNIST 784 / CNN
1568 / CTR 275 widths) and larger ones.  Per shape: forward (fp32 kernel / bf16 gemm_nt) and the
backward (dW + db + dX, act' folded in) in microseconds and TF/s.
Usage: python scripts/probe_fc.py [--iters 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops._ext import native  # noqa: E402
from ps_amd.ops import dense as D  # noqa: E402


def timed(fn, it):
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
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    shapes = [(1000, 784, 150), (100, 1568, 150), (1000, 275, 150), (8192, 1024, 1024), (16384, 4096, 1024)]
    nat = native()
    for dt in (torch.float32, torch.bfloat16):
        for m, k, n in shapes:
            x = torch.randn(m, k, device="cuda", dtype=dt)
            w = torch.randn(n, k, device="cuda", dtype=dt) * k ** -0.5
            b = torch.randn(n, device="cuda", dtype=torch.float32)
            dy = torch.randn(m, n, device="cuda", dtype=dt)
            y = torch.relu(torch.randn(m, n, device="cuda", dtype=dt))
            dx, dw = torch.empty_like(x), torch.empty_like(w)
            db = torch.empty(n, device="cuda", dtype=torch.float32)
            if dt == torch.float32:
                yo = torch.empty(m, n, device="cuda", dtype=dt)
                tf = timed(lambda: nat.fc_fwd_f32(x, w, b, yo, 1), a.iters)
            else:
                tf = timed(lambda: D.gemm_nt(x, w, b, 1), a.iters)
            tb = timed(lambda: nat.fc_bwd(dy, y, x, w, dw, db, dx, 1), a.iters)
            rf = timed(lambda: torch.relu(torch.addmm(b.to(dt), x, w.t())), a.iters)

            def ref_bwd():
                dz = dy * (y > 0)
                torch.mm(dz, w)
                torch.mm(dz.t(), x)
                dz.sum(0)

            rb = timed(ref_bwd, a.iters)
            fl = 2.0 * m * k * n
            print(json.dumps({"dtype": str(dt).split(".")[-1], "m": m, "k": k, "n": n,
                              "fwd_us": round(tf, 1), "fwd_tf": round(fl / tf / 1e6, 1),
                              "bwd_us": round(tb, 1), "bwd_tf": round(2 * fl / tb / 1e6, 1),
                              "torch_fwd_us": round(rf, 1), "torch_bwd_us": round(rb, 1)}), flush=True)


if __name__ == "__main__":
    main()
