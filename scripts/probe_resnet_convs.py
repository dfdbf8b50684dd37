"""Every distinct ResNet-50 convolution at batch 1024 on the in-house kernels (the production
dispatch: ops/convgemm.py argument order), forward with the BN-statistics epilogue, data gradient
(3x3 stride 1: epilogue 3 on the flipped weight; stride 2: the four phase GEMMs; 1x1: plain) and
weight gradient -- ms per call and TF/s (2 * M_out * N * K), plus the HBM floor of the call.

    python scripts/probe_resnet_convs.py > profiles/r4_resnet50_conv_tflops.txt
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops._ext import native  # noqa: E402
from ps_amd.ops.convgemm import _mat3, _mat3_dgrad, _phase_weights, geo  # noqa: E402

nat = native()
dev = torch.device("cuda")
NIMG = int(os.environ.get("PROBE_BATCH", "1024"))
# (H_in, Cin, Cout, k, stride, count in ResNet-50 v1.5)
SHAPES = [
    (56, 64, 64, 1, 1, 1), (56, 64, 64, 3, 1, 3), (56, 64, 256, 1, 1, 4), (56, 256, 64, 1, 1, 2),
    (56, 256, 128, 1, 1, 1), (56, 128, 128, 3, 2, 1), (56, 256, 512, 1, 2, 1),
    (28, 128, 512, 1, 1, 4), (28, 512, 128, 1, 1, 3), (28, 128, 128, 3, 1, 3),
    (28, 512, 256, 1, 1, 1), (28, 256, 256, 3, 2, 1), (28, 512, 1024, 1, 2, 1),
    (14, 256, 1024, 1, 1, 6), (14, 1024, 256, 1, 1, 5), (14, 256, 256, 3, 1, 5),
    (14, 1024, 512, 1, 1, 1), (14, 512, 512, 3, 2, 1), (14, 1024, 2048, 1, 2, 1),
    (7, 512, 2048, 1, 1, 3), (7, 2048, 512, 1, 1, 2), (7, 512, 512, 3, 1, 2),
]


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / reps)
    return sorted(ts)[1]


def rnd(*s, scale=1.0):
    return (torch.randn(*s, device=dev) * scale).bfloat16()


def coef(k):
    return torch.cat([torch.rand(k, device=dev) + 0.5, torch.randn(k, device=dev) * 0.5])


def main():
    print(f"# ResNet-50 convolutions at batch {NIMG}, 1x MI355X, in-house kernels (scripts/probe_resnet_convs.py)")
    print("# ms per call (median of 3 x 10); TF/s = 2 M_out N K / time; floor = max(FLOPs / 2.5 PF, bytes / 6.3 TB/s)")
    print(f"{'shape (H,Cin->Cout,k,s)':26s}{'x':>3s}{'GFLOP':>8s} | {'fwd ms':>7s}{'TF/s':>6s} | {'dgrad':>7s}{'TF/s':>6s}"
          f" | {'wgrad':>7s}{'TF/s':>6s} | {'floor':>6s}")
    tot = [0.0, 0.0, 0.0]
    for h, cin, cout, k, s, cnt in SHAPES:
        oh = (h - 1) // s + 1 if k == 3 else (h - 1) // s + 1
        m_in, m_out = NIMG * h * h, NIMG * oh * oh
        K = k * k * cin
        flops = 2.0 * m_out * cout * K
        x = rnd(m_in, cin)
        dz = rnd(m_out, cout)
        w = rnd(cout, cin, k, k, scale=K ** -0.5).contiguous(memory_format=torch.channels_last)
        ks = torch.randn(cout, device=dev) * 0.1
        z1, cf1 = rnd(m_in, cin), coef(cin)
        mean, invstd = torch.randn(cin, device=dev) * 0.1, torch.rand(cin, device=dev) + 0.5
        if k == 3:
            gfw = geo(h, h, 3, s, 1)
            wm = _mat3(w)
            f_fwd = lambda: nat.conv_gemm(x, wm, gfw, None, 1, None, ks)  # noqa: E731
            if s == 1:
                wd = _mat3_dgrad(w)
                f_dg = lambda: nat.conv_gemm(dz, wd, geo(oh, oh, 3, 1, 1), None, 3, z1, None, cf1, mean, invstd)  # noqa
            else:
                wph = _phase_weights(w)
                f_dg = lambda: nat.conv_dgrad_s2(dz, wph, h, h, 3, z1, cf1, mean, invstd)  # noqa: E731
            f_wg = lambda: nat.conv_wgrad(dz, x, gfw)  # noqa: E731
        else:
            gfw = geo(h, h, 1, s)
            wm = w.reshape(cout, cin)
            wt = wm.t().contiguous()
            f_fwd = lambda: nat.conv_gemm(x, wm, gfw, None, 1, None, ks)  # noqa: E731
            if s == 1:
                f_dg = lambda: nat.conv_gemm(dz, wt, geo(oh, oh), None, 3, z1, None, cf1, mean, invstd)  # noqa
            else:
                f_dg = None  # (the downsample data gradient is the strided epilogue of conv1's, epilogue 4)
            f_wg = lambda: nat.conv_wgrad(dz, x, gfw)  # noqa: E731
        tf, tg = timed(f_fwd), timed(f_dg) if f_dg is not None else float("nan")
        tw = timed(f_wg)
        byts = 2.0 * (m_in * cin + m_out * cout)
        floor = max(flops / 2.5e15, byts / 6.3e12) * 1e3
        tot[0] += cnt * tf
        tot[1] += cnt * (tg if tg == tg else 0.0)
        tot[2] += cnt * tw
        name = f"{h},{cin}->{cout},{k}x{k},s{s}"
        tfs = lambda t: flops / (t * 1e-3) / 1e12  # noqa: E731
        print(f"{name:26s}{cnt:3d}{flops / 1e9:8.1f} | {tf:7.3f}{tfs(tf):6.0f} | {tg:7.3f}{tfs(tg) if tg == tg else 0:6.0f}"
              f" | {tw:7.3f}{tfs(tw):6.0f} | {floor:6.3f}", flush=True)
        del x, dz, w, z1
        torch.cuda.empty_cache()
    print(f"# network totals (x count): fwd {tot[0]:.2f} ms, dgrad {tot[1]:.2f} ms, wgrad {tot[2]:.2f} ms")


if __name__ == "__main__":
    main()
