"""Two-source prologues on the ResNet-50 bs1024 shapes: the BN-backward prologue of the conv3
data gradient (epi 3) and the block-output prologue of conv1 (epi 1), each against the separate
apply pass + plain GEMM it replaces.  Which two-source variant runs (register-staged or
LDS-DMA) is fixed per process by PS_AMD_TWOSRC_GLDS_MIN_NK, so run this once per setting:

    PS_AMD_TWOSRC_GLDS_MIN_NK=99 python scripts/probe_twosrc.py   # register-staged everywhere
    PS_AMD_TWOSRC_GLDS_MIN_NK=4  python scripts/probe_twosrc.py   # LDS-DMA from K = 256

One JSON line per shape: ms of the fused launch and of apply + GEMM (median of 3 x 10 runs)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops._ext import native  # noqa: E402

nat = native()
dev = torch.device("cuda")
MIN_NK = (os.environ.get("PS_AMD_TWOSRC_GLDS_MIN_NK", "4") + "/" + os.environ.get("PS_AMD_PRO_GLDS_MIN_NK", "off") + "/st"
          + os.environ.get("PS_AMD_GLDS_STAGES", "2") + ":" + os.environ.get("PS_AMD_GLDS_DEEP_MIN_NK", "8"))


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


def bwd_case(M, K, N):
    g, z, z2 = rnd(M, K), rnd(M, K), rnd(M, N)
    w = rnd(N, K, scale=K ** -0.5)
    gamma, mean, invstd = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1, torch.rand(K, device=dev) + 0.5
    part = torch.randn(2, 1, K, device=dev)
    mc, m2, i2 = coef(N), torch.randn(N, device=dev) * 0.1, torch.rand(N, device=dev) + 0.5
    geo = [M, 1, M, 1, 1, 1, 0]
    _, _, cf = nat.bn_bwd_coef(part, gamma, mean, invstd, M)

    def fused():
        nat.conv_gemm(g, w, geo, None, 3, z2, None, mc, m2, i2, a2=z, bwd=cf)

    def split():
        dz = nat.bn_bwd_partials(g, z, part, gamma, mean, invstd)[0]
        nat.conv_gemm(dz, w, geo, None, 3, z2, None, mc, m2, i2)

    return timed(fused), timed(split)


def resp_case(M, K, N):
    z3, r = rnd(M, K), rnd(M, K)
    cf, ks = coef(K), torch.randn(N, device=dev) * 0.1
    w = rnd(N, K, scale=K ** -0.5)
    y = torch.empty_like(z3)
    bits = torch.empty(M * K // 8, dtype=torch.uint8, device=dev)
    geo = [M, 1, M, 1, 1, 1, 0]

    def fused():
        nat.conv_gemm(z3, w, geo, cf, 1, None, ks, a2=r, aout=y, abits=bits)

    def split():
        yy = nat.bn_apply_coef(z3, cf, r, None, 1, True)[0]
        nat.conv_gemm(yy, w, geo, None, 1, None, ks)

    return timed(fused), timed(split)


def pro_case(M, K, N):
    """conv3 forward: bn2 + ReLU applied while staging (one source) vs apply pass + plain GEMM."""
    z2 = rnd(M, K)
    cf, ks = coef(K), torch.randn(N, device=dev) * 0.1
    w = rnd(N, K, scale=K ** -0.5)
    geo = [M, 1, M, 1, 1, 1, 0]

    def fused():
        nat.conv_gemm(z2, w, geo, cf, 1, None, ks)

    def split():
        yy = nat.bn_apply_coef(z2, cf, None, None, 1)[0]
        nat.conv_gemm(yy, w, geo, None, 1, None, ks)

    return timed(fused), timed(split)


PRO = [(3211264, 64, 256), (802816, 128, 512), (200704, 256, 1024), (50176, 512, 2048)]
BWD = [(3211264, 256, 64), (802816, 512, 128), (200704, 1024, 256), (50176, 2048, 512)]
RESP = [(3211264, 256, 64), (3211264, 256, 128), (802816, 512, 128), (802816, 512, 256), (200704, 1024, 256),
        (200704, 1024, 512), (50176, 2048, 512)]
def c64_case(M, K, N):
    """3x3 64 -> 64 at 56 x 56: forward (epi 1) and data gradient (epi 3); 'fused' = the default
    routing (the default 3x3 route), 'split' = forward + data gradient sum."""
    n = M // (56 * 56)
    x, w = rnd(M, 64), rnd(64, 576, scale=576 ** -0.5)
    z1, cf = rnd(M, 64), coef(64)
    mean, invstd, ks = torch.randn(64, device=dev) * 0.1, torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev)
    geo = [56, 56, 56, 56, 3, 1, 1]

    def fwd():
        nat.conv_gemm(x, w, geo, None, 1, None, ks)

    def dgrad():
        nat.conv_gemm(x, w, geo, None, 3, z1, None, cf, mean, invstd)

    del n
    return timed(fwd), timed(dgrad)


def plain_case(M, K, N):
    """plain LDS-DMA GEMM (1x1, epi 1; K = 576 / N = 64: the 3x3 tall tile at 56 x 56): ms of the
    forward with statistics (both columns); compare runs with PS_AMD_GLDS_STAGES=2 / 3."""
    if K == 576:
        x, geo = rnd(M, 64), [56, 56, 56, 56, 3, 1, 1]
    else:
        x, geo = rnd(M, K), [M, 1, M, 1, 1, 1, 0]
    w, ks = rnd(N, K, scale=K ** -0.5), torch.randn(N, device=dev) * 0.1

    def fwd():
        nat.conv_gemm(x, w, geo, None, 1, None, ks)

    f = timed(fwd)
    return f, f


PLAIN = [(802816, 512, 128), (200704, 1024, 256), (50176, 2048, 512), (200704, 512, 1024), (3211264, 576, 64),
         (200704, 256, 1024), (802816, 128, 512)]
C64 = [(1024 * 56 * 56, 576, 64), (256 * 56 * 56, 576, 64)]
CASES = [("plain_gemm", PLAIN, plain_case), ("conv3x3_64 (fwd_ms, dgrad_ms)", C64, c64_case), ("bn_relu_prologue", PRO, pro_case), ("bn_bwd_prologue", BWD, bwd_case),
         ("block_output_prologue", RESP, resp_case)]
only = os.environ.get("PROBE_ONLY")
for kind, shapes, fn in CASES:
    if only and kind != only:
        continue
    for M, K, N in shapes:
        f, s = fn(M, K, N)
        print(json.dumps({"kind": kind, "M": M, "K": K, "N": N, "min_nk": MIN_NK, "fused_ms": round(f, 4),
                          "apply_plus_gemm_ms": round(s, 4)}), flush=True)
        torch.cuda.empty_cache()
