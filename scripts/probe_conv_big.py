"""Deep-K 1x1 convolution GEMMs of ResNet-50 (layers 2-4 at batch 1024 / 256) through conv_gemm:
time per call and TF/s.  Run once with PS_AMD_CONV_BIG=1 (256 x 256 tiles, conv_big.hip) and once
with PS_AMD_CONV_BIG=0 (the 128 x 128 conv_fwd_kernel) -- the switch is read once per process.
One JSON line per shape and batch."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native  # noqa: E402
from ps_amd.ops.convgemm import geo  # noqa: E402

# name, H (input map), K (input channels), N (output channels), stride, epilogue
SHAPES = [
    ("l3 conv1 14x14 1024->256", 14, 1024, 256, 1, 1),
    ("l3 conv3 dgrad 14x14 1024->256", 14, 1024, 256, 1, 3),
    ("l3 conv3 14x14 256->1024", 14, 256, 1024, 1, 1),
    ("l3b0 conv1 28x28 512->256", 28, 512, 256, 1, 1),
    ("l4 conv1 7x7 2048->512", 7, 2048, 512, 1, 1),
    ("l4 conv3 dgrad 7x7 2048->512", 7, 2048, 512, 1, 3),
    ("l4 conv3 7x7 512->2048", 7, 512, 2048, 1, 1),
    ("l4b0 conv1 14x14 1024->512", 14, 1024, 512, 1, 1),
    ("ds l2 56->28 256->512", 56, 256, 512, 2, 1),
    ("ds l3 28->14 512->1024", 28, 512, 1024, 2, 1),
    ("ds l4 14->7 1024->2048", 14, 1024, 2048, 2, 1),
]


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
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


def main():
    nat = native()
    mode = os.environ.get("PS_AMD_CONV_BIG", "1")
    for n in (1024, 256):
        for name, h, k, co, s, epi in SHAPES:
            gg = geo(h, h, 1, s)
            M = n * gg[2] * gg[3]
            a = (torch.randn(n * h * h, k, device="cuda") * 0.5).bfloat16()
            b = (torch.randn(co, k, device="cuda") * k ** -0.5).bfloat16()
            ks = torch.zeros(co, device="cuda")
            if epi == 1:
                fn = lambda: nat.conv_gemm(a, b, gg, None, 1, None, ks)  # noqa: E731
            else:
                z = torch.randn(M, co, device="cuda").bfloat16()
                mc = torch.cat([torch.ones(co, device="cuda"), torch.zeros(co, device="cuda")])
                mean, inv = torch.zeros(co, device="cuda"), torch.ones(co, device="cuda")
                fn = lambda: nat.conv_gemm(a, b, gg, None, 3, z, None, mc, mean, inv)  # noqa: E731
            t = timeit(fn)
            plan = nat.conv_gemm_plan(M, co, k, gg, False, epi)
            flops = 2.0 * M * k * co
            byts = 2.0 * (M * k + M * co * (2 if epi == 3 else 1))
            print(json.dumps({"big": mode, "batch": n, "shape": name, "tile": plan[:2], "ms": round(t, 4),
                              "TFs": round(flops / t / 1e9, 1), "TBs": round(byts / t / 1e9, 2)}), flush=True)
            del a, b
        torch.cuda.empty_cache()


if __name__ == "__main__" and not any(a.startswith("--fold") or a in ("--pro", "--tn", "--blas") for a in sys.argv):
    main()


PRO_SHAPES = [  # name, M (batch 1024), K, N, kind
    ("l3 BWD conv3 dgrad (g,z -> dz) 1024->256", 200704, 1024, 256, "bwd"),
    ("l4 BWD conv3 dgrad 2048->512", 50176, 2048, 512, "bwd"),
    ("l3 RESP conv1 1024->256", 200704, 1024, 256, "resp"),
    ("l3b0 RESP conv1 512->256 (28x28)", 802816, 512, 256, "resp"),
    ("l4 RESP conv1 2048->512", 50176, 2048, 512, "resp"),
    ("l4b0 RESP conv1 1024->512 (14x14)", 200704, 1024, 512, "resp"),
    ("l3 PRO1 conv3 256->1024", 200704, 256, 1024, "pro1"),
]


def main_pro():
    """The prologue variants at their ResNet-50 bs1024 shapes: ms, TF/s and the HBM rate over every
    tensor they move (A and a2 read, aout (+ bits) written, C written, epilogue rows read)."""
    nat = native()
    for name, M, K, N, kind in PRO_SHAPES:
        a = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
        b = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
        gg = [M, 1, M, 1, 1, 1, 0]
        ks = torch.zeros(N, device="cuda")
        coef = torch.cat([torch.ones(K, device="cuda"), torch.zeros(K, device="cuda")])
        if kind == "bwd":
            z = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
            cb = torch.cat([torch.ones(K, device="cuda"), torch.zeros(2 * K, device="cuda")])
            z2 = torch.randn(M, N, device="cuda").bfloat16()
            mc = torch.cat([torch.ones(N, device="cuda"), torch.zeros(N, device="cuda")])
            mean, inv = torch.zeros(N, device="cuda"), torch.ones(N, device="cuda")
            fn = lambda: nat.conv_gemm(a, b, gg, None, 3, z2, None, mc, mean, inv, a2=z, bwd=cb)  # noqa: E731
            byts = 2.0 * (3 * M * K + 2 * M * N)
            src2 = 2
        elif kind == "resp":
            r = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
            out = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
            bits = torch.empty(M * K // 8, device="cuda", dtype=torch.uint8)
            fn = lambda: nat.conv_gemm(a, b, gg, coef, 1, None, ks, a2=r, aout=out, abits=bits)  # noqa: E731
            byts = 2.0 * (3 * M * K + M * N) + M * K / 8
            src2 = 1
        else:
            fn = lambda: nat.conv_gemm(a, b, gg, coef, 1, None, ks)  # noqa: E731
            byts = 2.0 * (M * K + M * N)
            src2 = 0
        t = timeit(fn)
        plan = nat.conv_gemm_plan(M, N, K, gg, True, 3 if kind == "bwd" else 1, src2)
        print(json.dumps({"big": os.environ.get("PS_AMD_CONV_BIG", "1"), "pro_big": os.environ.get("PS_AMD_CONV_BIG_PRO", "1"),
                          "shape": name, "tile": plan[:2], "ms": round(t, 4),
                          "TFs": round(2.0 * M * K * N / t / 1e9, 1), "TBs": round(byts / t / 1e9, 2)}), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__" and "--pro" in sys.argv:
    main_pro()


FOLD_SHAPES = [  # name, images, H (conv1 input map), C1 (conv1 out = K), Cin (= N), epilogue
    ("l3 conv1 dgrad 14x14 256->1024 epi6", 1024, 14, 256, 1024, 6),
    ("l3 conv1 dgrad epi9", 1024, 14, 256, 1024, 9),
    ("l3b0 conv1 dgrad 28x28 256->512 epi8", 1024, 28, 256, 512, 8),
    ("l4 conv1 dgrad 7x7 512->2048 epi6", 1024, 7, 512, 2048, 6),
    ("l4b0 conv1 dgrad 14x14 512->1024 epi8", 1024, 14, 512, 1024, 8),
]


def main_fold():
    """The conv1 data-gradient GEMMs (residual / fold epilogues) at their ResNet-50 bs1024 shapes:
    GEMM alone, GEMM with bn1's backward in the prologue (256 x 256 tiles only), and the apply pass
    (bn_bwd_partials) the prologue replaces."""
    nat = native()
    for name, n, h, k, cin, epi in FOLD_SHAPES:
        gg = geo(h, h)
        M = n * h * h
        g = (torch.randn(M, k, device="cuda") * 0.5).bfloat16()
        z1 = (torch.randn(M, k, device="cuda") * 0.5).bfloat16()
        w = (torch.randn(cin, k, device="cuda") * k ** -0.5).bfloat16()
        if epi == 8:
            r = (h + 1) // 2
            aux = torch.randn(n * r * r, cin, device="cuda").bfloat16()
        else:
            aux = torch.randn(M, cin, device="cuda").bfloat16()
        bits = torch.randint(0, 256, (M * cin // 8,), device="cuda", dtype=torch.uint8)
        kw = dict(aux2=torch.randn(M, cin, device="cuda").bfloat16(), bits2=bits,
                  mean=torch.zeros(cin, device="cuda"), invstd=torch.ones(cin, device="cuda"))
        if epi in (6, 9):
            kw["bits"] = bits
        if epi == 9:
            kw.update(aux3=torch.randn(M, cin, device="cuda").bfloat16(), mean2=torch.zeros(cin, device="cuda"),
                      invstd2=torch.ones(cin, device="cuda"))
        t = timeit(lambda: nat.conv_gemm(g, w, gg, None, epi, aux, **kw))
        plan = nat.conv_gemm_plan(M, cin, k, gg, False, epi)
        rec = {"big": os.environ.get("PS_AMD_CONV_BIG_FOLD", "1"), "shape": name, "tile": plan[:2],
               "gemm_ms": round(t, 4), "TFs": round(2.0 * M * k * cin / t / 1e9, 1)}
        gamma, mean, inv = torch.ones(k, device="cuda"), torch.zeros(k, device="cuda"), torch.ones(k, device="cuda")
        part = torch.zeros(2, 4, k, device="cuda")
        rec["apply_ms"] = round(timeit(lambda: nat.bn_bwd_partials(g, z1, part, gamma, mean, inv)), 4)
        if tuple(nat.conv_gemm_plan(M, cin, k, gg, True, epi, 2)[:2]) == (256, 256):
            cb = torch.cat([torch.ones(k, device="cuda"), torch.zeros(2 * k, device="cuda")])
            rec["gemm_pro_ms"] = round(timeit(lambda: nat.conv_gemm(g, w, gg, None, epi, aux, a2=z1, bwd=cb, **kw)), 4)
        print(json.dumps(rec), flush=True)
        del g, z1, aux, kw
        torch.cuda.empty_cache()


if __name__ == "__main__" and "--fold" in sys.argv and "--fold-scan" not in sys.argv:
    main_fold()


def main_fold_scan():
    """Time vs epilogue bytes on the layer-3 conv1 data-gradient shape (M 200704, K 256, N 1024):
    epilogues 0 (store), 2 (+ residual rows), 5 (+ masked residual), 6 (+ fold reduce), 9."""
    nat = native()
    n, h, k, cin = 1024, 14, 256, 1024
    gg = geo(h, h)
    M = n * h * h
    g = (torch.randn(M, k, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(cin, k, device="cuda") * k ** -0.5).bfloat16()
    aux = torch.randn(M, cin, device="cuda").bfloat16()
    bits = torch.randint(0, 256, (M * cin // 8,), device="cuda", dtype=torch.uint8)
    fk = dict(aux2=torch.randn(M, cin, device="cuda").bfloat16(), bits2=bits,
              mean=torch.zeros(cin, device="cuda"), invstd=torch.ones(cin, device="cuda"))
    d3 = dict(aux3=torch.randn(M, cin, device="cuda").bfloat16(), mean2=torch.zeros(cin, device="cuda"),
              invstd2=torch.ones(cin, device="cuda"))
    mn = M * cin
    cases = [(0, (), {}, 2 * mn), (2, (aux,), {}, 4 * mn), (5, (aux,), dict(bits=bits), 4.125 * mn),
             (6, (aux,), dict(bits=bits, **fk), 6.25 * mn), (9, (aux,), dict(bits=bits, **fk, **d3), 8.25 * mn)]
    for epi, pos, kw, byts in cases:
        t = timeit(lambda: nat.conv_gemm(g, w, gg, None, epi, *pos, **kw))
        byts += 2.0 * M * k
        print(json.dumps({"big": os.environ.get("PS_AMD_CONV_BIG_FOLD", "1"), "epi": epi,
                          "tile": nat.conv_gemm_plan(M, cin, k, gg, False, epi)[:2], "ms": round(t, 4),
                          "GB": round(byts / 1e9, 3), "TBs": round(byts / t / 1e9, 2)}), flush=True)
    t = timeit(lambda: aux.clone())
    print(json.dumps({"copy_411MB_ms": round(t, 4), "TBs": round(4.0 * mn / t / 1e9, 2)}), flush=True)
    t = timeit(lambda: torch.add(aux, fk["aux2"]))
    print(json.dumps({"add_3x411MB_ms": round(t, 4), "TBs": round(6.0 * mn / t / 1e9, 2)}), flush=True)


if __name__ == "__main__" and "--fold-scan" in sys.argv:
    main_fold_scan()


TN_SHAPES = [  # name, M (batch 1024), K, N, epilogue, stride-2 input map (0: stride 1)
    ("L1 conv3 fwd 64->256", 3211264, 64, 256, 1, 0),
    ("L1 conv1 dgrad 64->256 epi6", 3211264, 64, 256, 6, 0),
    ("L2 conv3 fwd 128->512", 802816, 128, 512, 1, 0),
    ("L2 conv1 dgrad 128->512 epi6", 802816, 128, 512, 6, 0),
    ("L2 conv1 fwd 512->128", 802816, 512, 128, 1, 0),
    ("L3 conv3 fwd 256->1024", 200704, 256, 1024, 1, 0),
    ("L3 conv1 dgrad epi6", 200704, 256, 1024, 6, 0),
    ("L3 conv1 dgrad epi9", 200704, 256, 1024, 9, 0),
    ("L3 conv1 fwd 1024->256", 200704, 1024, 256, 1, 0),
    ("L3 conv3 dgrad 1024->256 epi3", 200704, 1024, 256, 3, 0),
    ("L4 conv3 fwd 512->2048", 50176, 512, 2048, 1, 0),
    ("L4 conv1 dgrad epi6", 50176, 512, 2048, 6, 0),
    ("ds L2 s2 256->512", 802816, 256, 512, 1, 56),
    ("ds L3 s2 512->1024", 200704, 512, 1024, 1, 28),
]


def main_tn():
    """Plain 1x1 GEMMs (no prologue) of ResNet-50 at bs1024 under the current PS_AMD_CONV_BIG_TN:
    the tile the planner picks and ms / TF/s / HBM rate over A + C + the epilogue's rows."""
    nat = native()
    for name, M, K, N, epi, hs in TN_SHAPES:
        if hs:
            gg = geo(hs, hs, 1, 2)
            a = (torch.randn(M * 4, K, device="cuda") * 0.5).bfloat16()
        else:
            gg = [M, 1, M, 1, 1, 1, 0]
            a = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
        pos, kw, extra = (), {}, 0
        if epi == 1:
            pos = (None, torch.zeros(N, device="cuda"))
        elif epi == 3:
            pos = (torch.randn(M, N, device="cuda").bfloat16(), None,
                   torch.cat([torch.ones(N, device="cuda"), torch.zeros(N, device="cuda")]),
                   torch.zeros(N, device="cuda"), torch.ones(N, device="cuda"))
            extra = 2 * M * N
        elif epi in (6, 9):
            bits = torch.randint(0, 256, (M * N // 8,), device="cuda", dtype=torch.uint8)
            pos = (torch.randn(M, N, device="cuda").bfloat16(),)
            kw = dict(bits=bits, aux2=torch.randn(M, N, device="cuda").bfloat16(), bits2=bits,
                      mean=torch.zeros(N, device="cuda"), invstd=torch.ones(N, device="cuda"))
            extra = 4.25 * M * N
            if epi == 9:
                kw.update(aux3=torch.randn(M, N, device="cuda").bfloat16(), mean2=torch.zeros(N, device="cuda"),
                          invstd2=torch.ones(N, device="cuda"))
                extra += 2 * M * N
        t = timeit(lambda: nat.conv_gemm(a, w, gg, None, epi, *pos, **kw))
        byts = 2.0 * M * K + 2.0 * M * N + extra
        print(json.dumps({"tn_env": os.environ.get("PS_AMD_CONV_BIG_TN", ""), "shape": name,
                          "tile": nat.conv_gemm_plan(M, N, K, gg, False, epi)[:2], "ms": round(t, 4),
                          "TFs": round(2.0 * M * K * N / t / 1e9, 1), "TBs": round(byts / t / 1e9, 2)}), flush=True)
        del a, w, pos, kw
        torch.cuda.empty_cache()


if __name__ == "__main__" and "--tn" in sys.argv:
    main_tn()


def main_blas():
    """The same GEMMs through torch.mm (hipBLASLt / rocBLAS): a ceiling check for the plain K loop."""
    nat = native()
    for name, h, k, co, s, epi in SHAPES:
        if s != 1:
            continue
        M = 1024 * h * h
        a = (torch.randn(M, k, device="cuda") * 0.5).bfloat16()
        b = (torch.randn(co, k, device="cuda") * k ** -0.5).bfloat16()
        bt = b.t()
        t = timeit(lambda: torch.mm(a, bt))
        gg = [M, 1, M, 1, 1, 1, 0]
        t2 = timeit(lambda: nat.conv_gemm(a, b, gg))
        print(json.dumps({"shape": name, "M": M, "K": k, "N": co, "torch_mm_ms": round(t, 4),
                          "torch_TFs": round(2.0 * M * k * co / t / 1e9, 1), "ours_epi0_ms": round(t2, 4),
                          "ours_TFs": round(2.0 * M * k * co / t2 / 1e9, 1)}), flush=True)
        del a, b, bt
        torch.cuda.empty_cache()


if __name__ == "__main__" and "--blas" in sys.argv:
    main_blas()
