"""Per-kernel bandwidth of the fused BN kernels at ResNet-50 batch-512 shapes.
Run under rocprofv3 --kernel-trace; then `probe_bn.py --report trace.csv`."""
import collections
import csv
import sys

SHAPES = [(512 * 3136, 64), (512 * 3136, 256), (512 * 784, 128), (512 * 784, 512), (512 * 196, 256),
          (512 * 196, 1024), (512 * 49, 512), (512 * 49, 2048)]
# bytes moved per element (bf16 = 2 B) by each kernel variant
BYTES = {"bn_stats_partial": 2, "bn_apply_kernel<false, 1": 4, "bn_apply_kernel<true, 1": 6,
         "bn_bwd_reduce_kernel<1>": 6, "bn_bwd_reduce_kernel<2>": 4, "bn_bwd_apply_kernel<1, true": 10,
         "bn_bwd_apply_kernel<2, false": 6}


def run():
    import torch

    from ps_amd.ops import native

    N = native()
    for R, C in SHAPES:
        x = torch.randn(R, C, device="cuda").bfloat16()
        r = torch.randn(R, C, device="cuda").bfloat16()
        dy = torch.randn(R, C, device="cuda").bfloat16()
        g = torch.ones(C, device="cuda")
        b = torch.zeros(C, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        for _ in range(3):
            y, mean, invstd, coef = N.bn_act_fwd(x, None, g, b, rm, rv, True, 0.1, 1e-5, 1)
            y2, _, _, _ = N.bn_act_fwd(x, r, g, b, rm, rv, True, 0.1, 1e-5, 1)
            N.bn_act_bwd(dy, y2, x, g, mean, invstd, 1, True, True, None)
            N.bn_act_bwd(dy, None, x, g, mean, invstd, 1, False, True, coef)
        torch.cuda.synchronize()
        del x, r, dy, y, y2


def report(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda q: int(q["Start_Timestamp"]))
    # kernels appear in launch order: per shape 3 reps x (fwd: stats, fin, apply) x 2 + bwd x 2
    per = collections.defaultdict(list)
    shape_i, seen = 0, 0
    bn = [q for q in rows if "psamd::bn_" in q["Kernel_Name"]]
    per_shape = len(bn) // len(SHAPES)
    for i, q in enumerate(bn):
        R, C = SHAPES[i // per_shape]
        name = q["Kernel_Name"]
        for k, bpe in BYTES.items():
            if k in name:
                t = (int(q["End_Timestamp"]) - int(q["Start_Timestamp"])) / 1e9
                per[(R, C, k)].append(R * C * bpe / t / 1e12)
    for (R, C, k), v in sorted(per.items()):
        print(f"R={R:8d} C={C:5d} {k:32s} {max(v):5.2f} TB/s (best of {len(v)})")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        run()
