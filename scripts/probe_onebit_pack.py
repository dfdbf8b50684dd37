"""1-bit pack + error feedback on one 64 MB bf16 bucket (csrc/kernels/compress.hip), isolated:
us per call and the bytes it moves (g + e read, e + words written) -> TB/s."""
import torch

from ps_amd.ops import compress as C


def main():
    n = 32 * 2**20  # 64 MB of bf16
    g = torch.randn(n, device="cuda").bfloat16()
    for edt in (torch.float32, torch.bfloat16):
        e = torch.zeros(n, device="cuda", dtype=edt)
        nw, ns = C.packed_sizes(n)
        w = torch.empty(nw, dtype=torch.int64, device="cuda")
        s = torch.empty(ns, device="cuda")
        for _ in range(5):
            C.onebit_pack(g, e, w, s)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(50):
            C.onebit_pack(g, e, w, s)
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / 50 * 1e3
        nbytes = n * 2 + 2 * n * e.element_size() + nw * 8
        print(f"64 MB bf16 bucket, {str(edt).replace('torch.', '')} error feedback: {us:.1f} us, "
              f"{nbytes / us / 1e6:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
