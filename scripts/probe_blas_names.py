"""torch.mm on two deep-K conv GEMM shapes, for rocprofv3 --kernel-trace (which hipBLASLt kernel runs)."""
import torch

for M, K, N in [(50176, 2048, 512), (200704, 1024, 512), (200704, 1024, 256)]:
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(N, K, device="cuda").bfloat16().t()
    for _ in range(5):
        torch.mm(a, b)
    torch.cuda.synchronize()
