import torch, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ps_amd.ops import native
nat = native()
R, D = 4096, 4096
x = torch.randn(R, D, device="cuda").bfloat16(); r = torch.randn(R, D, device="cuda").bfloat16()
w = torch.randn(D, device="cuda").bfloat16()
s, y, rstd = nat.rmsnorm_fwd(x, r, w, 1e-5)
dy = torch.randn(R, D, device="cuda").bfloat16(); dsin = torch.randn(R, D, device="cuda").bfloat16()
for _ in range(3): nat.rmsnorm_bwd(dy, s, w, rstd, dsin)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20): nat.rmsnorm_bwd(dy, s, w, rstd, dsin)
e1.record(); torch.cuda.synchronize()
print("rmsnorm_bwd 4096x4096 us:", e0.elapsed_time(e1) / 20 * 1e3)
