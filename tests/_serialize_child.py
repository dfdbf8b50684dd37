"""Child process of tests/test_serialize_gpu.py: a few PS steps exercising our HIP kernels
(fused Adam on the server shard, fused NHWC BN+ReLU, sparse gather / segment-sum / row-wise
Adagrad, MFMA fused linear), then prints a digest of every resulting tensor."""
import hashlib
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, sys.argv[1])
from ps_amd.models.layers import SparseLayerMixin  # noqa: E402
from ps_amd.ops.bn import BatchNormAct2d  # noqa: E402
from ps_amd.ops.dense import linear_act  # noqa: E402
from ps_amd.parallel.colocated import ColocatedPS  # noqa: E402
from ps_amd.parallel.sparse_table import SparseTable  # noqa: E402
from ps_amd.parallel.updaters import AdagradUpdater, AdamUpdater  # noqa: E402


class Net(SparseLayerMixin, torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.table = SparseTable("e", 32, 1000, AdagradUpdater(0.05, rowwise=True), init=(-0.1, 0.1), seed=3,
                                 device="cuda")
        self._pending = []
        self.fc1 = torch.nn.Linear(32, 256)
        self.bn = BatchNormAct2d(64)
        self.fc2 = torch.nn.Linear(256, 10)

    def forward(self, ids):
        e = self._lookup(self.table, ids, torch.bfloat16).sum(1)  # [B, 32]
        h = linear_act(e, self.fc1.weight, self.fc1.bias, 1)  # MFMA fused linear + relu
        h = self.bn(h.view(-1, 64, 2, 2).contiguous(memory_format=torch.channels_last))
        return linear_act(h.reshape(h.shape[0], -1).contiguous(), self.fc2.weight, self.fc2.bias, 0)


torch.manual_seed(0)
m = Net().cuda()
m.fc1.to(torch.bfloat16)
m.fc2.to(torch.bfloat16)
ps = ColocatedPS(m, AdamUpdater(1e-2, bias_correction="step"), bucket_mb=0.05)
g = torch.Generator(device="cuda").manual_seed(1)
ids = torch.randint(0, 1000, (64, 6), device="cuda", generator=g)
y = torch.randint(0, 10, (64,), device="cuda", generator=g)
for _ in range(5):
    loss = F.cross_entropy(m(ids).float(), y)
    loss.backward()
    m.push_sparse()
    ps.finish_step()
ps.synchronize()
torch.cuda.synchronize()
h = hashlib.sha256()
for t in list(m.state_dict().values()) + [m.table.table, m.table.states[0]]:
    h.update(t.detach().float().cpu().numpy().tobytes())
print("DIGEST", h.hexdigest(), float(loss))
