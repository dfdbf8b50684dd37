"""HIP-graph capture of a whole training step (forward + backward + PS round).

MI355X-first replacement for a tracing compiler: after the eager warm-up (which also runs
MIOpen's find for every convolution shape), the step -- every forward/backward kernel, the
bucket hooks' comm-stream work and the fused optimizer kernels -- is captured once with
``torch.cuda.graph`` and replayed with a single launch per step.  This removes the CPU
launch gaps that otherwise leave the GPU idle in the short-kernel tail of backward
(measured: ~9 % idle per ResNet-50 step, profiles/archive/r1_*).

Graph-safety rules the PS engine follows (parallel/colocated.py): static input/output
tensors, no host synchronisation inside the step, buffer bindings that do not change
between replays (BSP: one weight/grad slot), hyper-parameters fixed at capture time (use
``set_device_hyper`` style device scalars for schedules -- momentum SGD at constant LR
needs none).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch


class GraphedStep:
    def __init__(self, step_fn: Callable[[], Optional[torch.Tensor]], warmup: int = 3,
                 pool=None, feed: Optional[Callable[[], None]] = None):
        """``feed`` (optional) refreshes the step's static inputs; it runs eagerly before every
        warm-up step and every replay, never inside the graph."""
        if not torch.cuda.is_available():
            raise RuntimeError("GraphedStep needs a GPU")
        self.step_fn = step_fn
        self.feed = feed
        self.graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                if feed is not None:
                    feed()
                step_fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        with torch.cuda.graph(self.graph, pool=pool):
            self.out = step_fn()
        torch.cuda.synchronize()

    def __call__(self):
        if self.feed is not None:
            self.feed()
        self.graph.replay()
        return self.out
