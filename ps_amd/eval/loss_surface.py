"""Loss-surface scan (evaluate/LossSurface.java:45-64 + store/KVStore.java:153-155).

For s in [min, max) step ``scale``: every weight is set to s*w_init + (1-s)*w_final
(the HIP ``lerp`` kernel on a GPU), the loss on a fixed batch is evaluated and plotted as
series ``loss_surface_<step>``; the final weights are restored afterwards.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch

from ..context import Stat, ctx
from ..obs import metrics as _metrics
from ..ops import reduce as _red


class LossSurface:
    def __init__(self, batch: Dict[str, torch.Tensor], model, w_init: Dict[str, torch.Tensor],
                 lo: float = -2.0, hi: float = 2.0, scale: float = 0.1):
        self.batch, self.model = batch, model
        self.w_init = {k: v.detach().float().clone() for k, v in w_init.items()}
        self.lo, self.hi, self.scale = lo, hi, scale

    @torch.no_grad()
    def plot(self) -> List[Tuple[float, float]]:
        params = dict(self.model.named_parameters())
        final = {k: params[k].detach().float().clone() for k in self.w_init}
        prev = ctx.status
        ctx.status = Stat.LOSS_SURFACE_EVAL
        out = []
        try:
            n = int(round((self.hi - self.lo) / self.scale))
            for i in range(n):
                s = round(self.lo + i * self.scale, 2)
                ctx.weights_scale = s
                for k, w0 in self.w_init.items():
                    p = params[k]
                    tmp = torch.empty_like(final[k]) if p.dtype != torch.float32 else None
                    if tmp is None:
                        _red.lerp(w0.to(p.device).reshape(-1), final[k].reshape(-1), s, p.data.view(-1))
                    else:
                        _red.lerp(w0.to(p.device).reshape(-1), final[k].reshape(-1), s, tmp.view(-1))
                        p.data.copy_(tmp)
                pred = self.model.predict(self.batch)
                val = float(self.model.loss(pred, self.batch["Y"]))
                self.model.pull_weights()
                out.append((s, val))
                _metrics.plot(f"loss_surface_{ctx.step}", val, s)
        finally:
            for k in self.w_init:
                params[k].data.copy_(final[k].to(params[k].dtype))
            ctx.status = prev
            ctx.weights_scale = 0.0
        return out
