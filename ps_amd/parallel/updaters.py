"""Server-side optimizers ("updaters") and the spec-string registry.

Reference: update/Updater.java:8-10 (``update(key, w, dw)`` in place + ``getName()`` spec
string that doubles as the server registry key), SimpleUpdater.java, AdamUpdater.java,
FtrlUpdater.java, and the prefix resolution of store/KVStore.java:242-252.

Two entry points per updater:

* ``update(key, w, dw)`` -- the reference API: per-key, in place, state kept per key inside
  the updater (used by the standalone KVStore and by tests).
* ``step_flat(master, states, grad, wout, gscale_t)`` -- the PS hot path: one fused HIP
  kernel over a whole range-partitioned fp32 shard, writing the bf16/fp32 pull buffer in the
  same pass (csrc/kernels/optim.hip).

Spec strings keep the reference syntax (``"adam@alfa:0.005@beta1:0.9@beta2:0.999@epsilon:1e-08@"``)
so reference launch scripts port unchanged; ``parse_updater`` also accepts the new kinds.
FTRL's name uses the prefix ``ftrl@`` (the reference mislabels it ``adam@``, Q6).
"""
from __future__ import annotations

import math
import re
from typing import Dict, List, Optional

import torch

from ..ops import optim as _o


def _between(spec: str, key: str) -> Optional[str]:
    m = re.search(re.escape(key) + r":([^@]*)@", spec)
    return m.group(1) if m else None


def _fmt(v: float) -> str:
    return repr(float(v))


class Updater:
    """Base class. ``kind`` selects the fused kernel; ``n_state`` fp32 tensors per shard."""

    kind: int = _o.SGD
    n_state: int = 0
    prefix: str = ""

    def __init__(self):
        self._state: Dict[str, List[torch.Tensor]] = {}
        self.t = 0  # optimizer steps applied (for bias correction)

    # ---------------------------------------------------------------- spec string
    @property
    def name(self) -> str:
        return self.prefix + "@" + "".join(f"{k}:{_fmt(v)}@" for k, v in self.spec_items())

    def get_name(self) -> str:  # reference spelling (getName)
        return self.name

    def spec_items(self):
        return []

    # ---------------------------------------------------------------- kernel params
    def hyper(self, step: int) -> dict:
        raise NotImplementedError

    def new_states(self, like: torch.Tensor) -> List[torch.Tensor]:
        return [torch.zeros_like(like, dtype=torch.float32) for _ in range(self.n_state)]

    def step_flat(self, master: torch.Tensor, states: List[torch.Tensor], grad: torch.Tensor,
                  wout: Optional[torch.Tensor] = None, gscale: float = 1.0,
                  gscale_t: Optional[torch.Tensor] = None, step: Optional[int] = None) -> None:
        st = list(states) + [None] * (2 - len(states))
        h = self.hyper(self.t + 1 if step is None else step)
        h["gscale"] = h.get("gscale", 1.0) * gscale
        _o.fused_opt(self.kind, master, st[0], st[1], grad, wout=wout, gscale_t=gscale_t, **h)

    def step_rows(self, table: torch.Tensor, states: List[torch.Tensor], rows: torch.Tensor, grad: torch.Tensor,
                  gscale: float = 1.0, step: Optional[int] = None, rowwise: bool = False,
                  skip_zero: bool = False, perm: Optional[torch.Tensor] = None,
                  ncount: Optional[torch.Tensor] = None) -> None:
        """Row-sparse step; with ``perm`` the rows are sorted with repeats and each run's
        gradient rows are summed into one update (ops/optim.py sparse_opt); ``ncount`` bounds a
        device-counted row list."""
        st = list(states) + [None] * (2 - len(states))
        h = self.hyper(self.t + 1 if step is None else step)
        h["gscale"] = h.get("gscale", 1.0) * gscale
        _o.sparse_opt(self.kind, table, st[0], st[1], rows, grad, rowwise=rowwise, skip_zero=skip_zero, perm=perm,
                      ncount=ncount, **h)

    # ---------------------------------------------------------------- reference API
    def update(self, key: str, w: torch.Tensor, dw: torch.Tensor) -> torch.Tensor:
        """In-place update of ``w`` by ``dw`` with per-key state (update/Updater.java:8)."""
        if key not in self._state:
            self._state[key] = self.new_states(w.reshape(-1).float())
        flat = w.reshape(-1)
        master = flat if flat.dtype == torch.float32 else flat.float()
        self._key_step(key, master, self._state[key], dw.reshape(-1))
        if master is not flat:
            flat.copy_(master)
        return w

    def _key_step(self, key, master, states, g):
        self.step_flat(master, states, g)

    def tick(self) -> None:
        """Advance the optimizer clock (one PS round)."""
        self.t += 1

    def state_dict(self) -> dict:
        return {"t": self.t, "spec": self.name, "keys": {k: [s.cpu() for s in v] for k, v in self._state.items()}}

    def load_state_dict(self, d: dict) -> None:
        self.t = int(d.get("t", 0))
        for k, v in d.get("keys", {}).items():
            self._state[k] = [s.clone() for s in v]

    def __repr__(self):
        return f"{type(self).__name__}({self.name})"


class SimpleUpdater(Updater):
    """w += -eta * dw (update/SimpleUpdater.java:20-22)."""

    kind = _o.SGD
    prefix = "simple"

    def __init__(self, eta: float = 0.01):
        super().__init__()
        self.eta = float(eta)

    def spec_items(self):
        return [("eta", self.eta)]

    def hyper(self, step):
        return dict(lr=self.eta)


class MomentumUpdater(Updater):
    """SGD with (Nesterov) momentum and L2 weight decay -- ResNet-50's optimizer."""

    kind = _o.SGD
    n_state = 1
    prefix = "momentum"

    def __init__(self, lr: float = 0.1, momentum: float = 0.9, weight_decay: float = 0.0, nesterov: bool = False,
                 dampening: float = 0.0):
        super().__init__()
        self.lr, self.momentum, self.weight_decay = float(lr), float(momentum), float(weight_decay)
        self.nesterov, self.dampening = bool(nesterov), float(dampening)

    def spec_items(self):
        return [("lr", self.lr), ("momentum", self.momentum), ("wd", self.weight_decay),
                ("nesterov", float(self.nesterov))]

    def hyper(self, step):
        return dict(lr=self.lr, momentum=self.momentum, wd=self.weight_decay, nesterov=self.nesterov,
                    dampening=self.dampening)


class AdamUpdater(Updater):
    """Adam / AdamW.

    ``bias_correction``: ``"reference"`` divides m, v by the constant (1-beta) exactly like
    update/AdamUpdater.java:63-64 (Q5); ``"step"`` is the standard 1-beta^t; ``"none"``.
    """

    kind = _o.ADAM
    n_state = 2
    prefix = "adam"

    def __init__(self, alfa: float = 0.001, beta1: float = 0.9, beta2: float = 0.999, epsilon: float = 1e-8,
                 bias_correction: str = "step", weight_decay: float = 0.0, adamw: bool = True):
        super().__init__()
        self.alfa, self.beta1, self.beta2, self.epsilon = float(alfa), float(beta1), float(beta2), float(epsilon)
        if bias_correction not in ("reference", "step", "none"):
            raise ValueError(bias_correction)
        self.bias_correction = bias_correction
        self.weight_decay, self.adamw = float(weight_decay), bool(adamw)

    def spec_items(self):
        items = [("alfa", self.alfa), ("beta1", self.beta1), ("beta2", self.beta2), ("epsilon", self.epsilon)]
        if self.bias_correction != "reference":  # reference spec strings imply the constant form
            items.append(("bc", {"step": 1.0, "none": 0.0}[self.bias_correction]))
        return items

    def hyper(self, step):
        if self.bias_correction == "reference":
            bc1, bc2 = 1.0 / (1.0 - self.beta1), 1.0 / (1.0 - self.beta2)
        elif self.bias_correction == "step":
            s = max(1, int(step))
            bc1, bc2 = 1.0 / (1.0 - self.beta1 ** s), 1.0 / (1.0 - self.beta2 ** s)
        else:
            bc1 = bc2 = 1.0
        return dict(lr=self.alfa, beta1=self.beta1, beta2=self.beta2, eps=self.epsilon, bc1=bc1, bc2=bc2,
                    wd=self.weight_decay, adamw=self.adamw)

    def _key_step(self, key, master, states, g):
        # per-key clock for the reference API (each key is its own "t")
        t = getattr(self, "_kt", {})
        self._kt = t
        t[key] = t.get(key, 0) + 1
        self.step_flat(master, states, g, step=t[key])


class OneBitAdamUpdater(AdamUpdater):
    """The owner side of 1-bit Adam (Tang et al. 2021): ``warmup`` full-precision rounds of plain
    Adam, then the workers push their error-compensated 1-bit MOMENTUM (ColocatedPS
    ``compress="onebit"`` + ``onebit_momentum``: ops/compress.onebit_pack with ``mom``) and the
    variance is frozen.  On the owner that is Adam with beta1 = 0 (m := the decoded average of the
    workers' momenta) and beta2 = 1 (v unchanged) -- the same fused kernel, only the per-round
    hyper-parameters change.  ``refresh = k``: every k-th round after the warm-up is again a
    full-precision round (the workers push their gradient) in which the owners' Adam continues
    from the last decoded momentum and updates the variance -- a frozen variance from a short
    warm-up goes stale and the run diverges (profiles/r6_llama8b_onebit_adam.txt).  Compressing
    gradients into an owner Adam with a live variance instead learns far more slowly at 8B depth
    (profiles/r6_llama8b_full_onebit_w2.txt)."""

    prefix = "onebitadam"

    def __init__(self, alfa: float = 0.001, beta1: float = 0.9, beta2: float = 0.999, epsilon: float = 1e-8,
                 bias_correction: str = "step", weight_decay: float = 0.0, adamw: bool = True, warmup: int = 100,
                 refresh: int = 0):
        super().__init__(alfa, beta1, beta2, epsilon, bias_correction, weight_decay, adamw)
        if warmup < 1:
            raise ValueError("1-bit Adam needs >= 1 full-precision warm-up round to form the variance")
        if refresh < 0:
            raise ValueError("refresh >= 0")
        self.warmup, self.refresh = int(warmup), int(refresh)

    def spec_items(self):
        return super().spec_items() + [("warmup", float(self.warmup)), ("refresh", float(self.refresh))]

    def full_round(self, step: int) -> bool:
        """Whether step (1-based; round r is step r + 1) pushes full-precision gradients."""
        return step <= self.warmup or (self.refresh > 0 and (step - self.warmup) % self.refresh == 0)

    def _n_full(self, step: int) -> int:
        return step if step <= self.warmup else self.warmup + (
            (step - self.warmup) // self.refresh if self.refresh else 0)

    def hyper(self, step):
        if step <= self.warmup:
            return super().hyper(step)
        h = super().hyper(self.warmup)
        nf = self._n_full(step)
        if self.bias_correction == "step":
            h["bc2"] = 1.0 / (1.0 - self.beta2 ** nf)  # v has seen nf updates
        h["bc1"] = 1.0  # m continues from the workers' momenta, past its start-up bias
        if not self.full_round(step):
            h.update(beta1=0.0, beta2=1.0)
        return h


class AdagradUpdater(Updater):
    """h += g^2; w -= lr g / (sqrt(h) + eps) (north-star DLRM tables, K24)."""

    kind = _o.ADAGRAD
    n_state = 1
    prefix = "adagrad"

    def __init__(self, lr: float = 0.01, epsilon: float = 1e-10, weight_decay: float = 0.0, rowwise: bool = False):
        super().__init__()
        self.lr, self.epsilon, self.weight_decay, self.rowwise = float(lr), float(epsilon), float(weight_decay), rowwise

    def spec_items(self):
        return [("lr", self.lr), ("epsilon", self.epsilon), ("rowwise", float(self.rowwise))]

    def hyper(self, step):
        return dict(lr=self.lr, eps=self.epsilon, wd=self.weight_decay)


class FtrlUpdater(Updater):
    """FTRL-proximal.  ``mode="reference"`` reproduces update/FtrlUpdater.java:51-76 exactly
    (weights computed from (z, n_old) first, sigma = sqrt(n+g^2) - sqrt(n/alpha), l2 divided by
    alpha, and the whole key skipped when dw[0] == 0); ``mode="canonical"`` is McMahan et al."""

    kind = _o.FTRL
    n_state = 2
    prefix = "ftrl"

    def __init__(self, alfa: float = 0.005, beta: float = 1.0, l1: float = 0.001, l2: float = 0.001,
                 mode: str = "canonical"):
        super().__init__()
        self.alfa, self.beta, self.l1, self.l2 = float(alfa), float(beta), float(l1), float(l2)
        if mode not in ("reference", "canonical"):
            raise ValueError(mode)
        self.mode = mode

    def spec_items(self):
        items = [("alfa", self.alfa), ("beta", self.beta), ("l1", self.l1), ("l2", self.l2)]
        if self.mode == "reference":
            items.append(("reference", 1.0))
        return items

    def hyper(self, step):
        return dict(lr=self.alfa, fbeta=self.beta, l1=self.l1, l2=self.l2,
                    ftrl_mode=1 if self.mode == "reference" else 0)

    def _key_step(self, key, master, states, g):
        if self.mode == "reference" and float(g.reshape(-1)[0]) == 0.0:
            return  # FtrlUpdater.java:52-54
        self.step_flat(master, states, g)


_KINDS = {
    "simple": SimpleUpdater,
    "sgd": SimpleUpdater,
    "momentum": MomentumUpdater,
    "adam": AdamUpdater,
    "adagrad": AdagradUpdater,
    "ftrl": FtrlUpdater,
}


def parse_updater(spec: str) -> Updater:
    """Build an updater from a spec string.

    Accepts the reference formats (``simple@eta:0.1@``, ``adam@alfa:..@beta1:..@beta2:..@epsilon:..@``,
    and FTRL's ``adam@alfa:..@beta:..@l1:..@l2:..@`` which the reference emits by mistake) plus
    ``momentum@lr:..@momentum:..@wd:..@``, ``adagrad@lr:..@epsilon:..@``, ``ftrl@alfa:..@beta:..@l1:..@l2:..@``.
    """
    head = spec.split("@", 1)[0].strip().lower()
    g = lambda k, d=None: float(_between(spec, k)) if _between(spec, k) is not None else d  # noqa: E731
    if head == "adam" and _between(spec, "l1") is not None:
        # reference FtrlUpdater.getName() quirk (Q6): such strings come from the reference
        return FtrlUpdater(g("alfa", 0.005), g("beta", 1.0), g("l1", 0.001), g("l2", 0.001), mode="reference")
    if head in ("simple", "sgd"):
        return SimpleUpdater(g("eta", 0.01))
    if head == "momentum":
        return MomentumUpdater(g("lr", 0.1), g("momentum", 0.9), g("wd", 0.0), bool(g("nesterov", 0.0)))
    if head == "adam":
        bc = {0: "none", 1: "step", 2: "reference"}.get(int(g("bc", 2)), "reference")
        return AdamUpdater(g("alfa", 0.001), g("beta1", 0.9), g("beta2", 0.999), g("epsilon", 1e-8), bc)
    if head == "adagrad":
        return AdagradUpdater(g("lr", 0.01), g("epsilon", 1e-10), rowwise=bool(g("rowwise", 0.0)))
    if head == "ftrl":
        return FtrlUpdater(g("alfa", 0.005), g("beta", 1.0), g("l1", 0.001), g("l2", 0.001),
                           mode="reference" if g("reference", 0.0) else "canonical")
    raise ValueError(f"unknown updater spec {spec!r}")


def resolve_updater(key: str, updaters: Dict[str, Updater]) -> Updater:
    """exact key -> longest matching prefix -> "default" (store/KVStore.java:242-252; the
    reference picks the LAST matching prefix in hash-map order -- we pick the longest)."""
    if key in updaters:
        return updaters[key]
    best = None
    for p, u in updaters.items():
        if p != "default" and key.startswith(p) and (best is None or len(p) > len(best)):
            best = p
    if best is not None:
        return updaters[best]
    if "default" in updaters:
        return updaters["default"]
    raise KeyError(f"no updater for key {key!r} and no 'default'")


def lr_cosine(base: float, step: int, total: int, warmup: int = 0) -> float:
    """Cosine LR schedule helper (host-side hyper-parameter, passed to the kernel per round)."""
    if warmup and step < warmup:
        return base * (step + 1) / warmup
    p = min(1.0, (step - warmup) / max(1, total - warmup))
    return 0.5 * base * (1 + math.cos(math.pi * p))
