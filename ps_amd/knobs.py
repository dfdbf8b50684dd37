"""Route switches: ONE environment variable turns off any of the fused / HIP routes.

``PS_AMD_DISABLE=route[,route...]`` selects, for each named route, the plain path that is also
that route's numerics oracle in the tests (README "Knobs" lists every ``PS_AMD_*`` variable with
its default; the tuning thresholds the A/B records settled are constants in the code, and the
variants they rejected were removed in round 6 -- their records stay in ``profiles/``).

The variable is read on every query (parsed once per distinct value), so a test flips a route
in-process with ``monkeypatch.setenv("PS_AMD_DISABLE", "fold_bn3")``.
"""
from __future__ import annotations

import os
from typing import Dict, FrozenSet

ENV = "PS_AMD_DISABLE"

# route -> what turning it off selects instead
ROUTES: Dict[str, str] = {
    # ResNet-50 (ops/convgemm.py, ops/conv.py, models/resnet.py)
    "fused_block": "bottlenecks module by module (nn.Conv2d on MIOpen + BatchNormAct2d)",
    "conv3x3": "fused blocks' 3x3 convolutions on MIOpen instead of the implicit-GEMM kernels",
    "block_out": "block outputs applied by their own pass, not in the next conv1's prologue",
    "fold_bn3": "bn3's backward reduce as its own pass, not in the consumer's conv1 data-gradient epilogue",
    "fold_bn_ds": "the downsample BN's backward reduce as its own pass (epilogue 8 instead of 9)",
    "conv3_bwd_fused": "conv3's data + weight gradient as two GEMMs (dz3 through HBM)",
    "ds_bwd_fused": "the downsample's data + weight gradient as apply pass + two GEMMs",
    "weight_prep": "backward weight layouts built per block instead of in one launch per forward",
    "pool_bn_bwd": "stem max-pool backward and BN backward as separate passes",
    "stem_bwd_fused": "stem weight gradient reading a materialised dz",
    # dense / transformer (ops/dense.py, ops/linear.py, ops/transformer.py)
    "splitk_wgrad": "linear weight gradients on hipBLASLt instead of the split-K kernel",
    "linear_fork": "linear weight gradients on the compute stream",
    "fused_relu": "Linear + ReLU as separate ops",
    "ps_linear": "PS-owned linear weight gradients through autograd's ordinary accumulation",
    "fused_attn": "short-sequence attention on SDPA",
    "flash_attn": "causal GQA attention on SDPA",
    "fused_xent": "cross-entropy on fp32 logits through F.cross_entropy",
}

_cache: Dict[str, FrozenSet[str]] = {}


def _parse(raw: str) -> FrozenSet[str]:
    got = _cache.get(raw)
    if got is None:
        got = frozenset(s.strip() for s in raw.split(",") if s.strip())
        bad = sorted(got - set(ROUTES))
        if bad:
            raise ValueError(f"{ENV}: unknown route(s) {bad}; known: {sorted(ROUTES)}")
        _cache[raw] = got
    return got


def disabled(route: str) -> bool:
    """True when ``route`` is listed in PS_AMD_DISABLE."""
    if route not in ROUTES:
        raise KeyError(f"unknown route {route!r}")
    raw = os.environ.get(ENV)
    return bool(raw) and route in _parse(raw)


def enabled(route: str) -> bool:
    return not disabled(route)
