"""Tuned solution choices for the plain library GEMMs (hipBLASLt / rocBLAS through PyTorch TunableOp).

The transformer configs' linears are plain GEMMs, and those stay on the vendor library (the fused
conv / attention / split-K work is in our own HIP kernels).  hipBLASLt's heuristic returns one
solution per shape; TunableOp times the candidates and keeps the fastest.  Tuning is done once on an
MI355X (``scripts/runs/gpu_round5_tunable.sh``) and the result -- a CSV of (op, shape) -> solution,
with the PyTorch / ROCm / hipBLASLt versions and the GPU arch as validators -- ships in
``ps_amd/tuning/``.  At run time the table is only READ (tuning off), so a step never times
candidates.  A table whose validators do not match the running stack is ignored by TunableOp.

``PS_AMD_GEMM_TUNING``: ``auto`` (default: the shipped table for the config, if there is one),
``off``, or a path to a CSV.
"""
from __future__ import annotations

import os
import tempfile
from typing import Optional

import torch

_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning")


def table_for(config: str) -> Optional[str]:
    mode = os.environ.get("PS_AMD_GEMM_TUNING", "auto")
    if mode == "off":
        return None
    path = os.path.join(_DIR, f"{config}_gfx950.csv") if mode == "auto" else mode
    return path if os.path.isfile(path) else None


def load(config: str, device: torch.device) -> Optional[str]:
    """Enable TunableOp lookups from the config's tuned table; returns the table's path or None."""
    path = table_for(config)
    if path is None or device.type != "cuda":
        return None
    if not torch.cuda.get_device_properties(device).gcnArchName.startswith("gfx950"):
        return None
    tun = torch.cuda.tunable
    # results TunableOp would write at exit go to a scratch file, never over the shipped table
    tun.set_filename(os.path.join(tempfile.gettempdir(), f"psamd_tunableop_{os.getpid()}_%d.csv"))
    tun.enable(True)
    tun.tuning_enable(False)
    tun.read_file(path)
    return path
