"""Start-up probe of the one-sided REMOTE-WRITE paths (VERDICT r5 Next #2).

The reference's server receives pushes over gRPC and inserts them into its own store
(net/PServer.java:143-195).  The one-sided paths here write straight into the owner's memory and
rely on the owner's read path to see those bytes:

* AsyncPS push: a worker's copy kernel (csrc/kernels/plane.hip, ``plane.copy_many``) writes the
  bucket into the owner's IPC-mapped mailbox; the owner's native thread observes the completion
  through the control block and reads the mailbox in a kernel that starts with a system-scope
  acquire (``fused_opt_multi``);
* row plane response: the owner's ``row_plane_send`` kernel writes rows into every worker's
  arena; the worker's stream waits on the owners' inter-process events and reads its own arena.

Those reads had only ever run with every rank in one L2 domain (one GPU).  Before the first real
round, every rank writes a pattern into every peer by the PRODUCTION write kernel, publishes it by
the PRODUCTION protocol, and the reader reads it by the PRODUCTION read path -- ``rounds`` times
over the SAME lines, with the reader having read them already (a stale cached line shows as the
previous round's value).  All ranks agree on the outcome (``all_gather``, like the xGMI plane's
self-test, plane.py ``_agree``); on any failure every rank raises ``RemoteWriteUnavailable`` and
the caller falls back uniformly (AsyncPS -> pipelined collective SSP, row plane -> RCCL
all-to-alls).  ``PS_AMD_PROBE_FAIL=kind[@rank][,...]`` (kind: asyncps | rowplane | asyncrows |
all) injects a failure, for the fallback tests.
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import torch

from .transport import Transport


class RemoteWriteUnavailable(RuntimeError):
    """A one-sided remote-write path failed its start-up probe on some rank (same on every rank)."""


def injected(kind: str, rank: int) -> bool:
    for item in filter(None, (s.strip() for s in os.environ.get("PS_AMD_PROBE_FAIL", "").split(","))):
        k, _, r = item.partition("@")
        if k in (kind, "all") and (not r or int(r) == rank):
            return True
    return False


def run_probe(t: Transport, kind: str, rounds: int, write: Callable[[int], None], publish: Callable[[int], None],
              read: Callable[[int], torch.Tensor], want: Callable[[int], torch.Tensor],
              settle: Callable[[], None]) -> str:
    """Run ``rounds`` write -> publish -> read rounds (``settle`` after each read: this rank's reads
    are complete before any peer overwrites the lines), agree across ranks, return the record
    string for the engine's ``info`` or raise ``RemoteWriteUnavailable`` everywhere."""
    errs_local = []

    def step(fn):
        # every rank runs every step (the collective parts of publish / settle line up even
        # after a failure on one rank); the first error is the one reported
        try:
            return fn()
        except Exception as e:  # noqa: BLE001 -- a failing mapping / launch is a probe failure too
            errs_local.append(f"{type(e).__name__}: {e}")
            return None

    for k in range(-1, rounds):  # k = -1: the reader has the lines (zeros) before any remote write
        if k >= 0:
            step(lambda: write(k))
            step(lambda: publish(k))
        got = step(lambda: read(k))
        if k >= 0 and got is not None and not errs_local:
            exp = want(k)
            if not torch.equal(got, exp):
                bad = (got != exp).nonzero()
                i = tuple(int(v) for v in bad[0])
                errs_local.append(f"round {k}: read {float(got[i])} at {i}, expected {float(exp[i])} "
                                  f"({bad.shape[0]} of {exp.numel()} values wrong)")
        step(settle)
    err: Optional[str] = errs_local[0] if errs_local else None
    if err is None and injected(kind, t.rank):
        err = "injected failure (PS_AMD_PROBE_FAIL)"
    errs = t.all_gather_object(err) if t.world > 1 else [err]
    bad = {r: e for r, e in enumerate(errs) if e is not None}
    if bad:
        raise RemoteWriteUnavailable(f"{kind} remote-write probe failed on ranks {sorted(bad)}: "
                                     + "; ".join(f"rank {r}: {e}" for r, e in bad.items()))
    return f"ok ({rounds} rounds of peer writes over the same lines, production write + read path)"


def pattern(k: int, src: int, n: int) -> torch.Tensor:
    """The n fp32 values rank ``src`` writes in round ``k`` (each writer has lines of its own in
    the reader's buffer; values < 80, exact in bf16 too, and different in every round)."""
    return float(16 * (k + 1) + 4 * (src % 4)) + torch.arange(n, dtype=torch.float32) % 4
