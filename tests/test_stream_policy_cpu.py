"""Stream policy keyed on ranks per DEVICE, not on WORLD_SIZE (VERDICT r4 Next #2).

The weight-gradient side stream and the high-priority compute stream were tuned on a single
process; on a node every rank owns its GPU, which is that same case.  Only ranks that share one
GPU (the one-GPU rehearsals) keep the single-stream path at large batches."""
import pytest
import torch.distributed as dist

from ps_amd.ops import side_stream
from ps_amd.parallel import transport
from tests.dist_util import run


def test_count_sharing():
    keys = ["h/gpu/A", "h/gpu/B", "h/gpu/A", "h/gpu/C"]
    assert transport.count_sharing(keys, 0) == 2
    assert transport.count_sharing(keys, 1) == 1
    assert transport.count_sharing(keys, 2) == 2
    assert transport.count_sharing(["h/gpu/A"] * 8, 5) == 8
    assert transport.count_sharing([f"h/gpu/{i}" for i in range(8)], 7) == 1


@pytest.mark.parametrize("rpd,images,expect", [(1, 1024, True), (1, 256, True), (2, 1024, False),
                                               (2, 512, True), (4, 256, True), (8, 2048, False)])
def test_side_stream_policy_keys_on_ranks_per_device(monkeypatch, rpd, images, expect):
    monkeypatch.delenv("PS_AMD_WGRAD_STREAM", raising=False)
    monkeypatch.delenv("PS_AMD_WGRAD_STREAM_MAX_IMAGES", raising=False)
    monkeypatch.setattr(transport, "_RANKS_PER_DEVICE", rpd)
    # WORLD_SIZE plays no part: a real 8-GPU node (8 ranks, one per GPU) is the single-process case
    monkeypatch.setenv("WORLD_SIZE", "8")
    assert side_stream.enabled(images) is expect


def test_side_stream_policy_overrides(monkeypatch):
    monkeypatch.setattr(transport, "_RANKS_PER_DEVICE", 4)
    monkeypatch.setenv("PS_AMD_WGRAD_STREAM", "1")
    assert side_stream.enabled(4096)
    monkeypatch.setenv("PS_AMD_WGRAD_STREAM", "0")
    assert not side_stream.enabled(64)
    monkeypatch.delenv("PS_AMD_WGRAD_STREAM")
    monkeypatch.setenv("PS_AMD_WGRAD_STREAM_MAX_IMAGES", "128")
    assert not side_stream.enabled(256) and side_stream.enabled(128)


def _rpd_body(tp, shared):
    if shared:  # every rank claims the same device, as W processes on cuda:0 do
        transport.device_key = lambda device=None: "host/gpu/shared"
    n = transport.ranks_per_device(refresh=True)
    keys = [None] * tp.world
    dist.all_gather_object(keys, n)
    return keys


@pytest.mark.parametrize("shared", [False, True])
def test_ranks_per_device_gloo(shared):
    out = run(_rpd_body, 2, args=(shared,))
    assert out[0] == ([2, 2] if shared else [1, 1])


def _lazy_body(tp):
    # a process group made outside init_distributed: a policy query must not start a collective
    # (rank 1 never calls it, so a lazy all_gather would hang the job)
    transport._RANKS_PER_DEVICE = None
    n = transport.ranks_per_device() if tp.rank == 0 else 1
    return n, transport._RANKS_PER_DEVICE


def test_ranks_per_device_policy_query_is_not_a_collective():
    out = run(_lazy_body, 2)
    assert out[0] == (1, None)  # CPU ranks: the env estimate, cache left for the collective count
