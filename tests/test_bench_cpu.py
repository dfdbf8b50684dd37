"""bench.py driver contract, exercised on CPU tensors over gloo (``--device cpu``): the same
torchrun self-launch, barrier-bracketed timed region, MAX-over-ranks elapsed time, per-phase PS
timing and collective probe as the multi-GPU runs, ending in exactly ONE JSON line from rank 0
with the BASELINE.json metric."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [1, 2])
def test_bench_json_contract_cpu(world, tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", str(world), "--steps", "2",
           "--warmup", "1", "--batch-per-gpu", "2", "--image-size", "32"]
    out = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=540)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert KEYS <= set(rec)
    baseline = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert rec["metric"] == baseline["metric"]
    assert rec["n_gpus"] == world and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["config"]["model"] == "ResNet-50" and rec["config"]["global_batch"] == 2 * world
    # value is the whole-job rate: global batch x steps / (max over ranks of the timed region)
    assert rec["value"] == pytest.approx(2 * world * 1e3 / rec["ms_per_step"], rel=1e-2)
    # stream policy fields: keyed on ranks sharing a device (CPU ranks never share one)
    assert rec["config"]["ranks_per_device"] == 1
    assert rec["config"]["compute_priority"] == "normal" and rec["config"]["side_stream"] is False
    assert rec["config"]["streams_per_rank"] == 0
    if world > 1:
        assert set(rec["config"]["ps_phase_ms_per_step"]) >= {"push_ms", "serve_ms", "pull_ms"}
        if rec["config"].get("data_plane") == "xgmi":  # mapping mode / self-test / round end reported
            assert {"mode", "self_test", "round_end"} <= set(rec["config"]["plane_info"])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("config,extra", [("dlrm", ["--dlrm-rows", "2000", "--batch-per-gpu", "32"]),
                                          ("ctr-async", ["--batch-per-gpu", "32"]),
                                          ("llama-onebit", ["--tiny", "1", "--batch-per-gpu", "2", "--seq-len", "32"])])
def test_other_bench_configs_build_and_step_cpu(config, extra, tmp_path):
    """Every non-default bench config builds and times a step on CPU (world 1): a config that no
    longer constructs fails here, not on the GPU box."""
    env = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--config", config, "--steps", "1",
           "--warmup", "1"] + extra
    out = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=540)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert KEYS <= set(rec) and rec["value"] > 0
