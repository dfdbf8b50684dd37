"""SURVEY §5.2 b: stream/event discipline -- the same training steps give bitwise-identical
results with every kernel serialised (AMD_SERIALIZE_KERNEL=3, HIP_LAUNCH_BLOCKING=1) as in
the normal asynchronous multi-stream run; a missing event wait would show up as a diff."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra_env):
    env = {**os.environ, **extra_env}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "_serialize_child.py"), ROOT],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("DIGEST")][-1]
    return line.split()[1]


def test_serialized_kernels_give_identical_results():
    normal = _run({})
    serial = _run({"AMD_SERIALIZE_KERNEL": "3", "HIP_LAUNCH_BLOCKING": "1"})
    assert normal == serial
    assert normal == _run({})  # and the async run is itself deterministic
