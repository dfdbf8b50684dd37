#!/bin/bash
# GPU validation: selected (or all) gpu tests under a time limit, logs under gpurun_out/
# usage: bash scripts/gpu_tests.sh [pytest target ...]
mkdir -p gpurun_out/tests
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
targets=${@:-tests}
timeout -k 10 900 python -u -m pytest $targets -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/tests/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/tests/pytest.log
tail -5 gpurun_out/tests/pytest.log
exit $rc
