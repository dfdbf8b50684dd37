#!/bin/bash
# Re-validation after container re-creation: full GPU suite, smoke, default bench.
mkdir -p gpurun_out/v1
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/v1/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/v1/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/v1/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/v1/bench.log 2>&1 || exit $?
exit 0
