#!/bin/bash
# fc.hip v3 (layout-preserving LDS + transposed fragment reads, dW/dX in one launch): numerics + probe
mkdir -p gpurun_out/r3m
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_fc_gpu.py tests/test_zoo_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3m/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3m/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_fc.py > gpurun_out/r3m/fc_probe.jsonl 2>gpurun_out/r3m/fc_probe.err || exit $?
cut -c1-250 gpurun_out/r3m/fc_probe.jsonl
