#!/bin/bash
# BN + conv GEMM numerics, then a kernel trace of the bench step
mkdir -p gpurun_out/v18
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest tests/test_convgemm_gpu.py tests/test_bn_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/v18/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/v18/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 8 > gpurun_out/v18/bench.log 2>&1 || exit $?
bash scripts/gpu_trace1.sh
