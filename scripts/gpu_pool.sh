#!/bin/bash
# 32-bit index math in the NHWC maxpool kernels: pool tests, bench, trace.
mkdir -p gpurun_out/pool
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_pool_gpu.py tests/test_zoo_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pool/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/pool/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/pool/bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pool/prof -o run -- python3 bench.py --steps 10 --warmup 5 > gpurun_out/pool/bench_prof.log 2>&1 || exit $?
exit 0
