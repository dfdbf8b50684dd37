#!/bin/bash
# BN Welford stats: numerics + e2e + bench regression check
mkdir -p gpurun_out/s10
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -m pytest tests/test_bn_gpu.py -q > gpurun_out/s10/pytest.log 2>&1
echo "rc=$?" >> gpurun_out/s10/pytest.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/s10/bench.log 2>&1
echo "rc=$?" >> gpurun_out/s10/bench.log
exit 0
