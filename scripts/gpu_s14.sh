#!/bin/bash
mkdir -p gpurun_out/s14
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -m pytest tests/test_pool_gpu.py -q > gpurun_out/s14/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/s14/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 30 --warmup 5 > gpurun_out/s14/bench.log 2>&1 || exit $?
timeout -k 10 300 python scripts/probe_gemm.py > gpurun_out/s14/gemm.log 2>&1 || exit $?
exit 0
