#!/bin/bash
mkdir -p gpurun_out/s18
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
timeout -k 10 300 python -m pytest tests/test_pool_gpu.py -q -k stem > gpurun_out/s18/pytest_stem.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/s18/pytest_stem.log
if [ $rc -ne 0 ]; then exit 0; fi
timeout -k 10 600 python -m pytest tests/test_pool_gpu.py tests/test_bn_gpu.py tests/test_zoo_gpu.py -q > gpurun_out/s18/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/s18/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 30 --warmup 5 > gpurun_out/s18/bench.log 2>&1 || exit $?
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s18/prof -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 3 > $R/gpurun_out/s18/prof.log 2>&1 || exit $?
exit 0
