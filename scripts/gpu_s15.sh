#!/bin/bash
mkdir -p gpurun_out/s15
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
timeout -k 10 600 python -m pytest tests/test_bn_gpu.py tests/test_pool_gpu.py -q > gpurun_out/s15/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/s15/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 30 --warmup 5 > gpurun_out/s15/bench.log 2>&1 || exit $?
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s15/prof -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 3 > $R/gpurun_out/s15/prof.log 2>&1 || exit $?
exit 0
