#!/bin/bash
# Gradient landing + channels_last keys + NHWC avgpool backward: GPU suite, bench, kernel trace.
mkdir -p gpurun_out/land
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/land/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/land/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/land/bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/land/prof -o run -- python3 bench.py --steps 10 --warmup 5 > gpurun_out/land/bench_prof.log 2>&1 || exit $?
exit 0
