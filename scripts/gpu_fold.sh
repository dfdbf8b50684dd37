#!/bin/bash
# bn3 backward reduce folded into the next block's conv1 data-grad epilogue: tests, bench, trace.
mkdir -p gpurun_out/fold
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_convgemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fold/pytest_conv.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/fold/pytest_conv.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fold/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/fold/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/fold/bench.log 2>&1 || exit $?
timeout -k 10 300 env PS_AMD_FOLD_BN3=0 python bench.py > gpurun_out/fold/bench_nofold.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/fold/prof -o run -- python3 bench.py --steps 10 --warmup 5 > gpurun_out/fold/bench_prof.log 2>&1 || exit $?
exit 0
