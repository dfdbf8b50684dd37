#!/bin/bash
# conv-GEMM GPU tests, then the default bench and a kernel-trace step breakdown (A/B of a conv change)
O=${1:-gpurun_out/ab}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest ${AB_TESTS:-tests/test_convgemm_gpu.py tests/test_bn_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-220
bash scripts/gpu_prof_step.sh $O/pstep > /dev/null || exit $?
head -12 $O/pstep/breakdown.txt
