#!/bin/bash
# GPU tests of a change, then the default bench under each env setting given as arguments
# (e.g. "PS_AMD_MAT_Y2_MIN_C=0" "PS_AMD_MAT_Y2_MIN_C=128"); logs under gpurun_out/abenv/
O=gpurun_out/abenv
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest ${AB_TESTS:-tests/test_convgemm_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
i=0
for kv in "$@"; do
  i=$((i+1))
  env $kv timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_$i.log 2>&1 || exit $?
  echo "$kv $(tail -1 $O/bench_$i.log | cut -c100-175)"
done
