#!/bin/bash
# Stem max-pool forward with the nine taps loaded together (k = 3, BN prologue): tests, bench, profile.
O=gpurun_out/r4pool
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pool_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 8 > $O/bench_$i.log 2>&1 || exit $?
  grep '"metric"' $O/bench_$i.log | cut -c1-190
done
timeout -k 10 200 python bench.py --batch-per-gpu 256 --steps 20 --warmup 8 > $O/bench256.log 2>&1 || exit $?
grep '"metric"' $O/bench256.log | cut -c1-190
bash scripts/gpu_prof_step.sh $O/p1024 > /dev/null 2>&1 || exit $?
grep -E "maxpool|stem_conv|pool_bn" $O/p1024/timeline.txt | cut -c1-120
