#!/bin/bash
# Stem forward at four blocks per CU (4 x 1 wave layout, 104 VGPRs): tests, bench, step profile.
O=gpurun_out/r4stem
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pool_gpu.py tests/test_bn_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 8 > $O/bench_$i.log 2>&1 || exit $?
  grep '"metric"' $O/bench_$i.log | cut -c1-200
done
timeout -k 10 200 python bench.py --batch-per-gpu 256 --steps 20 --warmup 8 > $O/bench256.log 2>&1 || exit $?
grep '"metric"' $O/bench256.log | cut -c1-200
bash scripts/gpu_prof_step.sh $O/p1024 > /dev/null 2>&1 || exit $?
grep -E "stem|pool|maxpool" $O/p1024/breakdown.txt
