#!/bin/bash
mkdir -p gpurun_out/s6
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for cfg in "256 0" "256 1" "512 0" "384 0"; do
  set -- $cfg
  timeout -k 10 900 python bench.py --steps 20 --warmup 5 --batch-per-gpu $1 --graph $2 > gpurun_out/s6/bench_b$1_g$2.log 2>&1 || exit $?
done
exit 0
