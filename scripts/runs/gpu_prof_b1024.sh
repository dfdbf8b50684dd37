#!/bin/bash
# ResNet-50 bs1536/2048 sweep + rocprofv3 kernel trace of the bs1024 step (per-family breakdown)
mkdir -p gpurun_out/p1024
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
for b in 1536 2048; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 4 --batch-per-gpu $b --json-out gpurun_out/p1024/b$b.json > gpurun_out/p1024/b$b.log 2>&1 || exit $?
done
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p1024/prof -o run --output-format csv -- python $R/bench.py --steps 6 --warmup 3 --batch-per-gpu 1024 > $R/gpurun_out/p1024/prof.log 2>&1 || exit $?
cd $R && python scripts/step_breakdown.py $(ls gpurun_out/p1024/prof/*kernel_trace.csv | head -1) > gpurun_out/p1024/breakdown.txt
head -45 gpurun_out/p1024/breakdown.txt
cat gpurun_out/p1024/b*.json | cut -c1-200
