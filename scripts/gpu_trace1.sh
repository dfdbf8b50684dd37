#!/bin/bash
# kernel trace of the ResNet-50 bench step (per-family breakdown + per-call conv GEMM times)
mkdir -p gpurun_out/trace1
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace1/prof -o run --output-format csv \
  -- python3 $R/bench.py --steps 6 --warmup 4 > $R/gpurun_out/trace1/bench.log 2>&1 || exit $?
cd $R && python scripts/step_breakdown.py gpurun_out/trace1/prof/run_kernel_trace.csv > gpurun_out/trace1/breakdown.txt 2>&1
python scripts/kernel_calls.py gpurun_out/trace1/prof/run_kernel_trace.csv "" > gpurun_out/trace1/calls.txt 2>&1
rm -f gpurun_out/trace1/prof/run_kernel_trace.csv.gz
exit 0
