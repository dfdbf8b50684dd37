#!/bin/bash
# HBM bytes per kernel over ResNet-50 steps (FETCH_SIZE / WRITE_SIZE passes, kernel-trace only) +
# a clean kernel trace for durations -> gpurun_out/pmcstep/summary.txt
bash scripts/runs/gpu_pmc_step.sh || exit $?
R=$PWD
mkdir -p gpurun_out/pmcstep/clean
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/pmcstep/clean -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 > $R/gpurun_out/pmcstep/clean.log 2>&1 || exit $?
cd $R && python3 scripts/pmc_step_summary.py gpurun_out/pmcstep/fetch gpurun_out/pmcstep/write $(ls gpurun_out/pmcstep/clean/*kernel_trace.csv | head -1) --top 45 > gpurun_out/pmcstep/summary.txt 2>&1
head -30 gpurun_out/pmcstep/summary.txt
