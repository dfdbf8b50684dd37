#!/bin/bash
# ResNet-50 step trace after the epilogue spill fix: family breakdown + per-kernel aggregate
bash scripts/gpu_prof_step.sh gpurun_out/r3as || exit $?
python3 scripts/kernel_agg.py $(ls gpurun_out/r3as/prof/*kernel_trace.csv | head -1) 9 60 > gpurun_out/r3as/per_kernel.txt
find gpurun_out/r3as -name "*.csv" -delete
