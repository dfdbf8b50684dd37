#!/bin/bash
# per-kernel split of the flash probe (fwd / dQ / dKdV vs SDPA's kernels)
mkdir -p gpurun_out/r3h
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3h/prof -o run -- python $R/scripts/probe_flash.py 4 > $R/gpurun_out/r3h/probe.log 2>&1 || exit $?
python $R/scripts/kernel_stats_top.py $(find $R/gpurun_out/r3h/prof -name '*kernel_stats.csv' | head -1) 12 > $R/gpurun_out/r3h/top.txt || exit $?
find $R/gpurun_out/r3h/prof -name '*kernel_trace.csv' -delete
cat $R/gpurun_out/r3h/top.txt
