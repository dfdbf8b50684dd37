#!/bin/bash
# rocprofv3 kernel stats of the BERT-SSP bench -> gpurun_out/pb/
O=gpurun_out/pb
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python $R/bench.py --config bert-ssp --steps 4 --warmup 2 > $R/$O/prof.log 2>&1 || exit $?
cd $R && python scripts/kernel_stats_top.py $O/prof/run_kernel_stats.csv 45 > $O/top.txt 2>&1; head -40 $O/top.txt; tail -1 $O/prof.log | cut -c1-200
