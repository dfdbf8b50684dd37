#!/bin/bash
# BERT-base SSP(1) kernel stats: where the 100 ms step goes
set -o pipefail
O=gpurun_out/r5bertprof
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python $R/bench.py --config bert-ssp --steps 10 --warmup 3 > $R/$O/prof.log 2>&1
