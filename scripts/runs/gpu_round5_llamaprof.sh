#!/bin/bash
# Llama-3-8B (llama-onebit config, world 1) kernel stats: where the 815 ms step goes
set -o pipefail
O=gpurun_out/r5llamaprof
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python $R/bench.py --config llama-onebit --steps 3 --warmup 2 > $R/$O/prof.log 2>&1
