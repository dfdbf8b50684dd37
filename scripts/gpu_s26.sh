#!/bin/bash
mkdir -p gpurun_out/s26
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s26/prof -o run --output-format csv -- python3 $R/bench.py --config llama-onebit --steps 3 --warmup 2 --timing 2 > $R/gpurun_out/s26/prof.log 2>&1 || exit $?
exit 0
