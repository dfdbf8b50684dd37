#!/bin/bash
mkdir -p gpurun_out/s22
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s22/prof -o run --output-format csv -- python3 $R/bench.py --config bert-ssp --steps 6 --warmup 3 > $R/gpurun_out/s22/prof.log 2>&1 || exit $?
exit 0
