#!/bin/bash
mkdir -p gpurun_out/s16
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace -d $R/gpurun_out/s16/prof -o run --output-format csv -- python3 $R/scripts/probe_bn.py > $R/gpurun_out/s16/prof.log 2>&1 || exit $?
cd $R && python scripts/probe_bn.py --report gpurun_out/s16/prof/run_kernel_trace.csv > gpurun_out/s16/bn_bw.txt 2>&1
exit 0
