#!/bin/bash
# HBM bytes (FETCH_SIZE / WRITE_SIZE) and MFMA activity per kernel over ResNet-50 training steps:
# one counter group per rocprofv3 run, kernel-trace only.
mkdir -p gpurun_out/pmcstep
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp
pass() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" -d $R/gpurun_out/pmcstep/$name -o run --output-format csv \
    -- python3 $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/pmcstep/$name.log 2>&1
}
pass fetch FETCH_SIZE || exit $?
pass write WRITE_SIZE || exit $?
pass mfma SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES || exit $?
exit 0
