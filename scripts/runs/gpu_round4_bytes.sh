#!/bin/bash
# HBM bytes per kernel over the ResNet-50 bs1024 step: FETCH_SIZE and WRITE_SIZE in separate passes
# (the TCC block holds 4 counters: FETCH_SIZE takes 3, WRITE_SIZE 2), kernel trace only.
mkdir -p gpurun_out/r4bytes
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp
pass() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" -d $R/gpurun_out/r4bytes/$name -o run --output-format csv \
    -- python3 $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/r4bytes/$name.log 2>&1
}
pass fetch FETCH_SIZE || exit $?
pass write WRITE_SIZE || exit $?
cd $R && python3 scripts/pmc_summary.py gpurun_out/r4bytes/fetch gpurun_out/r4bytes/write --match conv_ bn_ stem pool \
  > gpurun_out/r4bytes/summary.txt
find gpurun_out/r4bytes -name '*kernel_trace.csv' -delete
find gpurun_out/r4bytes -name '*counter_collection.csv' -delete
wc -l gpurun_out/r4bytes/summary.txt
