#!/bin/bash
# conv GEMM micro-benchmark + available PMC counters on gfx950
R=$PWD
mkdir -p gpurun_out/v4
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u scripts/probe_convgemm.py > gpurun_out/v4/probe.jsonl 2>&1 || exit $?
cd /tmp && timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/v4/counters.txt 2>&1
exit 0
