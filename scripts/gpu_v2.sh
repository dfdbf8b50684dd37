#!/bin/bash
# Per-shape conv timing (MIOpen / hipBLASLt vs roofline) at batch 512.
mkdir -p gpurun_out/v2
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u scripts/probe_convs.py 512 > gpurun_out/v2/probe_convs_b512.jsonl 2> gpurun_out/v2/probe_convs.err || exit $?
exit 0
