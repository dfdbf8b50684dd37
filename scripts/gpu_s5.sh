#!/bin/bash
mkdir -p gpurun_out/s5
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python scripts/probe_conv1x1.py > gpurun_out/s5/conv1x1.log 2>&1 || exit $?
exit 0
