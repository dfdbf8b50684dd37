#!/bin/bash
mkdir -p gpurun_out/s13
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 900 python scripts/probe_convs.py 512 > gpurun_out/s13/convs.log 2>&1 || exit $?
exit 0
