#!/bin/bash
# Fresh kernel trace of the default ResNet-50 bench (current tree) + per-kernel stats.
mkdir -p gpurun_out/p3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/p3/prof -o run -- python3 bench.py --steps 10 --warmup 5 > gpurun_out/p3/bench.log 2>&1 || exit $?
exit 0
