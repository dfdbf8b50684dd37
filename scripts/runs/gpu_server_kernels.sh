#!/bin/bash
# server hot-path kernel bandwidth table + rocprofv3 kernel stats of the same run
mkdir -p gpurun_out/srv
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python scripts/bench_server_kernels.py --iters 20 --json gpurun_out/srv/server_kernels.json > gpurun_out/srv/bench.log 2>&1 || { tail -20 gpurun_out/srv/bench.log; exit 1; }
cat gpurun_out/srv/bench.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/srv/prof -o run -- python $GRAFT_REPO_ROOT/scripts/bench_server_kernels.py --iters 5 --big 0 --json /tmp/x.json > $GRAFT_REPO_ROOT/gpurun_out/srv/prof.log 2>&1 || exit $?
exit 0
