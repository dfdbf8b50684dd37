#!/bin/bash
# DLRM on the IPC row plane: W=1 line, then W=2 (two processes on cuda:0) with the row-plane stage
# table (PS_AMD_ROWPLANE_TIMING=1) and the dense plane's phases (--timing 3).
O=gpurun_out/r5dlrm
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 > $O/dlrm_w1.json 2> $O/dlrm_w1.err || exit $?
tail -c 600 $O/dlrm_w1.json
export PS_AMD_BENCH_ONE_GPU=1 PS_AMD_ROWPLANE_TIMING=1
timeout -k 10 300 python bench.py --config dlrm --gpus 2 --steps 10 --warmup 3 --comm-probe 0 --timing 3 > $O/dlrm_w2_timing.json 2> $O/dlrm_w2_timing.err || exit $?
tail -c 3000 $O/dlrm_w2_timing.json
