#!/bin/bash
# rocprofv3 kernel stats of the non-headline configs: DLRM (sparse path), BERT-SSP (async PS), and the
# server-kernel microbench (vectorised sparse / 1-bit kernels); CSV summaries under gpurun_out/pc/
mkdir -p gpurun_out/pc
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pc/dlrm -o run --output-format csv -- python $R/bench.py --config dlrm --steps 10 --warmup 5 > $R/gpurun_out/pc/dlrm.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pc/bert -o run --output-format csv -- python $R/bench.py --config bert-ssp --steps 10 --warmup 5 > $R/gpurun_out/pc/bert.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pc/srv -o run --output-format csv -- python $R/scripts/bench_server_kernels.py --iters 5 --big 0 --json /tmp/x.json > $R/gpurun_out/pc/srv.log 2>&1 || exit $?
ls -R $R/gpurun_out/pc | head -30
