#!/bin/bash
# GPU session 2: bench cold/warm MIOpen cache + rocprofv3 kernel stats of the PS step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
export MIOPEN_USER_DB_PATH=/tmp/miopen/udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen/cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_cold.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_warm.log 2>&1 || exit $?
du -sh /tmp/miopen/* > gpurun_out/miopen_size.txt; ls -laR /tmp/miopen >> gpurun_out/miopen_size.txt
sz=$(du -sm /tmp/miopen | cut -f1); if [ "$sz" -lt 48 ]; then cp -r /tmp/miopen gpurun_out/miopen_db; fi
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 3 > $R/gpurun_out/prof.log 2>&1 || exit $?
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch-per-gpu 256 --bucket-mb 100 > gpurun_out/bench_bucket100.log 2>&1
exit 0
