#!/bin/bash
# record the MIOpen find-db for batch 512 (merged with the existing 256 entries)
mkdir -p gpurun_out/s7 /tmp/mdb/udb /tmp/mdb/cache
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
cp miopen_db/udb/* /tmp/mdb/udb/ 2>/dev/null; cp miopen_db/cache/* /tmp/mdb/cache/ 2>/dev/null
export MIOPEN_USER_DB_PATH=/tmp/mdb/udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/mdb/cache
timeout -k 10 900 python bench.py --steps 20 --warmup 5 --batch-per-gpu 512 > gpurun_out/s7/bench_b512_cold.log 2>&1 || exit $?
cp -r /tmp/mdb gpurun_out/s7/mdb
timeout -k 10 600 python bench.py --steps 30 --warmup 5 --batch-per-gpu 512 > gpurun_out/s7/bench_b512_warm.log 2>&1 || exit $?
exit 0
