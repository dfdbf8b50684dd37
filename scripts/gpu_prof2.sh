#!/bin/bash
# GPU session 3: MIOpen find modes / warm-up cost, HIP-graph capture gain.
mkdir -p gpurun_out/s3
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
run() { # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/s3/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc" >> gpurun_out/s3/rc.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
export MIOPEN_USER_DB_PATH=/tmp/mio1/udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/mio1/cache
run immediate_cold python bench.py --steps 20 --warmup 5 --cudnn-benchmark 0 --graph 0
run immediate_graph python bench.py --steps 20 --warmup 5 --cudnn-benchmark 0 --graph 1
export MIOPEN_USER_DB_PATH=/tmp/mio2/udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/mio2/cache
run find_nonaive_cold MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0 MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_BWD=0 MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_WRW=0 python bench.py --steps 20 --warmup 5 --graph 0
run find_nonaive_warm_graph MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0 MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_BWD=0 MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_WRW=0 python bench.py --steps 20 --warmup 5 --graph 1
du -sh /tmp/mio1 /tmp/mio2 > gpurun_out/s3/sizes.txt
cp -r /tmp/mio2 gpurun_out/s3/mio_find_db
exit 0
