#!/bin/bash
# flash attention at the bench batch (B=4) + per-kernel profile of the Llama step, flash vs SDPA
mkdir -p gpurun_out/r3f
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 200 python scripts/probe_flash.py 4 > gpurun_out/r3f/flash_b4.jsonl 2>&1 || exit $?
cat gpurun_out/r3f/flash_b4.jsonl
cd /tmp
for f in 1 0; do
  PS_AMD_FLASH_ATTN=$f timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3f/prof$f -o run \
    -- python $GRAFT_REPO_ROOT/bench.py --config llama-onebit --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r3f/bench$f.json 2>$GRAFT_REPO_ROOT/gpurun_out/r3f/bench$f.err || exit $?
  python $GRAFT_REPO_ROOT/scripts/kernel_stats_top.py $(find $GRAFT_REPO_ROOT/gpurun_out/r3f/prof$f -name '*kernel_stats.csv' | head -1) 25 > $GRAFT_REPO_ROOT/gpurun_out/r3f/top$f.txt || exit $?
  find $GRAFT_REPO_ROOT/gpurun_out/r3f/prof$f -name '*kernel_trace.csv' -delete
done
cat $GRAFT_REPO_ROOT/gpurun_out/r3f/top1.txt $GRAFT_REPO_ROOT/gpurun_out/r3f/top0.txt
