#!/bin/bash
# xGMI plane on one GPU: 1-GPU headline bench, then the multi-rank bench path rehearsed with
# W processes on cuda:0 (gloo control plane, IPC data plane), per-phase timing on stderr.
mkdir -p gpurun_out/plane
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/plane/n1.json 2> gpurun_out/plane/n1.err &&
PS_AMD_BENCH_ONE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 --comm-probe 0 \
  --batch-per-gpu 256 --timing 3 > gpurun_out/plane/n2_rehearsal.json 2> gpurun_out/plane/n2_rehearsal.err &&
PS_AMD_BENCH_ONE_GPU=1 timeout -k 10 400 python bench.py --gpus 4 --steps 10 --warmup 3 --comm-probe 0 \
  --batch-per-gpu 128 --timing 3 > gpurun_out/plane/n4_rehearsal.json 2> gpurun_out/plane/n4_rehearsal.err
rc=$?
cat gpurun_out/plane/*.json
grep -h "bench" gpurun_out/plane/*.err | tail -12
exit $rc
