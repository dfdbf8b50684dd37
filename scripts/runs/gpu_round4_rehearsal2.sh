#!/bin/bash
# Multi-rank rehearsals on ONE MI355X (PS_AMD_BENCH_ONE_GPU=1: every rank on cuda:0, gloo control
# plane, IPC data planes): ResNet-50 on the xGMI plane at W = 2 / 4 / 8 (host-flag and IPC-event
# round ends at W = 2), the asynchronous CTR config and DLRM on the row plane at W = 2.
# Final tree (side stream on at the small batches, off at bs1024 as in the driver run).
# Shared-GPU throughput -- not scaling numbers; the point is the N > 1 driver path end to end
# with the plane's per-phase statistics in the JSON.
O=gpurun_out/r4reh2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH PS_AMD_BENCH_ONE_GPU=1
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs python bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?
  tail -c 600 $O/$name.json
  [ $rc -ge 124 ] && { echo "stopping after $name (rc=$rc)"; exit $rc; }
  return 0
}
run resnet_w2 300 --gpus 2 --steps 10 --warmup 3 --comm-probe 0 --batch-per-gpu 256 --timing 3 || exit $?
run resnet_w2_bs1024 400 --gpus 2 --steps 6 --warmup 3 --comm-probe 0 --timing 3 || exit $?
export PS_AMD_PLANE_IPC_EVENTS=1
run resnet_w2_ipcev 300 --gpus 2 --steps 10 --warmup 3 --comm-probe 0 --batch-per-gpu 256 --timing 3 || exit $?
unset PS_AMD_PLANE_IPC_EVENTS
run resnet_w4 300 --gpus 4 --steps 10 --warmup 3 --comm-probe 0 --batch-per-gpu 128 --timing 3 || exit $?
run resnet_w8 400 --gpus 8 --steps 10 --warmup 3 --comm-probe 0 --batch-per-gpu 64 --timing 3 || exit $?
run ctr_w2 300 --config ctr-async --gpus 2 --steps 20 --warmup 5 --comm-probe 0 || exit $?
run dlrm_w2 300 --config dlrm --gpus 2 --steps 10 --warmup 3 --comm-probe 0 --dlrm-rows 200000 || exit $?
