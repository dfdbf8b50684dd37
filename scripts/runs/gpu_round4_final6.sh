#!/bin/bash
# Final tree (side stream: any batch for one process, <= 512 with peers): side-stream + aux GPU
# tests, smoke, default bench twice, batch 256, and the N > 1 driver path at bs1024 (W = 2 on one GPU).
O=gpurun_out/r4final6
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
step() {  # name seconds command...  (any failure ends the call)
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  tail -c 300 $O/$name.log; echo
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_side_stream_gpu.py tests/test_convgemm_gpu.py -k "side_stream or chained or fused_bottleneck"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_a 200 python bench.py
step bench_b 200 python bench.py --steps 20 --warmup 8
step bench256 200 python bench.py --batch-per-gpu 256 --steps 20 --warmup 8
step reh_w2_bs1024 400 env PS_AMD_BENCH_ONE_GPU=1 python bench.py --gpus 2 --steps 6 --warmup 3 --comm-probe 0 --timing 3
