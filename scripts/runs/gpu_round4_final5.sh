#!/bin/bash
# Final tree with the weight gradients on the side stream at every batch size: default bench (the
# driver's N=1 line), smoke, the side-stream GPU tests, and the N > 1 driver path rehearsed on one
# GPU with the side stream on: ResNet-50 W = 2 and W = 4 at bs1024 per rank, W = 8 at bs256.
O=gpurun_out/r4final5
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
step() {  # name seconds command...  (any failure ends the call)
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  tail -c 400 $O/$name.log; echo
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_side_stream_gpu.py tests/test_plane_gpu.py
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_a 200 python bench.py
step bench_b 200 python bench.py --steps 20 --warmup 8
step bench256 200 python bench.py --batch-per-gpu 256 --steps 20 --warmup 8
export PS_AMD_BENCH_ONE_GPU=1
step reh_w2_bs1024 400 python bench.py --gpus 2 --steps 6 --warmup 3 --comm-probe 0 --timing 3
step reh_w4_bs1024 600 python bench.py --gpus 4 --steps 4 --warmup 2 --comm-probe 0 --timing 2
step reh_w8_bs256 400 python bench.py --gpus 8 --steps 6 --warmup 3 --comm-probe 0 --batch-per-gpu 256 --timing 3
