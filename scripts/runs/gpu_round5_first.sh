#!/bin/bash
# Round 5, first call: the changed GPU paths (row service status check, arena grow after pushes,
# stream policy by ranks per device) + the default bench line + W=2 one-GPU rehearsals whose JSON
# must show ranks_per_device = 2, side stream off at bs1024 and no placeholder phase zeros.
O=gpurun_out/r5first
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_row_plane_gpu.py \
  tests/test_side_stream_gpu.py tests/test_gpu_kvstore_gpu.py -m gpu > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench.json 2> $O/bench.err || exit $?
tail -c 1500 $O/bench.json
export PS_AMD_BENCH_ONE_GPU=1
timeout -k 10 400 python bench.py --gpus 2 --steps 6 --warmup 3 --comm-probe 0 --timing 3 > $O/resnet_w2_bs1024.json 2> $O/resnet_w2_bs1024.err || exit $?
tail -c 2500 $O/resnet_w2_bs1024.json
timeout -k 10 300 python bench.py --config dlrm --gpus 2 --steps 10 --warmup 3 --comm-probe 0 --dlrm-rows 1000000 > $O/dlrm_w2.json 2> $O/dlrm_w2.err || exit $?
tail -c 2000 $O/dlrm_w2.json
