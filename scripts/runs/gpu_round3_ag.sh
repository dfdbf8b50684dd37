#!/bin/bash
# one-launch backward weight layouts (weight_prep): tests + bench A/B
mkdir -p gpurun_out/r3ag
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convgemm_gpu.py tests/test_side_stream_gpu.py \
  tests/test_bn_gpu.py tests/test_ps_gpu.py > gpurun_out/r3ag/pytest.log 2>&1 || { tail -40 gpurun_out/r3ag/pytest.log; exit 1; }
tail -2 gpurun_out/r3ag/pytest.log
run() { env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 >> gpurun_out/r3ag/bench_ab.jsonl 2>>gpurun_out/r3ag/bench.err || exit $?;
        echo "$*: $(tail -1 gpurun_out/r3ag/bench_ab.jsonl | cut -c100-190)"; }
run PS_AMD_WEIGHT_PREP=1
run PS_AMD_WEIGHT_PREP=0
run PS_AMD_WEIGHT_PREP=1
run PS_AMD_WEIGHT_PREP=0
