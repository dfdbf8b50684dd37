#!/bin/bash
# patch-staged 3x3 forward / data gradient at >= 128 output channels only: tests (incl. forced 64-ch patch), bench A/B
mkdir -p gpurun_out/r3ai
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convgemm_gpu.py \
  > gpurun_out/r3ai/pytest.log 2>&1 || { tail -40 gpurun_out/r3ai/pytest.log; exit 1; }
PS_AMD_CONV_PATCH64=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convgemm_gpu.py \
  -k "patch_forward or conv3x3" >> gpurun_out/r3ai/pytest.log 2>&1 || { tail -40 gpurun_out/r3ai/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/r3ai/pytest.log
run() { env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 >> gpurun_out/r3ai/bench_ab.jsonl 2>>gpurun_out/r3ai/bench.err || exit $?;
        echo "$*: $(tail -1 gpurun_out/r3ai/bench_ab.jsonl | cut -c100-190)"; }
run PS_AMD_CONV_PATCH=1
run PS_AMD_CONV_PATCH=0
run PS_AMD_CONV_PATCH=1
run PS_AMD_CONV_PATCH=0
run PS_AMD_CONV_PATCH=1
run PS_AMD_CONV_PATCH=0
