#!/bin/bash
# 3x3 patch weight gradient (64/128 ch) + bn3 backward prologue cap: tests, wgrad probe vs MIOpen, bench A/B
mkdir -p gpurun_out/r3aa
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convgemm_gpu.py \
  tests/test_side_stream_gpu.py > gpurun_out/r3aa/pytest.log 2>&1 || { tail -40 gpurun_out/r3aa/pytest.log; exit 1; }
tail -2 gpurun_out/r3aa/pytest.log
timeout -k 10 300 python scripts/probe_wgrad.py --it 5 > gpurun_out/r3aa/wgrad_probe.jsonl 2>gpurun_out/r3aa/probe.err || exit $?
grep -E '"3x3 56x56 64|"3x3 28x28 128|step_total' gpurun_out/r3aa/wgrad_probe.jsonl | cut -c1-200
run() { env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 >> gpurun_out/r3aa/bench_ab.jsonl 2>>gpurun_out/r3aa/bench.err || exit $?;
        echo "$*: $(tail -1 gpurun_out/r3aa/bench_ab.jsonl | cut -c100-190)"; }
run PS_AMD_WGRAD_PATCH_MAX_C=128
run PS_AMD_WGRAD_PATCH_MAX_C=0
run PS_AMD_WGRAD_PATCH_MAX_C=128 PS_AMD_BN_BWD_PROLOGUE_MAX_C=0
run PS_AMD_WGRAD_PATCH_MAX_C=128
run PS_AMD_WGRAD_PATCH_MAX_C=0
run PS_AMD_WGRAD_PATCH_MAX_C=128 PS_AMD_BN_BWD_PROLOGUE_MAX_C=0
