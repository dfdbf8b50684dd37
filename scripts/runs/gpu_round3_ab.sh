#!/bin/bash
# bench A/B: 3x3 patch weight gradient (64/128 ch) and the bn3 backward prologue cap
mkdir -p gpurun_out/r3ab
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
run() { env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 >> gpurun_out/r3ab/bench_ab.jsonl 2>>gpurun_out/r3ab/bench.err || exit $?;
        echo "$*: $(tail -1 gpurun_out/r3ab/bench_ab.jsonl | cut -c100-190)"; }
run PS_AMD_WGRAD_PATCH_MAX_C=128
run PS_AMD_WGRAD_PATCH_MAX_C=0
run PS_AMD_WGRAD_PATCH_MAX_C=128 PS_AMD_BN_BWD_PROLOGUE_MAX_C=0
run PS_AMD_WGRAD_PATCH_MAX_C=128
run PS_AMD_WGRAD_PATCH_MAX_C=0
run PS_AMD_WGRAD_PATCH_MAX_C=128 PS_AMD_BN_BWD_PROLOGUE_MAX_C=0
