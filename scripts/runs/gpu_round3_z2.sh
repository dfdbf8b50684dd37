#!/bin/bash
# bn3 backward prologue: channel cap A/B (0 = off, 256 = layer 1, 512 + persistent 8-stage PRO grid)
mkdir -p gpurun_out/r3z2
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
run() { env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 >> gpurun_out/r3z2/bench_ab.jsonl 2>>gpurun_out/r3z2/bench.err || exit $?;
        echo "$*: $(tail -1 gpurun_out/r3z2/bench_ab.jsonl | cut -c100-190)"; }
run PS_AMD_BN_BWD_PROLOGUE_MAX_C=256
run PS_AMD_BN_BWD_PROLOGUE_MAX_C=0
run PS_AMD_BN_BWD_PROLOGUE_MAX_C=512 PS_AMD_PERSIST_NK_PRO=8
run PS_AMD_BN_BWD_PROLOGUE_MAX_C=256
run PS_AMD_BN_BWD_PROLOGUE_MAX_C=0
