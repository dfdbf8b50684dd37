#!/bin/bash
# bs256 knob sweep on the final tree (one box, back to back): which round-5 defaults hold at bs256
set -o pipefail
O=gpurun_out/r5knobs256
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/$tag.json 2> $O/$tag.err || exit 1; }
run base PS_AMD_NONE=1
run big0 PS_AMD_CONV_BIG=0
run fold0 PS_AMD_CONV_BIG_FOLD=0
run stem0 PS_AMD_STEM_BWD_FUSED=0
run ds0 PS_AMD_DS_BWD_FUSED=0
run c3f0 PS_AMD_CONV3_BWD_FUSED=0
run inflight3 PS_AMD_MAX_INFLIGHT=3
run wstream0 PS_AMD_WGRAD_STREAM=0
run base2 PS_AMD_NONE=1
