#!/bin/bash
# layer-3 conv1 data gradient: time vs epilogue bytes, 256 x 256 vs 128 x 128 tiles, vs copy / add
set -o pipefail
O=gpurun_out/r5foldscan
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 200 python scripts/probe_conv_big.py --fold-scan > $O/on.jsonl 2> $O/on.err && \
PS_AMD_CONV_BIG_FOLD=0 PS_AMD_CONV_BIG=0 timeout -k 10 200 python scripts/probe_conv_big.py --fold-scan > $O/off.jsonl 2> $O/off.err
