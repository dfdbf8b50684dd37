#!/bin/bash
# conv1 data-gradient GEMMs: 256 x 256 fold epilogues (+ bn1 backward prologue) vs the 128-pixel tiles
set -o pipefail
O=gpurun_out/r5foldprobe
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 200 python scripts/probe_conv_big.py --fold > $O/fold_on.jsonl 2> $O/fold_on.err && \
PS_AMD_CONV_BIG_FOLD=0 timeout -k 10 200 python scripts/probe_conv_big.py --fold > $O/fold_off.jsonl 2> $O/fold_off.err
