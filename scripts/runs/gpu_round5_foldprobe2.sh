#!/bin/bash
# conv1 data-gradient GEMMs on the 256 x 256 tiles, 16 epilogue rows in flight per thread
set -o pipefail
O=gpurun_out/r5foldprobe2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 200 python scripts/probe_conv_big.py --fold > $O/fold_on.jsonl 2> $O/fold_on.err
