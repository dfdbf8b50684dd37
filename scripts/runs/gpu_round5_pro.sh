#!/bin/bash
set -o pipefail
O=gpurun_out/r5pro
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 200 python scripts/probe_conv_big.py --pro > $O/probe.jsonl 2> $O/probe.err && \
PS_AMD_CONV_BIG_PRO=0 timeout -k 10 200 python scripts/probe_conv_big.py --pro >> $O/probe.jsonl 2>> $O/probe.err
