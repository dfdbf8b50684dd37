#!/bin/bash
set -o pipefail
O=gpurun_out/r5stall
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python scripts/probe_stall.py --steps 40 > $O/a.txt 2> $O/a.err && \
timeout -k 10 300 python scripts/probe_stall.py --steps 40 > $O/b.txt 2> $O/b.err
