#!/bin/bash
# reproduce: bench bs1024 with the driver's --warmup 5 (r5cfg run showed 225 ms/step), twice, then warmup 8
set -o pipefail
O=gpurun_out/r5w5
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/w5a.json 2> $O/w5a.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/w5b.json 2> $O/w5b.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/w8.json 2> $O/w8.err && \
timeout -k 10 300 python scripts/probe_step_gap.py --steps 20 > $O/gap256.json 2> $O/gap256.err && \
timeout -k 10 300 python scripts/probe_step_gap.py --batch-per-gpu 1024 --steps 12 > $O/gap1024.json 2> $O/gap1024.err
