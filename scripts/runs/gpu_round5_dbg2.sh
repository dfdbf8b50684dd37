#!/bin/bash
# c64r timing probes (no MFMA / no DMA / no stores) + HW-queue count A/B at bs256 / bs1024
set -o pipefail
O=gpurun_out/r5dbg2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for d in 0 1 2 3; do PS_AMD_CONV_C64=3 PS_AMD_C64R_DBG=$d timeout -k 10 200 python scripts/probe_conv3x3_c64.py | sed "s/\"mode\": \"3\"/\"mode\": \"3-dbg$d\"/" >> $O/probe.jsonl 2>> $O/probe.err || exit $?; done
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/b256_q8.json 2> $O/b256_q8.err && \
timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/b256_q4.json 2> $O/b256_q4.err && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/b1024_q8.json 2> $O/b1024_q8.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/b1024_q4.json 2> $O/b1024_q4.err
