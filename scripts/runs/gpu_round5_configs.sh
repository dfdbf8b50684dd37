#!/bin/bash
# the other BASELINE configs on the round-5 tree, 1 GPU -> gpurun_out/r5cfg/*.json
set -o pipefail
O=gpurun_out/r5cfg
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > $O/bert.json 2> $O/bert.err && \
timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 > $O/dlrm.json 2> $O/dlrm.err && \
timeout -k 10 300 python bench.py --config ctr-async --steps 20 --warmup 5 > $O/ctr.json 2> $O/ctr.err && \
timeout -k 10 500 python bench.py --config llama-onebit --steps 6 --warmup 3 > $O/llama.json 2> $O/llama.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/resnet.json 2> $O/resnet.err && \
timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/resnet256.json 2> $O/resnet256.err
