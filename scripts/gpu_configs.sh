#!/bin/bash
# All non-headline BASELINE configs on 1 GPU after the gradient-landing change.
mkdir -p gpurun_out/cfg
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 --json-out gpurun_out/cfg/bert.json > gpurun_out/cfg/bert.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 --json-out gpurun_out/cfg/dlrm.json > gpurun_out/cfg/dlrm.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config llama-onebit --steps 5 --warmup 2 --json-out gpurun_out/cfg/llama.json > gpurun_out/cfg/llama.log 2>&1 || exit $?
exit 0
