#!/bin/bash
# Non-headline BASELINE configs on 1 GPU (+ DLRM overlap A/B).  Logs/JSON under gpurun_out/cfg/
mkdir -p gpurun_out/cfg
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 --json-out gpurun_out/cfg/dlrm.json > gpurun_out/cfg/dlrm.log 2>&1 || exit $?
PS_AMD_SPARSE_OVERLAP=0 timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 --json-out gpurun_out/cfg/dlrm_nooverlap.json > gpurun_out/cfg/dlrm_nooverlap.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 --json-out gpurun_out/cfg/bert.json > gpurun_out/cfg/bert.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config llama-onebit --steps 5 --warmup 2 --json-out gpurun_out/cfg/llama.json > gpurun_out/cfg/llama.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/cfg/resnet.json > gpurun_out/cfg/resnet.log 2>&1 || exit $?
exit 0
