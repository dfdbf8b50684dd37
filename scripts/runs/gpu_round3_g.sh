#!/bin/bash
# flash v3: numerics, B=1/B=4 probe vs SDPA, Llama A/B
mkdir -p gpurun_out/r3g
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_flash_gpu.py tests/test_attention_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r3g/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r3g/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe_flash.py 1 > gpurun_out/r3g/flash.jsonl 2>&1 || exit $?
timeout -k 10 200 python scripts/probe_flash.py 4 >> gpurun_out/r3g/flash.jsonl 2>&1 || exit $?
cat gpurun_out/r3g/flash.jsonl
PS_AMD_FLASH_ATTN=1 timeout -k 10 400 python bench.py --config llama-onebit --steps 10 --warmup 3 > gpurun_out/r3g/llama_flash.json 2>gpurun_out/r3g/llama_flash.err || exit $?

cut -c1-300 gpurun_out/r3g/llama_flash.json
