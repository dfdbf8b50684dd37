#!/bin/bash
# flash attention v2: numerics, kernel probe vs SDPA, Llama bench A/B
mkdir -p gpurun_out/r3e
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_flash_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r3e/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r3e/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe_flash.py > gpurun_out/r3e/flash.jsonl 2>&1 || exit $?
cat gpurun_out/r3e/flash.jsonl
PS_AMD_FLASH_ATTN=1 timeout -k 10 400 python bench.py --config llama-onebit --steps 10 --warmup 3 > gpurun_out/r3e/llama_flash.json 2>gpurun_out/r3e/llama_flash.err || exit $?
PS_AMD_FLASH_ATTN=0 timeout -k 10 400 python bench.py --config llama-onebit --steps 10 --warmup 3 > gpurun_out/r3e/llama_sdpa.json 2>gpurun_out/r3e/llama_sdpa.err || exit $?
cat gpurun_out/r3e/llama_flash.json gpurun_out/r3e/llama_sdpa.json | cut -c1-400
