#!/bin/bash
# flash attention with XCD-aware block order: numerics, probe B=1/B=4, Llama bench
mkdir -p gpurun_out/r3q
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_flash_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3q/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r3q/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe_flash.py 1 > gpurun_out/r3q/flash.jsonl 2>&1 || exit $?
timeout -k 10 200 python scripts/probe_flash.py 4 >> gpurun_out/r3q/flash.jsonl 2>&1 || exit $?
grep shape gpurun_out/r3q/flash.jsonl
timeout -k 10 400 python bench.py --config llama-onebit --steps 10 --warmup 3 > gpurun_out/r3q/llama.json 2>gpurun_out/r3q/llama.err || exit $?
cut -c1-200 gpurun_out/r3q/llama.json
