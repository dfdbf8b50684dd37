#!/bin/bash
# fused LM-head cross-entropy: numerics, BERT / Llama benches
mkdir -p gpurun_out/r3v
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_zoo_gpu.py tests/test_flash_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3v/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3v/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > gpurun_out/r3v/bert.json 2>/dev/null || exit $?
timeout -k 10 400 python bench.py --config llama-onebit --steps 10 --warmup 3 > gpurun_out/r3v/llama.json 2>gpurun_out/r3v/llama.err || exit $?
cut -c1-200 gpurun_out/r3v/bert.json gpurun_out/r3v/llama.json
