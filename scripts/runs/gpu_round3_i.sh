#!/bin/bash
# attention kernels after the permlane change: numerics + BERT / Llama benches (flash default)
mkdir -p gpurun_out/r3i
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_flash_gpu.py tests/test_attention_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r3i/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3i/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config bert-ssp --steps 20 --warmup 5 > gpurun_out/r3i/bert.json 2>gpurun_out/r3i/bert.err || exit $?
timeout -k 10 400 python bench.py --config llama-onebit --steps 10 --warmup 3 > gpurun_out/r3i/llama.json 2>gpurun_out/r3i/llama.err || exit $?
cut -c1-250 gpurun_out/r3i/bert.json gpurun_out/r3i/llama.json
