#!/bin/bash
mkdir -p gpurun_out/s28
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -m pytest tests/test_transformer_gpu.py tests/test_zoo_gpu.py -q > gpurun_out/s28/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/s28/pytest.log
if [ $rc -ne 0 ]; then exit 0; fi
timeout -k 10 600 python bench.py --config bert-ssp --steps 20 --warmup 5 > gpurun_out/s28/bench_bert.log 2>&1 || exit $?
timeout -k 10 900 python bench.py --config llama-onebit --steps 5 --warmup 2 > gpurun_out/s28/bench_llama.log 2>&1 || exit $?
exit 0
