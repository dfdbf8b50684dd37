#!/bin/bash
mkdir -p gpurun_out/s27
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -m pytest tests/test_zoo_gpu.py -q > gpurun_out/s27/pytest.log 2>&1
echo "rc=$?" >> gpurun_out/s27/pytest.log
timeout -k 10 900 python bench.py --config llama-onebit --steps 5 --warmup 2 --timing 2 > gpurun_out/s27/bench_llama.log 2>&1 || exit $?
exit 0
