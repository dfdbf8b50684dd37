#!/bin/bash
# Session 8: whole GPU test suite + smoke + the other BASELINE configs on 1 GPU.
mkdir -p gpurun_out/s8
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/s8/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/s8/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/s8/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --config bert-ssp --steps 20 --warmup 5 > gpurun_out/s8/bench_bert.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --config dlrm --steps 20 --warmup 5 > gpurun_out/s8/bench_dlrm.log 2>&1 || exit $?
timeout -k 10 900 python bench.py --config llama-onebit --steps 5 --warmup 2 > gpurun_out/s8/bench_llama.log 2>&1 || exit $?
exit 0
