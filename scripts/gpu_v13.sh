#!/bin/bash
# conv GEMM numerics + micro-benchmark + fused-block bench
mkdir -p gpurun_out/v13
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest tests/test_convgemm_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/v13/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/v13/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_convgemm.py > gpurun_out/v13/probe.jsonl 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/v13/bench_fused.log 2>&1 || exit $?
exit 0
