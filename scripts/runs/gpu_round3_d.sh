#!/bin/bash
# wgrad big-tile kernel: numerics, per-shape probe, end-to-end bench A/B
mkdir -p gpurun_out/r3d
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_convgemm_gpu.py tests/test_splitk_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r3d/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r3d/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_wgrad.py --miopen 0 > gpurun_out/r3d/wgrad_big.jsonl 2>/dev/null || exit $?
PS_AMD_WGRAD_BIG=0 timeout -k 10 300 python scripts/probe_wgrad.py --miopen 0 > gpurun_out/r3d/wgrad_wide.jsonl 2>/dev/null || exit $?
paste -d' ' <(cut -c1-120 gpurun_out/r3d/wgrad_wide.jsonl) <(cut -c1-200 gpurun_out/r3d/wgrad_big.jsonl | sed 's/.*"us"/"us_big"/')
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3d/bench_big.json 2>/dev/null || exit $?
PS_AMD_WGRAD_BIG=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3d/bench_wide.json 2>/dev/null || exit $?
cat gpurun_out/r3d/bench_big.json gpurun_out/r3d/bench_wide.json | cut -c1-200
