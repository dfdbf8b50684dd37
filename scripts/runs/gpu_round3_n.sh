#!/bin/bash
# fc split-K + fused stem pool/BN backward: numerics, fc probe, ResNet bench A/B
mkdir -p gpurun_out/r3n
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest tests/test_fc_gpu.py tests/test_zoo_gpu.py tests/test_pool_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r3n/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3n/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_fc.py > gpurun_out/r3n/fc_probe.jsonl 2>gpurun_out/r3n/fc_probe.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3n/bench_fused.json 2>/dev/null || exit $?
PS_AMD_STEM_POOL_FUSED=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3n/bench_unfused.json 2>/dev/null || exit $?
cut -c1-250 gpurun_out/r3n/fc_probe.jsonl; cut -c1-200 gpurun_out/r3n/bench_fused.json gpurun_out/r3n/bench_unfused.json
