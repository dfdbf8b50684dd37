#!/bin/bash
# fast pixel decode in the conv staging loops: numerics, conv probes, ResNet bench
mkdir -p gpurun_out/r3u
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest tests/test_convgemm_gpu.py tests/test_splitk_gpu.py tests/test_fc_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3u/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r3u/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_wgrad.py --miopen 0 > gpurun_out/r3u/wgrad.jsonl 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3u/resnet.json 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3u/resnet2.json 2>/dev/null || exit $?
grep -E "3x3|step_total" gpurun_out/r3u/wgrad.jsonl | cut -c1-150; cut -c1-200 gpurun_out/r3u/resnet.json gpurun_out/r3u/resnet2.json
