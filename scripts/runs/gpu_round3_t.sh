#!/bin/bash
# wide wgrad LIN fast path: numerics, linear-wgrad + conv-wgrad probes, BERT / ResNet / DLRM benches
mkdir -p gpurun_out/r3t
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest tests/test_convgemm_gpu.py tests/test_splitk_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3t/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r3t/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe_linear_wgrad.py > gpurun_out/r3t/lin.jsonl 2>/dev/null || exit $?
cat gpurun_out/r3t/lin.jsonl
timeout -k 10 300 python scripts/probe_wgrad.py --miopen 0 > gpurun_out/r3t/wgrad.jsonl 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > gpurun_out/r3t/bert.json 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3t/resnet.json 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 > gpurun_out/r3t/dlrm.json 2>/dev/null || exit $?
cut -c1-150 gpurun_out/r3t/wgrad.jsonl; cut -c1-200 gpurun_out/r3t/bert.json gpurun_out/r3t/resnet.json gpurun_out/r3t/dlrm.json
