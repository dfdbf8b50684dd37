#!/bin/bash
# 256 x 128 tiles (two blocks per CU) vs the default planner on ResNet-50's plain 1x1 GEMMs,
# plus the per-block phase stamps with the 128-channel tiles
set -o pipefail
O=gpurun_out/r5tn
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_big_gpu.py > $O/pytest.log 2>&1 && \
timeout -k 10 300 python scripts/probe_conv_big.py --tn > $O/tn_default.jsonl 2> $O/tn_default.err && \
PS_AMD_CONV_BIG_TN=128 timeout -k 10 300 python scripts/probe_conv_big.py --tn > $O/tn_128.jsonl 2> $O/tn_128.err && \
PS_AMD_CONV_BIG_TN=128 timeout -k 10 200 python scripts/probe_big_phases.py > $O/phases_128.txt 2>&1
