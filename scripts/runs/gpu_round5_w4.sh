#!/bin/bash
# 256 x 256 tiles as 4 waves of 128 x 128 (PS_AMD_CONV_BIG_W4=1) vs 8 waves of 128 x 64: numerics,
# per-shape timing, phase stamps
set -o pipefail
O=gpurun_out/r5w4
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
PS_AMD_CONV_BIG_W4=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_big_gpu.py > $O/pytest.log 2>&1 && \
PS_AMD_CONV_BIG_W4=1 timeout -k 10 300 python scripts/probe_conv_big.py --tn > $O/tn_w4.jsonl 2> $O/tn_w4.err && \
timeout -k 10 300 python scripts/probe_conv_big.py --tn > $O/tn_w8.jsonl 2> $O/tn_w8.err && \
PS_AMD_CONV_BIG_W4=1 timeout -k 10 300 python scripts/probe_conv_big.py --pro > $O/pro_w4.jsonl 2> $O/pro_w4.err && \
timeout -k 10 300 python scripts/probe_conv_big.py --pro > $O/pro_w8.jsonl 2> $O/pro_w8.err && \
PS_AMD_CONV_BIG_W4=1 timeout -k 10 200 python scripts/probe_big_phases.py > $O/phases_w4.txt 2>&1
