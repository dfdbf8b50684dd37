#!/bin/bash
# whole-A-tile prefetch in memory order before the K loop (PS_AMD_CONV_BIG_L2PF=2) vs off
set -o pipefail
O=gpurun_out/r5l2pf2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
PS_AMD_CONV_BIG_L2PF=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_big_gpu.py > $O/pytest.log 2>&1 && \
PS_AMD_CONV_BIG_L2PF=2 timeout -k 10 300 python scripts/probe_conv_big.py > $O/big_pf.jsonl 2> $O/big_pf.err && \
timeout -k 10 300 python scripts/probe_conv_big.py > $O/big_nopf.jsonl 2> $O/big_nopf.err && \
PS_AMD_CONV_BIG_L2PF=2 timeout -k 10 200 python scripts/probe_big_phases.py > $O/phases_pf.txt 2>&1
