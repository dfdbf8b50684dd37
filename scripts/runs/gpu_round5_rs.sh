#!/bin/bash
# register-staged K loop (PS_AMD_CONV_BIG_RS=1: global_load -> VGPR -> ds_write) vs LDS-DMA staging
set -o pipefail
O=gpurun_out/r5rs
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
PS_AMD_CONV_BIG_RS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_big_gpu.py > $O/pytest.log 2>&1 && \
PS_AMD_CONV_BIG_RS=1 timeout -k 10 300 python scripts/probe_conv_big.py > $O/big_rs.jsonl 2> $O/big_rs.err && \
timeout -k 10 300 python scripts/probe_conv_big.py > $O/big_dma.jsonl 2> $O/big_dma.err && \
PS_AMD_CONV_BIG_RS=1 timeout -k 10 300 python scripts/probe_conv_big.py --tn > $O/tn_rs.jsonl 2> $O/tn_rs.err && \
timeout -k 10 300 python scripts/probe_conv_big.py --tn > $O/tn_dma.jsonl 2> $O/tn_dma.err && \
PS_AMD_CONV_BIG_RS=1 timeout -k 10 200 python scripts/probe_big_phases.py > $O/phases_rs.txt 2>&1
