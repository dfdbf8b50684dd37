#!/bin/bash
# 256x256-tile conv GEMM: numerics, per-shape timing vs the 128x128 kernel (BK 64 / 32), bench A/B
set -o pipefail
O=gpurun_out/r5big
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_big_gpu.py > $O/pytest.log 2>&1 && \
PS_AMD_CONV_BIG=0 timeout -k 10 200 python scripts/probe_conv_big.py > $O/probe.jsonl 2> $O/probe.err && \
PS_AMD_CONV_BIG=1 timeout -k 10 200 python scripts/probe_conv_big.py >> $O/probe.jsonl 2>> $O/probe.err && \
PS_AMD_CONV_BIG=1 PS_AMD_CONV_BIG_BK=32 timeout -k 10 200 python scripts/probe_conv_big.py | sed 's/"big": "1"/"big": "1-bk32"/' >> $O/probe.jsonl 2>> $O/probe.err && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_convgemm_gpu.py -k "fused_bottleneck or chained or layer1_chain or deep_k" > $O/pytest2.log 2>&1 && \
PS_AMD_CONV_BIG=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_off.json 2> $O/bench_off.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_on.json 2> $O/bench_on.err && \
timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/bench256_on.json 2> $O/bench256_on.err
