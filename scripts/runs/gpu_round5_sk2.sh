#!/bin/bash
# stream-K with coherent relaxed-atomic partials (no L2 write-back / invalidate): numerics, per-shape A/B, bench
set -o pipefail
O=gpurun_out/r5sk2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_big_gpu.py > $O/pytest.log 2>&1 && \
PS_AMD_CONV_BIG_SK=2 timeout -k 10 300 python scripts/probe_conv_big.py > $O/big_sk.jsonl 2> $O/big_sk.err && \
PS_AMD_CONV_BIG_SK=2 timeout -k 10 300 python scripts/probe_conv_big.py --pro > $O/pro_sk.jsonl 2> $O/pro_sk.err && \
PS_AMD_CONV_BIG_SK=2 PS_AMD_CONV_BIG_SK_SMALL=1 timeout -k 10 300 python scripts/probe_conv_big.py > $O/big_sksmall.jsonl 2> $O/big_sksmall.err && \
PS_AMD_CONV_BIG_SK=2 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_sk.json 2> $O/bench_sk.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_dp.json 2> $O/bench_dp.err
