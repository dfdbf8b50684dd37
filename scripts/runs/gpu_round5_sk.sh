#!/bin/bash
# stream-K for the 256 x 256 tiles: numerics (SK on by default where the last round is < 90 % full),
# per-shape A/B (PS_AMD_CONV_BIG_SK=0), then the bench A/B
set -o pipefail
O=gpurun_out/r5sk
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_big_gpu.py > $O/pytest.log 2>&1 && \
export PS_AMD_CONV_BIG_SK=2 && \
timeout -k 10 300 python scripts/probe_conv_big.py > $O/big_sk.jsonl 2> $O/big_sk.err && \
env PS_AMD_CONV_BIG_SK=0 timeout -k 10 300 python scripts/probe_conv_big.py > $O/big_dp.jsonl 2> $O/big_dp.err && \
timeout -k 10 300 python scripts/probe_conv_big.py --pro > $O/pro_sk.jsonl 2> $O/pro_sk.err && \
env PS_AMD_CONV_BIG_SK=0 timeout -k 10 300 python scripts/probe_conv_big.py --pro > $O/pro_dp.jsonl 2> $O/pro_dp.err && \
timeout -k 10 300 python scripts/probe_conv_big.py --tn > $O/tn_sk.jsonl 2> $O/tn_sk.err && \
env PS_AMD_CONV_BIG_SK=0 timeout -k 10 300 python scripts/probe_conv_big.py --tn > $O/tn_dp.jsonl 2> $O/tn_dp.err && \
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_convgemm_gpu.py tests/test_conv_bwd_fused_gpu.py tests/test_bn_gpu.py > $O/pytest2.log 2>&1 && \
env PS_AMD_CONV_BIG_SK=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_dp.json 2> $O/bench_dp.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_sk.json 2> $O/bench_sk.err && \
timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/bench256_sk.json 2> $O/bench256_sk.err && \
env PS_AMD_CONV_BIG_SK=0 timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/bench256_dp.json 2> $O/bench256_dp.err && \
# batch 256: deep-K GEMMs on fewer than 256 tiles through stream-K (PS_AMD_CONV_BIG_SK_SMALL=1)
PS_AMD_CONV_BIG_SK_SMALL=1 timeout -k 10 300 python scripts/probe_conv_big.py > $O/big_sksmall.jsonl 2> $O/big_sksmall.err && \
PS_AMD_CONV_BIG_SK_SMALL=1 timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/bench256_sksmall.json 2> $O/bench256_sksmall.err
