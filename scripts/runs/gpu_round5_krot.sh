#!/bin/bash
# K-order rotation per tile (PS_AMD_CONV_BIG_KROT=1), with and without stream-K: numerics + per-shape + bench
set -o pipefail
O=gpurun_out/r5krot
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
PS_AMD_CONV_BIG_KROT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_big_gpu.py > $O/pytest.log 2>&1 && \
PS_AMD_CONV_BIG_KROT=1 timeout -k 10 300 python scripts/probe_conv_big.py > $O/big_krot.jsonl 2> $O/big_krot.err && \
PS_AMD_CONV_BIG_KROT=1 PS_AMD_CONV_BIG_SK=2 timeout -k 10 300 python scripts/probe_conv_big.py > $O/big_krot_sk.jsonl 2> $O/big_krot_sk.err && \
PS_AMD_CONV_BIG_KROT=1 timeout -k 10 300 python scripts/probe_conv_big.py --pro > $O/pro_krot.jsonl 2> $O/pro_krot.err && \
timeout -k 10 300 python scripts/probe_conv_big.py > $O/big_base.jsonl 2> $O/big_base.err && \
PS_AMD_CONV_BIG_KROT=1 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_krot.json 2> $O/bench_krot.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_base.json 2> $O/bench_base.err
