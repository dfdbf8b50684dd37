#!/bin/bash
# one-launch BN finalize: numerics, per-call timing vs fold + finalize, model tests, bench A/B (bs1024, bs256)
set -o pipefail
O=gpurun_out/r5fin2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
PS_AMD_BN_FIN2=1 timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_fin2_gpu.py > $O/pytest.log 2>&1 && \
timeout -k 10 200 python scripts/probe_bn_fin.py > $O/fin_on.jsonl 2> $O/fin_on.err && \
PS_AMD_BN_FIN2=0 timeout -k 10 200 python scripts/probe_bn_fin.py > $O/fin_off.jsonl 2> $O/fin_off.err && \
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_convgemm_gpu.py tests/test_conv_bwd_fused_gpu.py tests/test_bn_gpu.py tests/test_conv_big_gpu.py > $O/pytest2.log 2>&1 && \
PS_AMD_BN_FIN2=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_off.json 2> $O/bench_off.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_on.json 2> $O/bench_on.err && \
PS_AMD_BN_FIN2=0 timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/bench256_off.json 2> $O/bench256_off.err && \
timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/bench256_on.json 2> $O/bench256_on.err
