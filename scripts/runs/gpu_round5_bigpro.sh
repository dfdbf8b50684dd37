#!/bin/bash
# big-tile prologues (BN+ReLU / BN backward / block output): numerics, model-path tests, bench A/B
set -o pipefail
O=gpurun_out/r5bigpro
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_big_gpu.py > $O/pytest.log 2>&1 && \
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_convgemm_gpu.py tests/test_bn_gpu.py > $O/pytest2.log 2>&1 && \
PS_AMD_CONV_BIG_PRO=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_off.json 2> $O/bench_off.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_on.json 2> $O/bench_on.err && \
timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/bench256_on.json 2> $O/bench256_on.err
