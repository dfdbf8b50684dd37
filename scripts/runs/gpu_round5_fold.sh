#!/bin/bash
# conv1 data gradients on the 256 x 256 tiles (residual / fold epilogues + bn1 backward prologue):
# numerics, model-path tests, bench A/B (off = PS_AMD_CONV_BIG_FOLD=0, i.e. the 128-pixel tiles)
set -o pipefail
O=gpurun_out/r5fold
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_big_gpu.py > $O/pytest.log 2>&1 && \
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_convgemm_gpu.py tests/test_conv_bwd_fused_gpu.py tests/test_bn_gpu.py > $O/pytest2.log 2>&1 && \
PS_AMD_CONV_BIG_FOLD=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_off.json 2> $O/bench_off.err && \
PS_AMD_CONV1_BWD_PRO=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_nopro.json 2> $O/bench_nopro.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_on.json 2> $O/bench_on.err && \
timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/bench256_on.json 2> $O/bench256_on.err
