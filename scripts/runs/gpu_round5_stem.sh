#!/bin/bash
# fused stem backward (BN apply inside the weight gradient): numerics + bench A/B
set -o pipefail
O=gpurun_out/r5stem
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pool_gpu.py > $O/pytest.log 2>&1 && \
PS_AMD_STEM_BWD_FUSED=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_off.json 2> $O/bench_off.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_on.json 2> $O/bench_on.err && \
timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/bench256_on.json 2> $O/bench256_on.err
