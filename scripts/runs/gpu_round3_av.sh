#!/bin/bash
# Stem max-pool backward on 2x2 dx quads (4 window reads per 4 dx pixels instead of 16):
# pool / kernel / conv tests, then bench A/B against the previous build (ab_old/) on one box.
O=gpurun_out/r3av
mkdir -p $O
R=$PWD
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pool_gpu.py tests/test_kernels_gpu.py tests/test_convgemm_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
rm -rf /tmp/abold && mkdir -p /tmp/abold && cp -r ps_amd bench.py miopen_db /tmp/abold/ && cp ab_old/_C*.so /tmp/abold/ps_amd/
for i in 1 2; do
  (cd /tmp/abold && PYTHONPATH=/tmp/abold timeout -k 10 300 python bench.py --steps 20 --warmup 5) > $O/old_$i.json 2>$O/old_$i.err || exit 1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/new_$i.json 2>$O/new_$i.err || exit 1
  tail -1 $O/old_$i.json; tail -1 $O/new_$i.json
done
