#!/bin/bash
set -o pipefail
O=gpurun_out/r5ctr
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_async_ps_gpu.py > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --config ctr-async --steps 20 --warmup 5 > $O/ctr1.json 2> $O/ctr1.err && \
timeout -k 10 300 python bench.py --config ctr-async --steps 20 --warmup 5 > $O/ctr2.json 2> $O/ctr2.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/resnet.json 2> $O/resnet.err
