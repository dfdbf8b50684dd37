#!/bin/bash
# sparse optimizer kernel with prefetched row ids / table rows: tests + DLRM bench (2 runs)
set -o pipefail
O=gpurun_out/r5sparseopt
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_sparse_gpu.py tests/test_row_plane_gpu.py tests/test_gpu_kvstore_gpu.py > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 > $O/dlrm1.json 2> $O/dlrm1.err && \
timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 > $O/dlrm2.json 2> $O/dlrm2.err
