#!/bin/bash
mkdir -p gpurun_out/tests gpurun_out/cfg
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest tests/test_sparse_gpu.py tests/test_kernels_gpu.py tests/test_multirank_gpu.py tests/test_zoo_gpu.py tests/test_serialize_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests/pytest_sparse2.log 2>&1 || { tail -30 gpurun_out/tests/pytest_sparse2.log; exit 1; }
tail -2 gpurun_out/tests/pytest_sparse2.log
timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 --json-out gpurun_out/cfg/dlrm.json > gpurun_out/cfg/dlrm.log 2>&1 || exit $?
cut -c1-330 gpurun_out/cfg/dlrm.json
