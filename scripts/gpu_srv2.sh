#!/bin/bash
mkdir -p gpurun_out/srv gpurun_out/tests
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest tests/test_sparse_gpu.py tests/test_kernels_gpu.py tests/test_multirank_gpu.py tests/test_zoo_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests/pytest_srv2.log 2>&1 || { tail -30 gpurun_out/tests/pytest_srv2.log; exit 1; }
tail -2 gpurun_out/tests/pytest_srv2.log
timeout -k 10 300 python scripts/bench_server_kernels.py --iters 20 --json gpurun_out/srv/server_kernels.json > gpurun_out/srv/bench.log 2>&1 || { tail -20 gpurun_out/srv/bench.log; exit 1; }
grep kernel gpurun_out/srv/bench.log
