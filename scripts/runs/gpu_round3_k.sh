#!/bin/bash
# sparse: sync-free W=1 path + row-kernel roofline; DLRM bench; Llama exposed_comm_ms at world 1
mkdir -p gpurun_out/r3k
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_sparse_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3k/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3k/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_server_kernels.py --big 0 --json gpurun_out/r3k/server_kernels.json > gpurun_out/r3k/server_kernels.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 > gpurun_out/r3k/dlrm.json 2>gpurun_out/r3k/dlrm.err || exit $?
timeout -k 10 400 python bench.py --config llama-onebit --steps 6 --warmup 3 --timing 3 > gpurun_out/r3k/llama_timing.json 2>gpurun_out/r3k/llama_timing.err || exit $?
grep -E "lazy_init|sorted_runs|gather_rows|segment" gpurun_out/r3k/server_kernels.log | cut -c1-200
cut -c1-400 gpurun_out/r3k/dlrm.json; grep bench-timing gpurun_out/r3k/llama_timing.err
