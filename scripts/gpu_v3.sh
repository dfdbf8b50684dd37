#!/bin/bash
# Implicit-GEMM conv kernels + fused bottleneck: numerics, model equivalence, A/B bench, rocprof.
R=$PWD
mkdir -p gpurun_out/v3
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest tests/test_convgemm_gpu.py tests/test_bn_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/v3/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/v3/pytest.log
[ $rc -eq 0 ] || exit $rc
PS_AMD_FUSED_BLOCK=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/v3/bench_unfused.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/v3/bench_fused.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/v3/prof -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 4 > $R/gpurun_out/v3/prof.log 2>&1 || exit $?
exit 0
