#!/bin/bash
# GPU session 4: fused BN kernels numerics + ResNet-50 A/B (fused vs MIOpen BN) + rocprof of fused.
mkdir -p gpurun_out/s4
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -m pytest tests/test_bn_gpu.py -q > gpurun_out/s4/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/s4/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --fused-bn 0 > gpurun_out/s4/bench_unfused.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --fused-bn 1 > gpurun_out/s4/bench_fused.log 2>&1 || exit $?
R=$PWD
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s4/prof -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 3 > $R/gpurun_out/s4/prof.log 2>&1 || exit $?
exit 0
