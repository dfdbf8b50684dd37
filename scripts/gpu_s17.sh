#!/bin/bash
mkdir -p gpurun_out/s17
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
timeout -k 10 600 python -m pytest tests/test_bn_gpu.py tests/test_pool_gpu.py -q > gpurun_out/s17/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/s17/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace -d $R/gpurun_out/s17/prof -o run --output-format csv -- python3 $R/scripts/probe_bn.py > $R/gpurun_out/s17/prof.log 2>&1 || exit $?
cd $R && python scripts/probe_bn.py --report gpurun_out/s17/prof/run_kernel_trace.csv > gpurun_out/s17/bn_bw.txt 2>&1
timeout -k 10 600 python bench.py --steps 30 --warmup 5 > gpurun_out/s17/bench.log 2>&1 || exit $?
exit 0
