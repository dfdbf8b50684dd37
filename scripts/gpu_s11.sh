#!/bin/bash
# Large-offset BN stats test + rocprofv3 kernel stats of the bs512 ResNet-50 PS step.
mkdir -p gpurun_out/s11
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
timeout -k 10 300 python -m pytest tests/test_bn_gpu.py -q -k large_mean > gpurun_out/s11/pytest.log 2>&1
echo "rc=$?" >> gpurun_out/s11/pytest.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s11/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 > $R/gpurun_out/s11/prof.log 2>&1 || exit $?
exit 0
