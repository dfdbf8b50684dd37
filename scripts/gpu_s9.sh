#!/bin/bash
mkdir -p gpurun_out/s9
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_bn_gpu.py -q -k "mfma or resnet_fused" > gpurun_out/s9/pytest.log 2>&1
echo "rc=$?" >> gpurun_out/s9/pytest.log
exit 0
