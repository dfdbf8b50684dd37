#!/bin/bash
mkdir -p gpurun_out/s24
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 900 python -m pytest tests/test_serialize_gpu.py -q > gpurun_out/s24/pytest.log 2>&1
echo "rc=$?" >> gpurun_out/s24/pytest.log
exit 0
