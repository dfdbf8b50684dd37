#!/bin/bash
# round 6: whole ResNet-50 at bs1024 on the production routes vs fp32
O=gpurun_out/r6g
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 850 --timeout-method thread tests/test_resnet_routes_gpu.py > $O/pytest.log 2>&1; rc=$?
grep -v "^$" $O/pytest.log | tail -30
exit $rc
