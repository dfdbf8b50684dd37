#!/bin/bash
# First GPU session: kernel numerics tests, smoke, ResNet-50 probe. Stops on any crash/timeout.
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 900 python scripts/probe_resnet.py > gpurun_out/probe.log 2>&1 || exit $?
exit $rc
