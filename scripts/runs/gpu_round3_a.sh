#!/bin/bash
# round 3 batch A: new GPU tests (plane W=8, tiny-Llama 1-bit, conv on K1/K2, async exact sum)
# + CNN-MNIST parity on the GPU kernels.
mkdir -p gpurun_out/r3a
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 900 python -u -m pytest tests/test_plane_gpu.py tests/test_fc_gpu.py tests/test_async_ps_gpu.py \
  -m gpu -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r3a/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r3a/pytest.log; tail -25 gpurun_out/r3a/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/mnist_parity.py --model cnn --device cuda > gpurun_out/r3a/cnn_parity_gpu.jsonl 2> gpurun_out/r3a/cnn_parity_gpu.err
rc=$?; cat gpurun_out/r3a/cnn_parity_gpu.jsonl; exit $rc
