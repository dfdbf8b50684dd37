#!/bin/bash
# round 3 batch B: async PS v2 GPU tests (segments, 2-deep mailboxes, async rows) + BERT SSP(1)
# async vs pipelined at equal batch (256 and 1024) + CNN-MNIST parity on the GPU kernels.
mkdir -p gpurun_out/r3b
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest tests/test_async_ps_gpu.py tests/test_plane_gpu.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r3b/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r3b/pytest.log; tail -15 gpurun_out/r3b/pytest.log
[ $rc -eq 0 ] || exit $rc
for B in 256 1024; do
  for A in 1 0; do
    PS_AMD_BERT_ASYNC=$A timeout -k 10 300 python bench.py --config bert-ssp --batch-per-gpu $B --steps 20 --warmup 5 \
      > gpurun_out/r3b/bert_b${B}_async${A}.json 2> gpurun_out/r3b/bert_b${B}_async${A}.err || exit $?
  done
done
cat gpurun_out/r3b/bert_*.json
timeout -k 10 600 python -u scripts/mnist_parity.py --model cnn --device cuda > gpurun_out/r3b/cnn_parity_gpu.jsonl \
  2> gpurun_out/r3b/cnn_parity_gpu.err
rc=$?; cat gpurun_out/r3b/cnn_parity_gpu.jsonl; exit $rc
