#!/bin/bash
# async PS: GPU tests, then BERT-SSP(1) bench async (mailboxes + native server) vs pipelined collective rounds
mkdir -p gpurun_out/async
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest tests/test_async_ps_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/async/pytest.log 2>&1 || { tail -30 gpurun_out/async/pytest.log; exit 1; }
tail -3 gpurun_out/async/pytest.log
PS_AMD_BERT_ASYNC=1 timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 --json-out gpurun_out/async/bert_async.json > gpurun_out/async/bert_async.log 2>&1 || exit $?
PS_AMD_BERT_ASYNC=0 timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 --json-out gpurun_out/async/bert_pipe.json > gpurun_out/async/bert_pipe.log 2>&1 || exit $?
cat gpurun_out/async/*.json
