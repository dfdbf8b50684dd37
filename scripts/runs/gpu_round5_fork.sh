#!/bin/bash
# BERT: residual gradients folded into the qkv / fc1 data-gradient GEMMs (PS_AMD_LINEAR_FORK) A/B + tests
set -o pipefail
O=gpurun_out/r5fork
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_splitk_gpu.py tests/test_transformer_gpu.py tests/test_zoo_gpu.py > $O/pytest.log 2>&1 && \
PS_AMD_LINEAR_FORK=0 timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > $O/bert_off.json 2> $O/bert_off.err && \
timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > $O/bert_on.json 2> $O/bert_on.err && \
PS_AMD_LINEAR_FORK=0 timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > $O/bert_off2.json 2> $O/bert_off2.err && \
timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > $O/bert_on2.json 2> $O/bert_on2.err
