#!/bin/bash
# BERT attention: staging loads batched, Q / O / dO / lse prefetched before the staging barrier
set -o pipefail
O=gpurun_out/r5attn3
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_transformer_gpu.py > $O/pytest.log 2>&1 && \
timeout -k 10 200 python scripts/probe_bert_attn.py > $O/attn.jsonl 2> $O/attn.err && \
timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > $O/bert1.json 2> $O/bert1.err && \
timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > $O/bert2.json 2> $O/bert2.err
