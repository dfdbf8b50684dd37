#!/bin/bash
# transformer tests + Llama bench after the RMSNorm materialize fix (2 runs)
set -o pipefail
O=gpurun_out/r5llama2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_transformer_gpu.py tests/test_ps_gpu.py > $O/pytest.log 2>&1 && \
timeout -k 10 500 python bench.py --config llama-onebit --steps 6 --warmup 3 > $O/llama1.json 2> $O/llama1.err && \
timeout -k 10 500 python bench.py --config llama-onebit --steps 6 --warmup 3 > $O/llama2.json 2> $O/llama2.err && \
timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > $O/bert.json 2> $O/bert.err
