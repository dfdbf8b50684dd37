#!/bin/bash
# Llama weight gradients straight into the PS gradient bucket (ops/linear.py PsLinear): test + bench A/B
set -o pipefail
O=gpurun_out/r5pslinear
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ps_gpu.py tests/test_plane_gpu.py > $O/pytest.log 2>&1 && \
PS_AMD_PS_LINEAR=0 timeout -k 10 500 python bench.py --config llama-onebit --steps 6 --warmup 3 > $O/llama_off.json 2> $O/llama_off.err && \
timeout -k 10 500 python bench.py --config llama-onebit --steps 6 --warmup 3 > $O/llama_on.json 2> $O/llama_on.err && \
PS_AMD_PS_LINEAR=0 timeout -k 10 500 python bench.py --config llama-onebit --steps 6 --warmup 3 > $O/llama_off2.json 2> $O/llama_off2.err && \
timeout -k 10 500 python bench.py --config llama-onebit --steps 6 --warmup 3 > $O/llama_on2.json 2> $O/llama_on2.err
