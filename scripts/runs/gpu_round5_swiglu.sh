#!/bin/bash
# round-5: SwiGLU with the fast sigmoid + 32-bit indexing -- numerics tests, kernel alone, Llama bench
set -o pipefail
O=${O:-gpurun_out/r5swiglu}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/probe_swiglu.py > $O/probe.json 2> $O/probe.err && cat $O/probe.json && \
timeout -k 10 500 python bench.py --config llama-onebit --steps 6 --warmup 3 > $O/llama.json 2> $O/llama.err && tail -1 $O/llama.json
