#!/bin/bash
# round 6: vectorized 1-bit pack (tests + isolated rate), then the full-depth Llama 1-bit vs none, 40 steps
O=gpurun_out/r6n
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k onebit tests/test_plane_gpu.py -k "onebit or llama" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python scripts/probe_onebit_pack.py > $O/pack.txt 2>&1 || { cat $O/pack.txt; exit 1; }
cat $O/pack.txt
SKIP_TESTS=1 LLAMA_MODES="onebit:bf16 none:fp32" LLAMA_STEPS=40 bash scripts/runs/gpu_r6_i.sh
