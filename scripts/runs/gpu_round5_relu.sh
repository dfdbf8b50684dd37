#!/bin/bash
# DLRM MLPs with bias + ReLU in the GEMM epilogue (PS_AMD_FUSED_RELU) A/B + tests
set -o pipefail
O=gpurun_out/r5relu
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_splitk_gpu.py > $O/pytest.log 2>&1 && \
PS_AMD_FUSED_RELU=0 timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 > $O/dlrm_off.json 2> $O/dlrm_off.err && \
timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 > $O/dlrm_on.json 2> $O/dlrm_on.err && \
PS_AMD_FUSED_RELU=0 timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 > $O/dlrm_off2.json 2> $O/dlrm_off2.err && \
timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 > $O/dlrm_on2.json 2> $O/dlrm_on2.err
