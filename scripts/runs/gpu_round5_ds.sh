#!/bin/bash
# layer-1 downsample fused backward: numerics + bench A/B; planar c64 kernel lookahead 1 vs 2
set -o pipefail
O=gpurun_out/r5ds
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_bwd_fused_gpu.py \
  tests/test_convgemm_gpu.py -k "fused or downsample or plain" > $O/pytest.log 2>&1 && \
PS_AMD_CONV_C64=2 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  "tests/test_convgemm_gpu.py::test_conv3x3_patch_forward_statistics_and_data_grad" >> $O/pytest.log 2>&1 && \
PS_AMD_CONV_C64=2 PS_AMD_C64_LOOKAHEAD=1 timeout -k 10 200 python scripts/probe_conv3x3_c64.py > $O/probe.jsonl 2>> $O/probe.err && \
PS_AMD_CONV_C64=2 timeout -k 10 200 python scripts/probe_conv3x3_c64.py >> $O/probe.jsonl 2>> $O/probe.err && \
PS_AMD_CONV_C64=0 timeout -k 10 200 python scripts/probe_conv3x3_c64.py >> $O/probe.jsonl 2>> $O/probe.err && \
PS_AMD_DS_BWD_FUSED=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_off.json 2> $O/bench_off.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_on.json 2> $O/bench_on.err && \
timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/bench256_on.json 2> $O/bench256_on.err
