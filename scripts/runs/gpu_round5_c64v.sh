#!/bin/bash
# rolling-window 3x3 64-channel kernel (PS_AMD_CONV_C64=4): numerics, probe vs mode 0, bench A/B
set -o pipefail
O=gpurun_out/r5c64v
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
PS_AMD_CONV_C64=4 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_convgemm_gpu.py::test_conv3x3_patch_forward_statistics_and_data_grad" \
  "tests/test_convgemm_gpu.py::test_fused_bottleneck_matches_module_path" -m gpu > $O/pytest.log 2>&1 && \
PS_AMD_CONV_C64=4 timeout -k 10 200 python scripts/probe_conv3x3_c64.py > $O/probe.jsonl 2> $O/probe.err && \
PS_AMD_CONV_C64=0 timeout -k 10 200 python scripts/probe_conv3x3_c64.py >> $O/probe.jsonl 2>> $O/probe.err && \
PS_AMD_CONV_C64=4 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench4.json 2> $O/bench4.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench0.json 2> $O/bench0.err
