#!/bin/bash
# Planar 3x3 64-channel kernel (PS_AMD_CONV_C64=2): numerics (conv3x3 patch test at 56 x 56 + the
# fused bottleneck), per-shape timing vs the tall im2col tile (mode 0), bench A/B.
O=gpurun_out/r5c64
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
PS_AMD_CONV_C64=2 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_convgemm_gpu.py::test_conv3x3_patch_forward_statistics_and_data_grad" \
  "tests/test_convgemm_gpu.py::test_fused_bottleneck_matches_module_path" -m gpu > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for m in 0 2; do PS_AMD_CONV_C64=$m timeout -k 10 200 python scripts/probe_conv3x3_c64.py >> $O/probe.jsonl 2>> $O/probe.err || exit $?; done
cat $O/probe.jsonl
PS_AMD_CONV_C64=2 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench2.json 2> $O/bench2.err || exit $?
grep -o '"value": [0-9.]*' $O/bench2.json
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench0.json 2> $O/bench0.err || exit $?
grep -o '"value": [0-9.]*' $O/bench0.json
