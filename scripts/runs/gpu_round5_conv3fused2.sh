#!/bin/bash
# Fused conv3 backward, 5-slot DMA ring + z3 two stages ahead: tests, per-shape timing, bench line.
O=gpurun_out/r5c3b
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_conv_bwd_fused_gpu.py \
  "tests/test_convgemm_gpu.py::test_chained_blocks_fold_bn3_backward" -m gpu > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/probe_conv3_bwd.py > $O/probe.jsonl 2> $O/probe.err || exit $?
cat $O/probe.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench.json 2> $O/bench.err || exit $?
grep -o '"value": [0-9.]*' $O/bench.json
