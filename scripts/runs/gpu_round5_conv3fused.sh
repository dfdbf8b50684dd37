#!/bin/bash
# Fused conv3 backward: numerics tests (new kernel + the fused bottleneck vs the module path),
# per-shape timing vs the chain, bench line; then the DLRM row-plane stage table.
O=gpurun_out/r5c3
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_conv_bwd_fused_gpu.py \
  "tests/test_convgemm_gpu.py::test_fused_bottleneck_matches_module_path" \
  "tests/test_convgemm_gpu.py::test_chained_blocks_fold_bn3_backward" -m gpu > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/probe_conv3_bwd.py > $O/probe.jsonl 2> $O/probe.err || exit $?
cat $O/probe.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench.json 2> $O/bench.err || exit $?
tail -c 400 $O/bench.json
PS_AMD_CONV3_BWD_FUSED=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench_off.json 2> $O/bench_off.err || exit $?
tail -c 400 $O/bench_off.json
bash scripts/runs/gpu_round5_dlrm_timing.sh
