#!/bin/bash
# Batch 2: layer-2 fused conv3 backward (tests + probe + bench), late-created KV keys on the GPU,
# row-plane accumulate / apply fixes (tests + DLRM W=1 / W=2 stage table).
O=gpurun_out/r5b2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_conv_bwd_fused_gpu.py \
  "tests/test_convgemm_gpu.py::test_fused_bottleneck_matches_module_path" \
  "tests/test_convgemm_gpu.py::test_chained_blocks_fold_bn3_backward" -m gpu > $O/pytest_conv.log 2>&1; rc=$?
tail -4 $O/pytest_conv.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/probe_conv3_bwd.py > $O/probe.jsonl 2> $O/probe.err || exit $?
cat $O/probe.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench.json 2> $O/bench.err || exit $?
grep -o '"value": [0-9.]*' $O/bench.json
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_row_plane_gpu.py \
  tests/test_gpu_kvstore_gpu.py -m gpu > $O/pytest_ps.log 2>&1; rc=$?
tail -4 $O/pytest_ps.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 > $O/dlrm_w1.json 2> $O/dlrm_w1.err || exit $?
grep -o '"value": [0-9.]*' $O/dlrm_w1.json
export PS_AMD_BENCH_ONE_GPU=1 PS_AMD_ROWPLANE_TIMING=1
timeout -k 10 300 python bench.py --config dlrm --gpus 2 --steps 10 --warmup 3 --comm-probe 0 --timing 3 > $O/dlrm_w2_timing.json 2> $O/dlrm_w2_timing.err || exit $?
python3 -c "import json;d=json.loads(open('$O/dlrm_w2_timing.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step']);print(json.dumps(d['config'].get('row_plane_stages')));print(json.dumps(d['config'].get('ps_phase_ms_per_step')))"
