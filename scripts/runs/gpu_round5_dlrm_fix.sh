#!/bin/bash
# Row plane after the accumulate / apply fixes: numerics tests, then DLRM W=1 and W=2 with the stage table.
O=gpurun_out/r5dlrm2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_row_plane_gpu.py \
  tests/test_sparse_gpu.py -m gpu > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 > $O/dlrm_w1.json 2> $O/dlrm_w1.err || exit $?
grep -o '"value": [0-9.]*, "unit": "samples/s", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*' $O/dlrm_w1.json
export PS_AMD_BENCH_ONE_GPU=1 PS_AMD_ROWPLANE_TIMING=1
timeout -k 10 300 python bench.py --config dlrm --gpus 2 --steps 10 --warmup 3 --comm-probe 0 --timing 3 > $O/dlrm_w2_timing.json 2> $O/dlrm_w2_timing.err || exit $?
python3 -c "import json;d=json.loads(open('$O/dlrm_w2_timing.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step']);print(json.dumps(d['config'].get('row_plane_stages')));print(json.dumps(d['config'].get('ps_phase_ms_per_step')))"
unset PS_AMD_ROWPLANE_TIMING
timeout -k 10 300 python bench.py --config dlrm --gpus 2 --steps 10 --warmup 3 --comm-probe 0 > $O/dlrm_w2.json 2> $O/dlrm_w2.err || exit $?
grep -o '"value": [0-9.]*' $O/dlrm_w2.json
