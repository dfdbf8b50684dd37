#!/bin/bash
# weight gradients on the side stream: GPU tests (side stream, convgemm, PS, plane) + bench A/B + kernel trace
mkdir -p gpurun_out/r3y
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_side_stream_gpu.py \
  tests/test_convgemm_gpu.py tests/test_ps_gpu.py tests/test_plane_gpu.py > gpurun_out/r3y/pytest.log 2>&1 || { tail -30 gpurun_out/r3y/pytest.log; exit 1; }
tail -2 gpurun_out/r3y/pytest.log
for f in 1 0 1; do
  PS_AMD_WGRAD_STREAM=$f timeout -k 10 300 python bench.py --steps 20 --warmup 8 >> gpurun_out/r3y/bench_ab.jsonl 2>>gpurun_out/r3y/bench.err || exit $?
  echo "wgrad_stream=$f: $(tail -1 gpurun_out/r3y/bench_ab.jsonl | cut -c1-200)"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3y/prof -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 4 > $GRAFT_REPO_ROOT/gpurun_out/r3y/prof.log 2>&1 || exit $?
echo done
