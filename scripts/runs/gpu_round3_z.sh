#!/bin/bash
# bn3 backward in the conv3 data-gradient prologue: kernel + fused-block tests, bench A/B, kernel trace
mkdir -p gpurun_out/r3z
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convgemm_gpu.py \
  tests/test_side_stream_gpu.py tests/test_bn_gpu.py > gpurun_out/r3z/pytest.log 2>&1 || { tail -40 gpurun_out/r3z/pytest.log; exit 1; }
tail -2 gpurun_out/r3z/pytest.log
for f in 1 0 1 0; do
  PS_AMD_BN_BWD_PROLOGUE=$f timeout -k 10 300 python bench.py --steps 20 --warmup 8 >> gpurun_out/r3z/bench_ab.jsonl 2>>gpurun_out/r3z/bench.err || exit $?
  echo "bn_bwd_prologue=$f: $(tail -1 gpurun_out/r3z/bench_ab.jsonl | cut -c1-200)"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3z/prof -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 4 > $GRAFT_REPO_ROOT/gpurun_out/r3z/prof.log 2>&1 || exit $?
echo done
