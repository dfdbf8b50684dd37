#!/bin/bash
# A/B of the BN reduction block cap (PS_AMD_BN_RED_MAXG): bench + kernel-trace summary per setting.
mkdir -p gpurun_out/redcap
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/redcap/pytest.log 2>&1 || exit $?
for g in 2048 4096 8192 16384; do
  timeout -k 10 300 env PS_AMD_BN_RED_MAXG=$g python bench.py > gpurun_out/redcap/bench_$g.log 2>&1 || exit $?
  timeout -k 10 300 env PS_AMD_BN_RED_MAXG=$g rocprofv3 --kernel-trace -d /tmp/redprof_$g -o run -- python3 bench.py --steps 8 --warmup 4 > gpurun_out/redcap/prof_$g.log 2>&1 || exit $?
  python scripts/db_summary.py /tmp/redprof_$g/run_results.db --top 80 > gpurun_out/redcap/summary_$g.txt || exit $?
done
exit 0
