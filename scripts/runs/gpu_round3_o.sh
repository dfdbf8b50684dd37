#!/bin/bash
# per-kernel times of the stem backward: fused (pool gathered in the BN passes) vs two-step
mkdir -p gpurun_out/r3o
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_pool_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3o/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r3o/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
for f in 1 0; do
  PS_AMD_STEM_POOL_FUSED=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3o/p$f -o run --output-format csv \
    -- python $R/bench.py --steps 4 --warmup 3 > $R/gpurun_out/r3o/b$f.log 2>&1 || exit $?
  rm -f $R/gpurun_out/r3o/p$f/*kernel_trace.csv
done
cd $R && python3 - <<'PY'
import csv
for f in ('gpurun_out/r3o/p1/run_kernel_stats.csv','gpurun_out/r3o/p0/run_kernel_stats.csv'):
    print(f)
    for r in csv.DictReader(open(f)):
        n=r['Name']
        if any(k in n for k in ('bn_bwd_reduce_kernel<2','bn_bwd_apply_kernel<2','maxpool_nhwc_bwd','stem_conv_wrw')):
            print(f"  {int(r['Calls']):4d} calls avg {float(r['AverageNs'])/1e3:8.1f} us  {n[:90]}")
PY
