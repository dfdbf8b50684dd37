#!/bin/bash
# kernel stats of the BERT-SSP and DLRM bench steps (where the remaining time goes)
mkdir -p gpurun_out/r3r
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_flash_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3r/pytest.log 2>&1 || { tail -20 gpurun_out/r3r/pytest.log; exit 1; }
tail -2 gpurun_out/r3r/pytest.log
cd /tmp
for c in bert-ssp dlrm; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3r/$c -o run --output-format csv \
    -- python $R/bench.py --config $c --steps 5 --warmup 3 > $R/gpurun_out/r3r/$c.log 2>&1 || exit $?
  python $R/scripts/kernel_stats_top.py $(ls $R/gpurun_out/r3r/$c/*kernel_stats.csv | head -1) 25 > $R/gpurun_out/r3r/$c.top.txt || exit $?
  rm -f $R/gpurun_out/r3r/$c/*kernel_trace.csv
done
cat $R/gpurun_out/r3r/bert-ssp.top.txt $R/gpurun_out/r3r/dlrm.top.txt | cut -c1-170
