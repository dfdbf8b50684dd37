#!/bin/bash
# round 6: stem forward with LDS-staged whole-pixel-row stores -- numerics + in-step kernel time + bench
O=gpurun_out/${OUT:-r6ah4}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pool_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for b in 1024 256; do
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof$b -o run --output-format csv -- python $R/bench.py --steps 6 --warmup 3 --batch-per-gpu $b > $R/$O/prof$b.log 2>&1 || { tail -20 $R/$O/prof$b.log; exit 1; }
cd $R && grep -h "stem_conv_fwd\|stem_conv_wrw\|maxpool_nhwc_fwd\|pool_bn_bwd" $O/prof$b/run_kernel_stats.csv | cut -c1-200
done
for b in 1024 256 1024 256; do
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --batch-per-gpu $b 2> /dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($b, d['value'], d['ms_per_step'])"
done
