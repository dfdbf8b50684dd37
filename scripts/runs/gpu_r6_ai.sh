#!/bin/bash
# round 6: branch-free bit masks in the data-gradient epilogues (convgemm / conv_big) -- numerics, kernel times, bench
O=gpurun_out/${OUT:-r6ai2}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convgemm_gpu.py tests/test_conv_big_gpu.py tests/test_conv_bwd_fused_gpu.py tests/test_resnet_routes_gpu.py tests/test_pool_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for b in 1024; do
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof$b -o run --output-format csv -- python $R/bench.py --steps 6 --warmup 3 --batch-per-gpu $b > $R/$O/prof$b.log 2>&1 || { tail -20 $R/$O/prof$b.log; exit 1; }
cd $R && python scripts/step_breakdown.py $O/prof$b/run_kernel_trace.csv > $O/breakdown_$b.txt && head -30 $O/breakdown_$b.txt | cut -c1-110
done
for b in 1024 256 1024 256; do
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --batch-per-gpu $b 2> /dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($b, d['value'], d['ms_per_step'])"
done
