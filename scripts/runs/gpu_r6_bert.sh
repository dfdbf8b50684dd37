#!/bin/bash
# round 6: idle gaps in the BERT-base SSP and DLRM steps (kernel + HIP API trace, launch lag), and their benches
O=gpurun_out/r6bert
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
for c in bert-ssp dlrm; do
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace -d $R/$O/k_$c -o run --output-format csv -- python $R/bench.py --config $c --steps 8 --warmup 4 > $R/$O/k_$c.log 2>&1 || { tail -20 $R/$O/k_$c.log; exit 1; }
cd $R && python scripts/gpu_idle.py $O/k_$c/run_kernel_trace.csv 0.5 12 > $O/idle_$c.txt; cat $O/idle_$c.txt
timeout -k 10 300 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
tail -1 $O/bench_$c.json | cut -c1-200
done
