#!/bin/bash
# round 6, final tree: kernel-trace step breakdown + per-dispatch timeline + idle gaps at bs1024 and bs256
O=gpurun_out/${OUT:-r6ag2}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
for b in ${BATCHES:-1024 256}; do
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace -d $R/$O/prof$b -o run --output-format csv -- python $R/bench.py --steps 6 --warmup 3 --batch-per-gpu $b > $R/$O/prof$b.log 2>&1 || { tail -20 $R/$O/prof$b.log; exit 1; }
cd $R && python scripts/step_breakdown.py $O/prof$b/run_kernel_trace.csv > $O/breakdown_$b.txt && tail -6 $O/breakdown_$b.txt
python scripts/gpu_idle.py $O/prof$b/run_kernel_trace.csv 0.3 8 > $O/idle_$b.txt && cat $O/idle_$b.txt | cut -c1-150
done
for b in ${BATCHES:-1024 256}; do
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --batch-per-gpu $b > $O/bench_$b.json 2> $O/bench_$b.err && tail -1 $O/bench_$b.json
done
