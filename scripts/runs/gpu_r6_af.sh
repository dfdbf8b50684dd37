#!/bin/bash
# round 6: host launch vs GPU start at bs1024 and bs256 with the inline serve (kernel + HIP API trace)
O=gpurun_out/${OUT:-r6af}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
for b in ${BATCHES:-1024 256}; do
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --hip-runtime-trace -d $R/$O/prof$b -o run --output-format csv -- python $R/bench.py --steps 6 --warmup 3 --batch-per-gpu $b > $R/$O/prof$b.log 2>&1 || { tail -20 $R/$O/prof$b.log; exit 1; }
cd $R && python scripts/launch_lag.py $O/prof$b/run_kernel_trace.csv $O/prof$b/run_hip_api_trace.csv 20 > $O/launch_lag_$b.txt && cat $O/launch_lag_$b.txt | cut -c1-160
python scripts/step_breakdown.py $O/prof$b/run_kernel_trace.csv > $O/breakdown_$b.txt && tail -5 $O/breakdown_$b.txt
done
