#!/bin/bash
# rocprofv3 kernel trace of the default ResNet-50 bench step (bs1024) + per-family breakdown
# usage: scripts/gpu_prof_step.sh OUTDIR [extra bench.py args, e.g. --batch-per-gpu 256]
O=${1:-gpurun_out/pstep}
shift
EXTRA="$@"
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python $R/bench.py --steps 6 --warmup 3 $EXTRA > $R/$O/prof.log 2>&1 || exit $?
cd $R && python scripts/step_breakdown.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/breakdown.txt
cp $O/prof/*kernel_trace.csv.timeline.txt $O/timeline.txt; head -45 $O/breakdown.txt
