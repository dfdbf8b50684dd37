#!/bin/bash
# DLRM (1 GPU, batch 65536) kernel stats: where the 5.3 ms step goes
set -o pipefail
O=${O:-gpurun_out/r5dlrmprof}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python $R/bench.py --config dlrm --steps 20 --warmup 5 > $R/$O/prof.log 2>&1
