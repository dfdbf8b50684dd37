#!/bin/bash
# round-5: whole-step HIP graph vs eager on the final tree (bs256 has ~2.9 ms of GPU idle per 20.8 ms step)
set -o pipefail
O=${O:-gpurun_out/r5graph}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for bs in 256 1024; do
  timeout -k 10 300 python bench.py --batch-per-gpu $bs --steps 30 --warmup 5 > $O/eager_$bs.json 2> $O/eager_$bs.err || exit $?
  timeout -k 10 300 python bench.py --batch-per-gpu $bs --steps 30 --warmup 5 --graph 1 > $O/graph_$bs.json 2> $O/graph_$bs.err || exit $?
done
cat $O/*.json
