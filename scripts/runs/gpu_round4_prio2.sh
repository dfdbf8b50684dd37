#!/bin/bash
# bench.py with the single-process default of a high-priority compute stream: every config runs,
# ResNet-50 twice; the W = 2 rehearsal (peers: normal priority) still runs.
O=gpurun_out/r4prio2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for c in resnet50 resnet50 bert-ssp dlrm ctr-async llama-onebit; do
  timeout -k 10 400 python bench.py --config $c > $O/$c.json 2> $O/$c.err || { echo "$c failed rc=$?"; tail -5 $O/$c.err; exit 1; }
  grep '"metric"' $O/$c.json | cut -c1-170
done
PS_AMD_BENCH_ONE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 6 --warmup 3 --comm-probe 0 --timing 3 > $O/w2.json 2> $O/w2.err || { echo "w2 failed rc=$?"; tail -5 $O/w2.err; exit 1; }
grep '"metric"' $O/w2.json | cut -c1-170
