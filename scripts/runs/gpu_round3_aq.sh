#!/bin/bash
# bench lines of the other BASELINE configs on the final round-3 tree
mkdir -p gpurun_out/r3aq
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for c in bert-ssp dlrm llama-onebit; do
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 4 > gpurun_out/r3aq/$c.json 2> gpurun_out/r3aq/$c.err || exit $?
  cut -c1-220 gpurun_out/r3aq/$c.json
done
