#!/bin/bash
# round 6 final tree: the non-default bench configs at N=1
O=gpurun_out/r6cfgs
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for c in ctr-async bert-ssp llama-onebit; do
timeout -k 10 600 python bench.py --config $c > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
tail -1 $O/$c.json | cut -c1-260
done
