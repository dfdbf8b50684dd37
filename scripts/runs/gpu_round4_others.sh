#!/bin/bash
# The non-headline bench configs on the final round-4 tree (1 GPU): BERT-base SSP(1), DLRM, Llama-3-8B, CTR async.
O=gpurun_out/r4oth
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for c in bert-ssp dlrm ctr-async llama-onebit; do
  timeout -k 10 400 python bench.py --config $c > $O/$c.json 2> $O/$c.err || { echo "$c failed rc=$?"; tail -5 $O/$c.err; exit 1; }
  grep '"metric"' $O/$c.json | cut -c1-220
done
