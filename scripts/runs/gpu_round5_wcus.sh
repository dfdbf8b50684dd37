#!/bin/bash
# side-stream CU mask for the weight gradients (PS_AMD_WGRAD_CUS) A/B, bs1024 and bs256
set -o pipefail
O=gpurun_out/r5wcus
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for c in 0 240 224 192; do
  PS_AMD_WGRAD_CUS=$c timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/b1024_$c.json 2> $O/b1024_$c.err || exit 1
  PS_AMD_WGRAD_CUS=$c timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > $O/b256_$c.json 2> $O/b256_$c.err || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/b1024_0b.json 2> $O/b1024_0b.err
