#!/bin/bash
# the warmup-5 stall: with the host run-ahead bound (PS_AMD_MAX_INFLIGHT=2) vs unbounded, three runs each
set -o pipefail
O=gpurun_out/r5w5b
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for i in 1 2 3; do
  PS_AMD_MAX_INFLIGHT=2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/if2_$i.json 2> $O/if2_$i.err || exit $?
  PS_AMD_MAX_INFLIGHT=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/if0_$i.json 2> $O/if0_$i.err || exit $?
done
PS_AMD_MAX_INFLIGHT=2 timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 5 > $O/if2_256.json 2> $O/if2_256.err
