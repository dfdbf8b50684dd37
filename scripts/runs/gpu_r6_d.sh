#!/bin/bash
# round 6: where the unbounded run-ahead stall blocks (per-thread kernel wait channel + syscall sampling)
O=gpurun_out/r6d
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for i in 1 2 3 4; do
  PS_AMD_MAX_INFLIGHT=0 timeout -k 10 240 python scripts/probe_stall_alloc.py --steps 30 > $O/stall_$i.jsonl 2> $O/stall_$i.err || exit $?
  grep -c stall $O/stall_$i.jsonl; tail -1 $O/stall_$i.jsonl | cut -c1-80
done
grep -h "stall\]" $O/stall_*.jsonl | head -60
