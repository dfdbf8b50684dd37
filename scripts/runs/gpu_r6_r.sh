#!/bin/bash
# round 6: BN finalize chain standalone (event time per call + rocprofv3 per-kernel durations)
O=gpurun_out/r6r
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
cd /tmp && cd - > /dev/null
timeout -k 10 200 python scripts/probe_bn_finalize.py > $O/fin_events.jsonl 2> $O/fin_events.err || { tail -5 $O/fin_events.err; exit 1; }
cat $O/fin_events.jsonl
IT=50 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o fin -- python3 scripts/probe_bn_finalize.py > $O/fin_prof.log 2>&1 || { tail -20 $O/fin_prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
