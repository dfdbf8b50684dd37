#!/bin/bash
# round 6: CTR-async variance on ONE box: 3 bench runs + 3 step-splitter probes, interleaved
O=gpurun_out/r6o
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
nproc; cat /proc/loadavg
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --config ctr-async --steps 100 --warmup 10 > $O/bench_$i.json 2> $O/bench_$i.err || { tail -5 $O/bench_$i.err; exit 1; }
  python -c "import json;r=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]);print('bench', $i, r['value'], r['ms_per_step'], r['config'].get('sync_audit'))"
  timeout -k 10 200 python scripts/probe_ctr_async.py --steps 100 > $O/probe_$i.json 2> $O/probe_$i.err || { tail -5 $O/probe_$i.err; exit 1; }
  tail -1 $O/probe_$i.json
done
