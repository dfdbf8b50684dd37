#!/bin/bash
# round 6: the unbounded run-ahead stall seen from outside the process (every thread, no GIL)
O=gpurun_out/r6e
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
python -c "import torch; f,t=torch.cuda.mem_get_info(); print('mem_get_info free/total GB', f/2**30, t/2**30)"
for i in 1 2 3; do
  PROBE_PROC_OUT=$O/proc_$i.jsonl PS_AMD_MAX_INFLIGHT=0 timeout -k 10 240 python scripts/probe_stall_alloc.py --steps 12 > $O/stall_$i.jsonl 2> $O/stall_$i.err || exit $?
  python scripts/stall_threads.py $O/stall_$i.jsonl $O/proc_$i.jsonl | head -40
done
rm -f $O/proc_*.jsonl.gz; gzip $O/proc_*.jsonl
