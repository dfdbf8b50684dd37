#!/bin/bash
# round 6 first call: BERT baseline + kernel stats (before the GELU epilogues), stall root-cause probe
O=gpurun_out/r6a
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > $O/bert_before.json 2> $O/bert_before.err || exit $?
tail -1 $O/bert_before.json
for i in 1 2 3; do
  PS_AMD_MAX_INFLIGHT=0 timeout -k 10 240 python scripts/probe_stall_alloc.py --steps 40 > $O/stall_if0_$i.jsonl 2> $O/stall_if0_$i.err || exit $?
  tail -1 $O/stall_if0_$i.jsonl
done
PS_AMD_MAX_INFLIGHT=2 timeout -k 10 240 python scripts/probe_stall_alloc.py --steps 40 > $O/stall_if2.jsonl 2> $O/stall_if2.err || exit $?
tail -1 $O/stall_if2.jsonl
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python $R/bench.py --config bert-ssp --steps 4 --warmup 2 > $R/$O/prof.log 2>&1 || exit $?
cd $R && python scripts/kernel_stats_top.py $O/prof/run_kernel_stats.csv 45 > $O/bert_top.txt 2>&1; head -30 $O/bert_top.txt
