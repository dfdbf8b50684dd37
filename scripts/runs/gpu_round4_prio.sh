#!/bin/bash
# Compute-stream priority with the side stream at bs1024: interleaved A/B, three pairs on one box.
O=gpurun_out/r4prio
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
run() {  # name env...
  local name=$1; shift
  timeout -k 10 200 env "$@" python bench.py --steps 30 --warmup 8 > $O/$name.log 2>&1
  local rc=$?
  printf "%-12s " $name; grep '"metric"' $O/$name.log | python3 -c "import sys,json;d=json.loads(sys.stdin.readline());print(d['value'],d['ms_per_step'])" || tail -1 $O/$name.log
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for i in 1 2 3; do
  run normal_$i PS_AMD_COMPUTE_PRIORITY=normal
  run high_$i PS_AMD_COMPUTE_PRIORITY=high
done
