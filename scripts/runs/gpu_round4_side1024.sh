#!/bin/bash
# Side stream at bs1024: interleaved A/B, three pairs on one box (policy threshold check).
O=gpurun_out/r4s1k
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
  run base_$i PS_AMD_WGRAD_STREAM=0
  run side_$i PS_AMD_WGRAD_STREAM=1
done
