#!/bin/bash
# Weight gradients on the side stream (PS_AMD_WGRAD_STREAM=1) at batch 256 and 1024 on one box:
# the small layer-3/4 grids of bs256 leave CUs idle that a second queue could fill.
O=gpurun_out/r4side
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
run() {  # name batch env...
  local name=$1 b=$2; shift 2
  timeout -k 10 200 env "$@" python bench.py --batch-per-gpu $b --steps 20 --warmup 8 > $O/$name.log 2>&1
  local rc=$?
  printf "%-28s " $name; grep '"metric"' $O/$name.log | python3 -c "import sys,json;d=json.loads(sys.stdin.readline());print(d['value'],d['ms_per_step'])" || tail -1 $O/$name.log
  [ $rc -ge 124 ] && exit $rc
  return 0
}
for b in 256 1024; do
  run base_$b $b PS_AMD_NOOP=1
  run side_$b $b PS_AMD_WGRAD_STREAM=1
  run side_hiprio_$b $b PS_AMD_WGRAD_STREAM=1 PS_AMD_COMPUTE_PRIORITY=high
  run base2_$b $b PS_AMD_NOOP=2
  run side2_$b $b PS_AMD_WGRAD_STREAM=1
done
