#!/bin/bash
# Knob sweep at batch 256 and 1024 on one box: which dispatch policies depend on the batch size.
O=gpurun_out/r4knobs
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
bash scripts/gpu_prof_step.sh $O/p256 --batch-per-gpu 256 > /dev/null 2>&1 || exit $?
for b in 256 1024; do
  run base_$b $b PS_AMD_NOOP=1
  run patch64_$b $b PS_AMD_CONV_PATCH64=1
  run notall_$b $b PS_AMD_CONV_TALL=0
  run persist2_$b $b PS_AMD_PERSIST_NK_PRO=2
  run twosrc_off_$b $b PS_AMD_TWOSRC_MAX_N=0
  run profuse512_$b $b PS_AMD_PRO_FUSE_MAX_K=512
  run base2_$b $b PS_AMD_NOOP=2
done
