#!/bin/bash
# Fold epilogues (6-9) on one-tile-per-block LDS-DMA grids (PS_AMD_FOLD_GLDS=1) vs the persistent
# register-staged grid (whose epilogue-9 variant spills): numerics under the knob, then bench A/B.
O=gpurun_out/r4fg
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
PS_AMD_FOLD_GLDS=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pool_gpu.py tests/test_convgemm_gpu.py \
  -k "chained or fused_bottleneck or resnet or stem" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # name batch env...
  local name=$1 b=$2; shift 2
  timeout -k 10 200 env "$@" python bench.py --batch-per-gpu $b --steps 20 --warmup 8 > $O/$name.log 2>&1
  local rc=$?
  printf "%-28s " $name; grep '"metric"' $O/$name.log | python3 -c "import sys,json;d=json.loads(sys.stdin.readline());print(d['value'],d['ms_per_step'])" || tail -1 $O/$name.log
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for b in 1024 256; do
  run base_$b $b PS_AMD_FOLD_GLDS=0
  run fg_$b $b PS_AMD_FOLD_GLDS=1
  run base2_$b $b PS_AMD_FOLD_GLDS=0
  run fg2_$b $b PS_AMD_FOLD_GLDS=1
done
PS_AMD_FOLD_GLDS=1 bash scripts/gpu_prof_step.sh $O/p1024 > /dev/null 2>&1 || exit $?
grep -E "<128, 128, 0, (6|7|8|9),|stem" $O/p1024/timeline.txt | head -24
