#!/bin/bash
# Stride-2 data gradient: the four phase GEMMs in one grid (conv_dgrad_phases_kernel) vs four
# launches; weight gradients on the side stream for small layers (PS_AMD_WGRAD_STREAM_MAX_ROWS).
O=gpurun_out/r4ph
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_convgemm_gpu.py \
  tests/test_side_stream_gpu.py -k "stride2 or side_stream or chained or resnet" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python scripts/probe_resnet_convs.py > $O/convs_merged.log 2>&1 || exit $?
timeout -k 10 200 env PS_AMD_DGRAD_S2_MERGED=0 python scripts/probe_resnet_convs.py > $O/convs_legacy.log 2>&1 || exit $?
grep -E ",s2" $O/convs_merged.log; grep -E ",s2" $O/convs_legacy.log
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
  run legacy_$b $b PS_AMD_DGRAD_S2_MERGED=0
  run rows64k_$b $b PS_AMD_WGRAD_STREAM_MAX_ROWS=65536 PS_AMD_COMPUTE_PRIORITY=high
  run rows200k_$b $b PS_AMD_WGRAD_STREAM_MAX_ROWS=200704 PS_AMD_COMPUTE_PRIORITY=high
  run sideall_$b $b PS_AMD_WGRAD_STREAM=1 PS_AMD_COMPUTE_PRIORITY=high
  run base2_$b $b PS_AMD_NOOP=2
  run legacy2_$b $b PS_AMD_DGRAD_S2_MERGED=0
done
