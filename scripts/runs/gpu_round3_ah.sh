#!/bin/bash
# patch-staged 3x3 forward / data gradient: tests, 3x3 probe patch on/off, bench A/B
mkdir -p gpurun_out/r3ah
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convgemm_gpu.py \
  > gpurun_out/r3ah/pytest.log 2>&1 || { tail -40 gpurun_out/r3ah/pytest.log; exit 1; }
tail -2 gpurun_out/r3ah/pytest.log
for f in 0 1; do
  PS_AMD_CONV_PATCH=$f timeout -k 10 300 python scripts/probe_conv3x3.py --miopen 0 > gpurun_out/r3ah/conv3x3_patch$f.jsonl 2>>gpurun_out/r3ah/probe.err || exit $?
  python3 -c "
import json
for l in open('gpurun_out/r3ah/conv3x3_patch$f.jsonl'):
    r=json.loads(l)
    if 'shape' in r: print('patch=$f', r['shape'], 'fwd', r['ours_fwd_nopro_us'], 'dgrad', r.get('ours_dgrad_bnsums_us'))"
done
run() { env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 >> gpurun_out/r3ah/bench_ab.jsonl 2>>gpurun_out/r3ah/bench.err || exit $?;
        echo "$*: $(tail -1 gpurun_out/r3ah/bench_ab.jsonl | cut -c100-190)"; }
run PS_AMD_CONV_PATCH=1
run PS_AMD_CONV_PATCH=0
run PS_AMD_CONV_PATCH=1
run PS_AMD_CONV_PATCH=0
