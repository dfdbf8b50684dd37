#!/bin/bash
# LDS-DMA forward GEMM: one barrier per K stage (PS_AMD_FWD_1BAR=1) vs two -- conv tests, 3x3 probe, bench A/B
mkdir -p gpurun_out/r3af
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
PS_AMD_FWD_1BAR=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convgemm_gpu.py \
  > gpurun_out/r3af/pytest.log 2>&1 || { tail -40 gpurun_out/r3af/pytest.log; exit 1; }
tail -2 gpurun_out/r3af/pytest.log
for f in 0 1; do
  PS_AMD_FWD_1BAR=$f timeout -k 10 300 python scripts/probe_conv3x3.py --miopen 0 > gpurun_out/r3af/conv3x3_1bar$f.jsonl 2>>gpurun_out/r3af/probe.err || exit $?
  python3 -c "
import json,sys
for l in open('gpurun_out/r3af/conv3x3_1bar$f.jsonl'):
    r=json.loads(l)
    if 'shape' in r: print('1bar=$f', r['shape'], 'fwd', r['ours_fwd_nopro_us'], 'dgrad', r.get('ours_dgrad_bnsums_us'))"
done
run() { env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 >> gpurun_out/r3af/bench_ab.jsonl 2>>gpurun_out/r3af/bench.err || exit $?;
        echo "$*: $(tail -1 gpurun_out/r3af/bench_ab.jsonl | cut -c100-190)"; }
run PS_AMD_FWD_1BAR=1
run PS_AMD_FWD_1BAR=0
run PS_AMD_FWD_1BAR=1
run PS_AMD_FWD_1BAR=0
