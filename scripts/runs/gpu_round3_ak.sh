#!/bin/bash
# 8-wave 256 x 128 LDS-DMA tile for deep-K GEMMs (PS_AMD_CONV_BIG): tests with it forced on, probes, bench A/B
mkdir -p gpurun_out/r3ak
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
PS_AMD_CONV_BIG=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convgemm_gpu.py \
  > gpurun_out/r3ak/pytest.log 2>&1 || { tail -40 gpurun_out/r3ak/pytest.log; exit 1; }
tail -1 gpurun_out/r3ak/pytest.log
for f in 0 1; do
  PS_AMD_CONV_BIG=$f timeout -k 10 300 python scripts/probe_conv_fwd.py > gpurun_out/r3ak/conv_fwd_big$f.jsonl 2>>gpurun_out/r3ak/probe.err || exit $?
  PS_AMD_CONV_BIG=$f timeout -k 10 300 python scripts/probe_conv3x3.py --miopen 0 > gpurun_out/r3ak/conv3x3_big$f.jsonl 2>>gpurun_out/r3ak/probe.err || exit $?
  python3 -c "
import json
for l in open('gpurun_out/r3ak/conv_fwd_big$f.jsonl'):
    r=json.loads(l); print('big=$f', r['shape'], r['us'], 'blas', r['blas_us'])
for l in open('gpurun_out/r3ak/conv3x3_big$f.jsonl'):
    r=json.loads(l)
    if 'shape' in r: print('big=$f', r['shape'], 'fwd', r['ours_fwd_nopro_us'], 'dgrad', r.get('ours_dgrad_bnsums_us'))"
done
run() { env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 >> gpurun_out/r3ak/bench_ab.jsonl 2>>gpurun_out/r3ak/bench.err || exit $?;
        echo "$*: $(tail -1 gpurun_out/r3ak/bench_ab.jsonl | cut -c100-190)"; }
run PS_AMD_CONV_BIG=1
run PS_AMD_CONV_BIG=0
run PS_AMD_CONV_BIG=1
run PS_AMD_CONV_BIG=0
