#!/bin/bash
# 4-stage LDS-DMA ring, one block per CU, for deep-K 1x1 GEMMs (PS_AMD_CONV_DEEP): tests forced on, probe, bench A/B
mkdir -p gpurun_out/r3ap
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
PS_AMD_CONV_DEEP=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convgemm_gpu.py \
  > gpurun_out/r3ap/pytest.log 2>&1 || { tail -40 gpurun_out/r3ap/pytest.log; exit 1; }
tail -1 gpurun_out/r3ap/pytest.log
for f in 0 1; do
  PS_AMD_CONV_DEEP=$f timeout -k 10 300 python scripts/probe_conv_fwd.py > gpurun_out/r3ap/conv_fwd_deep$f.jsonl 2>>gpurun_out/r3ap/probe.err || exit $?
  python3 -c "
import json
for l in open('gpurun_out/r3ap/conv_fwd_deep$f.jsonl'):
    r=json.loads(l); print('deep=$f', r['shape'], r['us'], 'blas', r['blas_us'])"
done
run() { env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 >> gpurun_out/r3ap/bench_ab.jsonl 2>>gpurun_out/r3ap/bench.err || exit $?;
        echo "$*: $(tail -1 gpurun_out/r3ap/bench_ab.jsonl | cut -c100-190)"; }
run PS_AMD_CONV_DEEP=1
run PS_AMD_CONV_DEEP=0
run PS_AMD_CONV_DEEP=1
run PS_AMD_CONV_DEEP=0
