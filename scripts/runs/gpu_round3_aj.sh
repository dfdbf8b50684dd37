#!/bin/bash
# 128 x 64 tiles where they cut the last-round tail of one-tile-per-block LDS-DMA grids (PS_AMD_CONV_QUANT64)
mkdir -p gpurun_out/r3aj
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for f in 0 1; do
  PS_AMD_CONV_QUANT64=$f timeout -k 10 300 python scripts/probe_conv_fwd.py > gpurun_out/r3aj/conv_fwd_q$f.jsonl 2>>gpurun_out/r3aj/probe.err || exit $?
  python3 -c "
import json
for l in open('gpurun_out/r3aj/conv_fwd_q$f.jsonl'):
    r=json.loads(l); print('q64=$f', r['shape'], r['us'], 'blas', r['blas_us'])"
done
PS_AMD_CONV_QUANT64=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convgemm_gpu.py \
  > gpurun_out/r3aj/pytest.log 2>&1 || { tail -40 gpurun_out/r3aj/pytest.log; exit 1; }
tail -1 gpurun_out/r3aj/pytest.log
run() { env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 >> gpurun_out/r3aj/bench_ab.jsonl 2>>gpurun_out/r3aj/bench.err || exit $?;
        echo "$*: $(tail -1 gpurun_out/r3aj/bench_ab.jsonl | cut -c100-190)"; }
run PS_AMD_CONV_QUANT64=1
run PS_AMD_CONV_QUANT64=0
run PS_AMD_CONV_QUANT64=1
run PS_AMD_CONV_QUANT64=0
