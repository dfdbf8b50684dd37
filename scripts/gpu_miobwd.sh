#!/bin/bash
# A/B: MIOpen 3x3 data-grad without the asm igemm_bwd NHWC solver (it zero-fills dx first).
mkdir -p gpurun_out/miobwd
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
export MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0
timeout -k 10 600 python bench.py > gpurun_out/miobwd/bench1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/miobwd/bench2.log 2>&1 || exit $?
cp -r /tmp/ps_amd_miopen_$(id -u)_0 gpurun_out/miobwd/db
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/miobwd/prof -o run -- python3 bench.py --steps 10 --warmup 5 > gpurun_out/miobwd/bench_prof.log 2>&1 || exit $?
exit 0
