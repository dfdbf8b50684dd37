#!/bin/bash
# forward 1x1 GEMM cost split (statistics epilogue / BN prologue) + a kernel trace of the current ResNet-50 step
mkdir -p gpurun_out/r3ad
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python scripts/probe_conv_fwd.py --variants 1 > gpurun_out/r3ad/conv_fwd_variants.jsonl 2>gpurun_out/r3ad/probe.err || exit $?
cut -c1-260 gpurun_out/r3ad/conv_fwd_variants.jsonl
R=$PWD; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r3ad/prof -o run -- \
  python3 $R/bench.py --steps 3 --warmup 5 > $R/gpurun_out/r3ad/prof.log 2>&1 || exit $?
cd $R && f=$(find gpurun_out/r3ad/prof -name '*kernel_trace.csv' | head -1) && python3 scripts/step_breakdown.py $f > gpurun_out/r3ad/step_breakdown.txt && \
  python3 scripts/trace_summary.py $f > gpurun_out/r3ad/trace_summary.txt 2>&1; head -40 gpurun_out/r3ad/step_breakdown.txt
grep -i -c "igemm\|miopen\|SubTensor" $f || true
