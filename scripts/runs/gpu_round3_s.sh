#!/bin/bash
# split-K linear wgrad on the BERT shapes: timing vs hipBLASLt + PMC passes (MFMA busy, waits, LDS)
mkdir -p gpurun_out/r3s
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
timeout -k 10 200 python scripts/probe_linear_wgrad.py > gpurun_out/r3s/probe.jsonl 2>gpurun_out/r3s/probe.err || exit $?
cat gpurun_out/r3s/probe.jsonl
cd /tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $R/gpurun_out/r3s/$name -o run --output-format csv \
    -- python3 $R/scripts/probe_linear_wgrad.py --blas 0 --it 3 > $R/gpurun_out/r3s/$name.log 2>&1
}
pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA || exit $?
pass p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU SQ_INST_LEVEL_VMEM TCC_HIT_sum TCC_MISS_sum || exit $?
cd $R && python3 scripts/pmc_summary.py gpurun_out/r3s/p1 gpurun_out/r3s/p2 --match wgrad > gpurun_out/r3s/summary.txt
cat gpurun_out/r3s/summary.txt
