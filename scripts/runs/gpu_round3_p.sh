#!/bin/bash
# PMC passes over the flash-attention probe (our fwd / dQ / dKdV vs aotriton's on the same shape):
# one counter group per rocprofv3 run, kernel-trace only
mkdir -p gpurun_out/r3p
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $R/gpurun_out/r3p/$name -o run --output-format csv \
    -- python3 $R/scripts/probe_flash.py 1 > $R/gpurun_out/r3p/$name.log 2>&1
}
pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA || exit $?
pass p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU SQ_INST_LEVEL_VMEM TCC_HIT_sum TCC_MISS_sum || exit $?
cd $R && python3 scripts/pmc_summary.py gpurun_out/r3p/p1 gpurun_out/r3p/p2 --match fa_ attn_fwd bwd_kernel > gpurun_out/r3p/summary.txt
cat gpurun_out/r3p/summary.txt | head -80
