#!/bin/bash
# PMC passes over the conv-GEMM probe (--quick: deep-K LDS-DMA shape + BN-prologue shape, and
# hipBLASLt on the same GEMMs): one counter group per rocprofv3 run, kernel-trace only.
mkdir -p gpurun_out/pmc1
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $R/gpurun_out/pmc1/$name -o run --output-format csv \
    -- python3 $R/scripts/probe_convgemm.py --quick > $R/gpurun_out/pmc1/$name.log 2>&1
}
pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA || exit $?
pass p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU SQ_INST_LEVEL_VMEM TCC_HIT_sum TCC_MISS_sum || exit $?
pass p3 FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum || exit $?
exit 0
