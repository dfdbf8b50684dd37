#!/bin/bash
# SQ / LDS counters of the flash-attention kernels (fwd, dQ, dK/dV) on the Llama shape (B4 S4096)
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
O=$R/gpurun_out/r5fapmc
mkdir -p $O
cd /tmp
cpass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $O/$name -o run --output-format csv \
    -- python3 $R/scripts/probe_flash.py 4 > $O/$name.log 2>&1
}
cpass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA || exit $?
cpass p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_VALU SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum || exit $?
cd $R && python3 scripts/pmc_summary.py $O/p1 $O/p2 --match fa_ > $O/fa.txt 2>&1; cat $O/fa.txt
