#!/bin/bash
# SQ / LDS / cache counters of the 256 x 256-tile kernel: a deep-K GEMM and a fold-epilogue GEMM
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
O=$R/gpurun_out/r5bigpmc
mkdir -p $O
cd /tmp
cpass() {
  local kind=$1 name=$2; shift 2
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $O/${kind}_$name -o run --output-format csv \
    -- python3 $R/scripts/probe_big_pmc.py $kind > $O/${kind}_$name.log 2>&1
}
for k in deep fold; do
  cpass $k p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA || exit $?
  cpass $k p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_VALU SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum || exit $?
  cpass $k p3 FETCH_SIZE TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum || exit $?
  cpass $k p4 WRITE_SIZE TA_BUSY_avr TA_TA_BUSY_sum || exit $?
  cd $R && python3 scripts/pmc_summary.py $O/${k}_p1 $O/${k}_p2 $O/${k}_p3 $O/${k}_p4 --match conv_big > $O/$k.txt 2>&1; cd /tmp
done
